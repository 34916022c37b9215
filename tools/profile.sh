#!/bin/bash
# rocprofv3 kernel-trace stats + separate PMC passes (FETCH_SIZE, WRITE_SIZE) of the bench's
# timed step, per MI355X_MICROARCH.md: counters in their own runs, never combined with
# sys/runtime traces. Summarise afterwards with tools/prof_summary.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${1:-gpurun_out/prof}
ARGS=${BENCH_ARGS:---steps 20 --warmup 5 --no-headline --no-chain --no-batched --no-host-path --no-cpu-baseline}
mkdir -p "$OUT"
run() {  # run <name> <secs> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?; echo "rc=$rc"; tail -n 2 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then echo "stop"; exit $rc; fi
}
run trace 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 bench.py $ARGS
run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- python3 bench.py $ARGS
run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- python3 bench.py $ARGS
find "$OUT" -name "*.csv" | sort
