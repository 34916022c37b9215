#!/bin/bash
# rocprofv3 kernel-trace stats + separate PMC passes of the bench (per the MI355X guide:
# counters in their own runs, never combined with sys/runtime traces).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${1:-gpurun_out/prof}
shift || true
ARGS=${BENCH_ARGS:---steps 10 --warmup 3 --no-cpu-baseline}
mkdir -p "$OUT"
run() {  # run <name> <secs> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?; echo "rc=$rc"; tail -n 5 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then echo "stop"; exit $rc; fi
}
run trace 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 bench.py $ARGS
run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- python3 bench.py $ARGS
run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- python3 bench.py $ARGS
run pmc_sq 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmc_sq" -o run -- python3 bench.py $ARGS
find "$OUT" -name "*.csv" | head -50
