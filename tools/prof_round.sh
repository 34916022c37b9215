#!/bin/bash
# End-of-round profiles: tools/profile.sh (kernel trace + FETCH_SIZE / WRITE_SIZE passes of the
# bench's timed step), then a kernel trace of the batched / next_rows lines. Results under $1.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${1:-gpurun_out/prof_end}
bash tools/profile.sh "$OUT" || exit $?
echo "== batched trace"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/batched" -o run -- python3 bench.py --steps 5 --warmup 2 --no-headline --no-chain --no-host-path --no-cpu-baseline > "$OUT/batched.log" 2>&1
rc=$?; echo "rc=$rc"; tail -n 2 "$OUT/batched.log"; exit $rc
