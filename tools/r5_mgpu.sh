#!/bin/bash
# Round 5 rehearsal of the N > 1 bench path on the one-GPU box (never a measurement): bench.py --gpus 2
# and 4 starting their own ranks (LK_BENCH_BACKEND=gloo: ranks share the GPU, torch gathers), and
# torchrun at world size 1 on the RCCL path (--sharded).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for n in 2 4; do
  LK_BENCH_BACKEND=gloo timeout -k 10 400 python bench.py --gpus $n --steps 3 --warmup 1 --no-cpu-baseline --no-host-path > gpurun_out/r5_gloo_n$n.log 2>&1
  rc=$?; echo "gloo n$n rc=$rc"; grep '^{' gpurun_out/r5_gloo_n$n.log | tail -n 1 | cut -c 1-600
  [ $rc -eq 0 ] || exit $rc
done
exit 0
