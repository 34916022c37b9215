#!/bin/bash
# GPU session for the multi-GPU path on the one-GPU box: sharded tests (world-1 RCCL C-ABI), the
# N=1 bench step, and the gloo rehearsal of the N=2 step (two ranks sharing the GPU; never a measurement).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread -k "shard" > gpurun_out/mgpu_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 5 gpurun_out/mgpu_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-chain --no-headline --no-batched --no-cpu-baseline --no-host-path > gpurun_out/mgpu_n1.log 2>&1
rc=$?; echo "bench n1 rc=$rc"; tail -c 1200 gpurun_out/mgpu_n1.log
[ $rc -eq 0 ] || exit $rc
LK_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/mgpu_gloo.log 2>&1
rc=$?; echo "gloo n2 rc=$rc"; tail -c 1500 gpurun_out/mgpu_gloo.log
exit $rc
