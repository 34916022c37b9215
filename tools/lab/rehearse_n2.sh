#!/bin/bash
# N = 2 bench path rehearsal on one GPU (gloo collectives, both ranks on the visible GPU)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
LK_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/rehearsal.log 2>&1
rc=$?; echo "rc=$rc"; tail -3 gpurun_out/rehearsal.log
[ $rc -eq 0 ] || exit $rc
grep "^{" gpurun_out/rehearsal.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('value','n_gpus','scaling','ms_per_step')}, d['config']['parallelism'])"
