#!/bin/bash
# GPU session for host-path changes: the selected GPU tests (PYTEST_K, default all), then the
# bench's host-path lines only.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
K=${PYTEST_K:-}
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread ${K:+-k "$K"} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 15 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-chain --no-headline --no-batched --no-cpu-baseline > gpurun_out/bench_host.log 2>&1
rc=$?; echo "bench rc=$rc"; python -c "import json;d=json.loads(open('gpurun_out/bench_host.log').read().strip().splitlines()[-1]);print(json.dumps(d.get('host_path_pcie')))"
exit $rc
