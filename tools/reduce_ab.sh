#!/bin/bash
# split-K reduce change: skinny/batched parity tests, then the batched probe
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread -k "skinny or batched or wide or mul_mat_vs" > gpurun_out/ab_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/ab_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/skinny_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
