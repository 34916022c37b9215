#!/bin/bash
# One GPU session for a kernel change: the selected GPU tests (PYTEST_K), then the batched probe.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
K=${PYTEST_K:-batched or skinny or mul_mat_vs_oracle}
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread -k "$K" > gpurun_out/quick_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 15 gpurun_out/quick_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/gemm_probe.py > gpurun_out/quick_probe.log 2>&1
rc=$?; echo "probe rc=$rc"; tail -n 5 gpurun_out/quick_probe.log
exit $rc
