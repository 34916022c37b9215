#!/bin/bash
# GPU session for a kernel change: the selected GPU tests (PYTEST_K), then the batched configs
# (tools/gemm_probe.py) and their kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
K=${PYTEST_K:-batched or skinny or q32 or mul_mat_vs_oracle}
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread -k "$K" > gpurun_out/k_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 25 gpurun_out/k_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/gemm_probe.py > gpurun_out/k_probe.log 2>&1
rc=$?; echo "probe rc=$rc"; tail -n 3 gpurun_out/k_probe.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/k_prof -o run -- python3 tools/gemm_probe.py > gpurun_out/k_prof.log 2>&1
rc=$?; echo "prof rc=$rc"
grep -h "lk::" gpurun_out/k_prof/run_kernel_stats.csv | cut -d, -f1-4
exit $rc
