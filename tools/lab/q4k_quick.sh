#!/bin/bash
# lab: K-quant GPU tests, then the Q4_K bench lines (tools/lab/q4k_layers.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kquant.py -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/kq_pytest.log 2>&1
rc=$?; tail -n 2 gpurun_out/kq_pytest.log; [ $rc -eq 0 ] || exit $rc
tools/lab/q4k_layers.sh
