#!/bin/bash
# lab: skinny pair kernel change: skinny parity tests on the product build, then C3 probe times on
# the product build and a lab build ($1)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread -k "skinny or batched or mul_mat_vs or gemm or c3" > gpurun_out/skp_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/skp_pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/lab/lib_ab.sh "$1"
