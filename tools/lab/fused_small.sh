#!/bin/bash
# fused split-K reduction in the one-wave skinny kernel (N <= 16): skinny parity tests, then the
# skinny probe shapes fused vs LK_SKP_UNFUSED=1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread -k "skinny or batched or mul_mat_vs or gemm" > gpurun_out/fs_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 2 gpurun_out/fs_pytest.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1 0 1; do
  echo "== unfused $v"
  if [ $v = 1 ]; then export LK_SKP_UNFUSED=1; else unset LK_SKP_UNFUSED; fi
  timeout -k 10 120 python tools/skinny_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
done
