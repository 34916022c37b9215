#!/bin/bash
# lab A/B: gemm_wide2_kernel (LK_WIDE2=1, loader/consumer waves) vs gemm_wide_kernel: wide-GEMM
# parity tests on the new kernel, then the batched configs (C5 N=512) on both; W2=2 for 8 consumers
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
W2=${W2:-1}
mkdir -p gpurun_out
LK_WIDE2=$W2 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -m gpu -x --timeout 120 --timeout-method thread -k "wide or c5 or mul_mat_vs" > gpurun_out/w2_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/w2_pytest.log; [ $rc -eq 0 ] || exit $rc
for v in $W2 0 $W2 0; do
  echo "== LK_WIDE2=$v"
  LK_WIDE2=$v timeout -k 10 120 python tools/gemm_probe.py 2>&1 | grep -v amdgpu.ids | python3 -c "import sys,ast; d=ast.literal_eval(sys.stdin.read().strip()); print({k: v['avg_launch_us'] for k, v in d.items()})" || exit 1
done
