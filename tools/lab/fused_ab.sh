#!/bin/bash
# fused split-K reduction (skinny pair kernel, gemm_sk_kernel): skinny / batched / K-quant parity
# tests, then C3 and Q4_K N=32 per call, fused vs LK_SKP_UNFUSED=1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread -k "skinny or batched or mul_mat_vs or gemm or c3 or c5 or wide or kquant or q4_k" > gpurun_out/fused_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/fused_pytest.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1 0 1; do
  echo "== unfused $v"
  if [ $v = 1 ]; then export LK_SKP_UNFUSED=1; else unset LK_SKP_UNFUSED; fi
  timeout -k 10 120 python tools/gemm_probe.py 2>&1 | grep -v amdgpu.ids | python3 -c "import sys,ast; d=ast.literal_eval(sys.stdin.read().strip()); print({k: v['avg_launch_us'] for k, v in d.items() if k[:2] in ('c3', 'c5')})" || exit 1
  timeout -k 10 120 python tools/lab/next_rows.py 2>&1 | grep -v amdgpu.ids | python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip()); print({k: v['avg_launch_us'] for k, v in d.items() if 'n32' in k})" || exit 1
done
