#!/bin/bash
# fused split-K reduction in the skinny pair kernel: skinny/batched parity tests (fused, then
# unfused), then C3 per call fused vs LK_SKP_UNFUSED=1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread -k "skinny or batched or mul_mat_vs or gemm or c3" > gpurun_out/fused_pytest.log 2>&1
rc=$?; echo "pytest fused rc=$rc"; tail -n 3 gpurun_out/fused_pytest.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1 0 1; do
  echo "== unfused $v"
  if [ $v = 1 ]; then export LK_SKP_UNFUSED=1; else unset LK_SKP_UNFUSED; fi
  timeout -k 10 120 python tools/gemm_probe.py 2>&1 | grep -v amdgpu.ids | python3 -c "import sys,ast; d=ast.literal_eval(sys.stdin.read().strip()); print({k: v['avg_launch_us'] for k, v in d.items() if k.startswith('c3')})" || exit 1
done
