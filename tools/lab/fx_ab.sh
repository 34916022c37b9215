#!/bin/bash
# lab A/B of the in-kernel activation split (gemm_sk_kernel fx): parity on the wave-pair kernel
# (LK_SK=1) incl. K-quants, then C3 timings: fused split, separate xsplit, round-1 kernels
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
LK_SK=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_kquant.py -q -m gpu -x --timeout 120 --timeout-method thread -k "skinny or batched or mul_mat_vs or gemm or kquant or q4_k" > gpurun_out/fx_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/fx_pytest.log; [ $rc -eq 0 ] || exit $rc
for cfg in "LK_SK=1" "LK_SK=1 LK_SK_XSPLIT=1" "LK_SK=0" "LK_SK=1"; do
  echo "== $cfg"
  env $cfg timeout -k 10 120 python tools/skinny_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
done
for cfg in "LK_SK_XSPLIT=0" "LK_SK_XSPLIT=1"; do
  echo "== Q4_K $cfg"
  if [ "$cfg" = "LK_SK_XSPLIT=1" ]; then export LK_SK_XSPLIT=1; else unset LK_SK_XSPLIT; fi
  timeout -k 10 300 python tools/lab/next_rows.py 2>/dev/null | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print({k: v['avg_launch_us'] for k, v in d.items() if 'n32' in k})" || exit 1
done
