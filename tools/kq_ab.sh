#!/bin/bash
# Q4_K batched A/B: K-quant parity tests, then next_rows' Q4_K N=32 line on the MFMA kernel
# (default) and on kquant_nc_kernel (LK_KQ_SK=0)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kquant.py -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/kq_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 5 gpurun_out/kq_pytest.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0 1; do
  echo "== LK_KQ_SK=$v"
  LK_KQ_SK=$v timeout -k 10 300 python tools/lab/next_rows.py 2>/dev/null | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print({k: v[\"avg_launch_us\"] for k, v in d.items() if \"q4_k\" in k})" || exit 1
done
