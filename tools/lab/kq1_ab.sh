#!/bin/bash
# Q4_K batch-1 change: K-quant parity tests, then next_rows (K-quant lines)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kquant.py -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/kq1_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/kq1_pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 120 python tools/lab/next_rows.py 2>&1 | grep -v amdgpu.ids | python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip()); print({k: v['avg_launch_us'] for k, v in d.items() if k.startswith('q')})" || exit 1
done
