#!/bin/bash
# lab: K-quant GPU tests, then Q2_K and Q4_K batch-1 A/B (kquant_n1_kernel vs the stream kernel)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kquant.py -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/kq_pytest.log 2>&1
rc=$?; tail -n 3 gpurun_out/kq_pytest.log; [ $rc -eq 0 ] || exit $rc
for t in Q2_K Q4_K; do for v in 0 1 0 1; do
  KQ_TYPE=$t LK_KQ_STREAM=$v timeout -k 10 180 python tools/lab/kq_stream_probe.py 2>&1 | grep LK_KQ_STREAM || exit 1
done; done
