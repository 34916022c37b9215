#!/bin/bash
# Round 5: the whole GPU suite on the current library (gemm_q_* split-K on the sc1 hand-off).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 150 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r5_full3.log 2>&1
rc=$?; echo "gpu suite rc=$rc"; grep -E "FAILED|ERROR|passed|failed|^E  " gpurun_out/r5_full3.log | tail -n 30
exit $rc
