#!/bin/bash
# Round 5: adjacent-node merging in plans — the plan / chain / graph / sharded / p2p GPU tests, then the
# A/B against LK_NO_MERGE=1 on the layer launch and the decode chain.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_chain_gpu.py tests/test_graph_gpu.py tests/test_sharded_gpu.py tests/test_p2p_gpu.py \
  tests/test_p2p_chain_gpu.py tests/test_gpu_parity.py -q -m gpu --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/merge_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 3 gpurun_out/merge_tests.log
[ $rc -eq 0 ] || exit $rc
ROUNDS=3 bash tools/ab_env.sh "- LK_NO_MERGE=1" chain layer || exit $?
cp gpurun_out/ab_env.jsonl gpurun_out/ab_merge.jsonl
exit 0
