#!/bin/bash
# Round 5 root cause: the round-4 library with its tile counters visible (liblk_hip_r4c.so), the full
# GPU suite up to the resident-graph tests, the counter sum logged after every test.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/counters_trace.log
timeout -k 10 600 env LK_HIP_LIB=$PWD/llama.kotlin_amd/ggml_hip/liblk_hip_r4c.so LK_DIAG_COUNTERS=$PWD/gpurun_out/counters_trace.log \
  python -u -m pytest tests --ignore tests/test_scratch_gpu.py \
  -q -m gpu --timeout 150 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/r5_diag2.log 2>&1
rc=$?
echo "rc=$rc"; grep -E "^(FAILED|ERROR)|passed|failed" gpurun_out/r5_diag2.log | tail -n 8
awk '$2 != "0"' gpurun_out/counters_trace.log | head -n 20
exit 0
