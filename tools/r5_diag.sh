#!/bin/bash
# Round 5: the full GPU suite on the round-4 library (LK_HIP_LIB, lab build of the round-4 tree, without
# the round-5 tests that need the new diagnostics), then on the current library. A test failure (rc 1)
# does not stop the session; anything else (fault, abort, timeout) does.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # run <log> <env...> -- pytest args
  local log=$1; shift
  timeout -k 10 600 env "$@" > "gpurun_out/$log" 2>&1
  local rc=$?
  echo "$log rc=$rc"; grep -E "^(FAILED|ERROR)|passed|failed" "gpurun_out/$log" | tail -n 8
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
  return 0
}
if [ -z "$SKIP_R4" ]; then
  run r5_suite_r4lib.log LK_HIP_LIB=$PWD/llama.kotlin_amd/ggml_hip/liblk_hip_r4.so \
    python -u -m pytest tests -q -m gpu --timeout 150 --timeout-method thread --ignore tests/test_scratch_gpu.py -p no:cacheprovider
fi
run r5_suite.log LK_X=1 python -u -m pytest tests -q -m gpu -x --timeout 150 --timeout-method thread -p no:cacheprovider
exit 0
