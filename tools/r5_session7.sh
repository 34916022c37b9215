#!/bin/bash
# Round 5 A/B on C5: 2-block stages with a 5-deep ring (LK_WIDE_SB=2)
# (LK_WIDE_EARLYT=1 lab build) against the product; the batched parity tests on that build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ROUNDS=3 bash tools/ab.sh "default llama.kotlin_amd/ggml_hip/liblk_hip_sb2.so" c5 || exit $?
cp gpurun_out/ab.jsonl gpurun_out/ab_c5_sb2.jsonl
timeout -k 10 300 env LK_HIP_LIB=$PWD/llama.kotlin_amd/ggml_hip/liblk_hip_sb2.so python -u -m pytest tests -q -m gpu -k "wide or c5 or batched or sync" \
  --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/sb2_tests.log 2>&1
echo "sb2 tests rc=$?"; tail -n 3 gpurun_out/sb2_tests.log
exit 0
