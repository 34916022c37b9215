#!/bin/bash
# Round 5 root cause: tile-counter growth on the host path, round-4 library vs current.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in liblk_hip_r4.so liblk_hip.so; do
  timeout -k 10 300 env LK_HIP_LIB=$PWD/llama.kotlin_amd/ggml_hip/$lib python -u tests/diag_counter_growth.py > gpurun_out/r5_growth_$lib.log 2>&1
  rc=$?; echo "$lib rc=$rc"; tail -n 12 gpurun_out/r5_growth_$lib.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
exit 0
