#!/bin/bash
# Round 5 root cause, built directly: tile-counter growth while torch's default (null) stream is busy,
# round-4 library vs current (tests/diag_counter_growth.py BUSY=1); then the new scratch test, the
# fixed multi-GPU chain test and the chain probe (32 layers) on the current library.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in liblk_hip_r4.so liblk_hip.so; do
  timeout -k 10 240 env LK_HIP_LIB=$PWD/llama.kotlin_amd/ggml_hip/$lib BUSY=1 REPS=2 python -u tests/diag_counter_growth.py \
    > gpurun_out/r5_busy_$lib.log 2>&1
  rc=$?; echo "busy growth $lib rc=$rc"; head -n 6 gpurun_out/r5_busy_$lib.log; tail -n 1 gpurun_out/r5_busy_$lib.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
timeout -k 10 400 python -u -m pytest tests/test_scratch_gpu.py tests/test_p2p_chain_gpu.py -v -m gpu --timeout 150 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/r5_scratch_chain.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASSED|FAILED|ERROR|^E  " gpurun_out/r5_scratch_chain.log | head -n 30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/chain_probe.py 32 > gpurun_out/r5_chain_probe32.json 2> gpurun_out/r5_chain_probe32.err
rc=$?; echo "chain probe rc=$rc"; cat gpurun_out/r5_chain_probe32.json; tail -n 3 gpurun_out/r5_chain_probe32.err
exit 0
