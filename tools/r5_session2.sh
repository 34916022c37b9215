#!/bin/bash
# Round 5: the multi-GPU chain and scratch tests on the current library, then the round-4 library over
# the test files up to the graph tests, four times, dumping a wrong node-by-node down projection.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_p2p_chain_gpu.py tests/test_scratch_gpu.py tests/test_p2p_gpu.py tests/test_chain_gpu.py \
  -v -m gpu --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/r5_chain.log 2>&1
rc=$?; echo "chain tests rc=$rc"; grep -E "PASSED|FAILED|ERROR|^E  " gpurun_out/r5_chain.log | head -n 40
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/chain_probe.py 8 > gpurun_out/r5_chain_probe.json 2> gpurun_out/r5_chain_probe.err
rc=$?; echo "chain probe rc=$rc"; cat gpurun_out/r5_chain_probe.json; tail -n 3 gpurun_out/r5_chain_probe.err
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
ROUNDS=3 bash tools/ab.sh "default llama.kotlin_amd/ggml_hip/liblk_hip_ws1.so" c5
echo "ab rc=$?"
bash tools/r5_diag4.sh
exit 0
