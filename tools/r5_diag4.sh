#!/bin/bash
# Round 5 root cause: the round-4 library over the GPU test files up to the graph tests, four times,
# the graph test dumping a wrong node-by-node down projection (gpurun_out/diag_d_<i>.npz).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2 3 4; do
  timeout -k 10 300 env LK_HIP_LIB=$PWD/llama.kotlin_amd/ggml_hip/liblk_hip_r4.so LK_DIAG_DUMP=$PWD/gpurun_out/diag_d_$i.npz \
    python -u -m pytest tests/test_abi.py tests/test_chain_gpu.py tests/test_direct_dots.py tests/test_gguf.py tests/test_gguf_gpu.py \
    tests/test_golden.py tests/test_gpu_parity.py tests/test_graph_gpu.py -q -m gpu --timeout 150 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/r5_diag4_$i.log 2>&1
  rc=$?; echo "r4 run $i rc=$rc"; grep -E "^E  |passed|failed" gpurun_out/r5_diag4_$i.log | head -n 12
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
exit 0
