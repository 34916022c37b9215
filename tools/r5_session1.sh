#!/bin/bash
# Round 5 session: (1) the round-4 library over the test files up to the graph tests, twice, dumping a
# wrong down projection; (2) the full GPU suite on the current library; (3) A/B of kernel-argument
# preloading (layer, chain, n1). Test failures (rc 1) do not stop the session; faults do.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
chk() { if [ $1 -ne 0 ] && [ $1 -ne 1 ]; then echo "stopping after rc=$1"; exit $1; fi; }
for i in 1 2; do
  timeout -k 10 300 env LK_HIP_LIB=$PWD/llama.kotlin_amd/ggml_hip/liblk_hip_r4.so LK_DIAG_DUMP=$PWD/gpurun_out/diag_d_$i.npz \
    python -u -m pytest tests/test_abi.py tests/test_chain_gpu.py tests/test_direct_dots.py tests/test_gguf.py tests/test_gguf_gpu.py \
    tests/test_golden.py tests/test_gpu_parity.py tests/test_graph_gpu.py -q -m gpu --timeout 150 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/r5_diag3_$i.log 2>&1
  rc=$?; echo "r4 run $i rc=$rc"; grep -E "^E  |passed|failed" gpurun_out/r5_diag3_$i.log | head -n 12; chk $rc
done
timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/r5_suite2.log 2>&1
rc=$?; echo "suite rc=$rc"; grep -E "^(FAILED|ERROR)|passed|failed" gpurun_out/r5_suite2.log | tail -n 8; chk $rc
ROUNDS=2 bash tools/ab.sh "default llama.kotlin_amd/ggml_hip/liblk_hip_preload.so" layer chain n1
echo "ab rc=$?"
exit 0
