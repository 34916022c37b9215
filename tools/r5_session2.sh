#!/bin/bash
# Round 5: the whole GPU suite on the current library (multi-GPU chain, scratch lifetime, Q4_1 pitch),
# the chain probe, A/Bs (C5: LK_WIDE_SCHED=1 lab build; C3 / Q4_1 N = 16: the pre-pitch build), then
# the round-4 library over the test files up to the graph tests, dumping a wrong node-by-node down
# projection.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 150 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r5_full.log 2>&1
rc=$?; echo "gpu suite rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r5_full.log | tail -n 20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/chain_probe.py 8 > gpurun_out/r5_chain_probe.json 2> gpurun_out/r5_chain_probe.err
rc=$?; echo "chain probe rc=$rc"; cat gpurun_out/r5_chain_probe.json; tail -n 3 gpurun_out/r5_chain_probe.err
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
ROUNDS=3 bash tools/ab.sh "default llama.kotlin_amd/ggml_hip/liblk_hip_ws1.so" c5 || exit $?
cp gpurun_out/ab.jsonl gpurun_out/ab_c5_ws1.jsonl
ROUNDS=3 bash tools/ab.sh "default llama.kotlin_amd/ggml_hip/liblk_hip_base.so" c3 skinny41 || exit $?
cp gpurun_out/ab.jsonl gpurun_out/ab_c3_pitch.jsonl
bash tools/r5_diag4.sh
exit 0
