#!/bin/bash
# Round 5 lab A/Bs: decode-chain successor prefetch (LK_PF = 1 / 3 units per wave, tools/pf_probe.py:
# plain vs linked plans alternating in one process), and C5 with the wide kernel's MFMA / scale-FMA
# interleave (LK_WIDE_SCHED=2) against the product.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for u in 1 3; do
  timeout -k 10 300 env LK_HIP_LIB=$PWD/llama.kotlin_amd/ggml_hip/liblk_hip_pf$u.so LK_PF_UNITS=$u python -u tools/pf_probe.py 3 \
    > gpurun_out/r5_pf$u.json 2> gpurun_out/r5_pf$u.err
  rc=$?; echo "pf$u rc=$rc"; cat gpurun_out/r5_pf$u.json; tail -n 3 gpurun_out/r5_pf$u.err
  if [ $rc -ne 0 ]; then exit $rc; fi
done
ROUNDS=3 bash tools/ab.sh "default llama.kotlin_amd/ggml_hip/liblk_hip_ws2.so" c5 || exit $?
cp gpurun_out/ab.jsonl gpurun_out/ab_c5_ws2.jsonl
exit 0
