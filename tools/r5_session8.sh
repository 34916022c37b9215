#!/bin/bash
# Round 5: the pair kernel's split on v_cvt_pk_bf16_f32 — bit-identical outputs vs the build before it
# (liblk_hip_cur.so) on a set of batched calls, then the C3 / N = 24 A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/bitcmp.py gpurun_out/bit_new.npz > gpurun_out/bit.log 2>&1 || { tail -5 gpurun_out/bit.log; exit 1; }
timeout -k 10 300 env LK_HIP_LIB=$PWD/llama.kotlin_amd/ggml_hip/liblk_hip_cur.so python tools/bitcmp.py gpurun_out/bit_old.npz >> gpurun_out/bit.log 2>&1 || { tail -5 gpurun_out/bit.log; exit 1; }
python tools/bitcmp.py --cmp gpurun_out/bit_old.npz gpurun_out/bit_new.npz
ROUNDS=3 bash tools/ab.sh "default llama.kotlin_amd/ggml_hip/liblk_hip_cur.so" c3 || exit $?
cp gpurun_out/ab.jsonl gpurun_out/ab_c3_cvt.jsonl
exit 0
