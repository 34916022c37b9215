#!/bin/bash
# Round 5 A/B: filler DMAs reading one line (product candidate) vs the build before it (liblk_hip_cur.so).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ROUNDS=3 bash tools/ab.sh "default llama.kotlin_amd/ggml_hip/liblk_hip_cur.so" chain layer n1 || exit $?
cp gpurun_out/ab.jsonl gpurun_out/ab_filler.jsonl
exit 0
