#!/bin/bash
# A/B of lab builds of liblk_hip.so on the batched configs (C3 lines of tools/gemm_probe.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in ${LIBS:-liblk_hip.so}; do
  LK_HIP_LIB=$PWD/llama.kotlin_amd/ggml_hip/$lib timeout -k 10 120 python tools/gemm_probe.py > gpurun_out/ab_$lib.log 2>&1 || { echo "$lib failed"; tail -3 gpurun_out/ab_$lib.log; exit 1; }
  python3 -c "
import ast,sys; d=ast.literal_eval(open('gpurun_out/ab_$lib.log').read().strip().splitlines()[-1])
print('$lib', {k: v['avg_launch_us'] for k, v in d.items()})"
done
if [ -n "$PMC" ]; then bash tools/lab/sk_pmc.sh 2>&1 | tail -42; fi
