#!/bin/bash
# lab: Q4_K bench lines on the product library vs a build with ring depth 4 (tools/lab/liblk_hip_d4.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
for lib in "" "$PWD/tools/lab/liblk_hip_d4.so" "" "$PWD/tools/lab/liblk_hip_d4.so"; do
  echo "== ${lib:-product}"
  LK_HIP_LIB=$lib tools/lab/q4k_layers.sh | grep -E "avg_layer_us|q2_k" || exit 1
done
