#!/bin/bash
# Build + run the GEMV lab on the GPU box (links the in-tree liblk_hip.so).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
LIB=llama.kotlin_amd/ggml_hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/lab/lab.hip -o tools/lab/lab -L$LIB -llk_hip -Wl,-rpath,$PWD/$LIB || exit 1
timeout -k 10 300 tools/lab/lab "$@"
