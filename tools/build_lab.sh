#!/bin/bash
# Lab builds of liblk_hip.so with compile-time switches (never the product): tools/build_lab.sh <name> [-DFLAG ...]
# -> llama.kotlin_amd/ggml_hip/liblk_hip_<name>.so (load with LK_HIP_LIB)
cd "$(dirname "$0")/../llama.kotlin_amd"
name=$1; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -fno-slp-vectorize \
  -mllvm -amdgpu-kernarg-preload-count=8 "$@" \
  -shared -o ggml_hip/liblk_hip_$name.so csrc/lk_hip.hip csrc/lk_gguf.cpp csrc/lk_comm.cpp csrc/lk_p2p.hip -L/opt/rocm/lib -lrccl
