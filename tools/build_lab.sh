#!/bin/bash
# Lab builds of liblk_hip.so with compile-time switches (never the product): tools/build_lab.sh <name> [-DFLAG ...]
# -> llama.kotlin_amd/ggml_hip/liblk_hip_<name>.so (load with LK_HIP_LIB). Same units and flags as the Makefile.
cd "$(dirname "$0")/../llama.kotlin_amd"
name=$1; shift
F=(--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -fno-slp-vectorize -mllvm -amdgpu-kernarg-preload-count=8)
O=build/lab_$name
rm -rf $O; mkdir -p $O
for s in lk_hip.hip lk_gguf.cpp lk_comm.cpp lk_p2p.hip; do
  /opt/rocm/bin/hipcc "${F[@]}" "$@" -c -o $O/$s.o csrc/$s &
done
/opt/rocm/bin/hipcc "${F[@]}" -mllvm -amdgpu-mfma-vgpr-form "$@" -c -o $O/lk_w32.hip.o csrc/lk_w32.hip &
wait
wait; for s in lk_hip.hip lk_gguf.cpp lk_comm.cpp lk_p2p.hip lk_w32.hip; do [ -s $O/$s.o ] || { echo "lab build failed: $s"; exit 1; }; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ggml_hip/liblk_hip_$name.so $O/*.o -L/opt/rocm/lib -lrccl
