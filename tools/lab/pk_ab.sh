#!/bin/bash
# lab A/B: packed (default build) vs scalar (LK_PK_SCALE=0 build, liblk_hip_pk0.so) scale FMAs in the
# batched kernels: batched parity tests on the default build, then C3 / C5 timings of both.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread -k "skinny or batched or mul_mat_vs or gemm or wide or c5" > gpurun_out/pk_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/pk_pytest.log; [ $rc -eq 0 ] || exit $rc
for lib in "" llama.kotlin_amd/ggml_hip/liblk_hip_pk0.so "" llama.kotlin_amd/ggml_hip/liblk_hip_pk0.so; do
  echo "== lib ${lib:-default}"
  LK_HIP_LIB=$lib timeout -k 10 120 python tools/skinny_probe.py 2>&1 | grep -v amdgpu.ids | head -2 || exit 1
  LK_HIP_LIB=$lib timeout -k 10 120 python tools/gemm_probe.py 2>&1 | grep -v amdgpu.ids | python3 -c "import sys,ast; d=ast.literal_eval(sys.stdin.read().strip()); print({k: v['avg_launch_us'] for k, v in d.items()})" || exit 1
done
