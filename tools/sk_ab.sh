#!/bin/bash
# skinny GEMM A/B: batched parity tests on the kernel LK_SK selects (default: the product's), probe
# timings for LK_SK = 2 (one wave per SIMD), 1 (wave pairs), 0 (round-1 kernels), then a kernel
# trace of the probe (xsplit / GEMM / reduce split). usage: [SKT=2] tools/sk_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
LK_SK=${SKT:-2} timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread -k "skinny or batched or mul_mat_vs or gemm" > gpurun_out/sk_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 5 gpurun_out/sk_pytest.log; [ $rc -eq 0 ] || exit $rc
for v in 2 1 0 2; do
  LK_SK=$v TAG=sk$v timeout -k 10 120 python tools/skinny_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
done
LK_SK=${SKT:-2} timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sk_prof -o run -- python3 tools/skinny_probe.py > gpurun_out/sk_prof.log 2>&1 || exit 1
python tools/trace_split.py gpurun_out/sk_prof/run_kernel_trace.csv
