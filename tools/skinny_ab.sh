#!/bin/bash
# skinny GEMM A/B: parity tests with the wave-pair kernel forced on for every N (LK_SKINNY_PAIR=2),
# then probe timings: 1 = pairs for N > 16 (default), 2 = pairs for every N, 0 = one wave per SIMD.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
LK_SKINNY_PAIR=2 timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread -k "skinny or batched or mul_mat_vs" > gpurun_out/ab_pytest.log 2>&1
rc=$?; echo "pytest(pair=2) rc=$rc"; tail -n 3 gpurun_out/ab_pytest.log; [ $rc -eq 0 ] || exit $rc
for v in 2 0 2 0; do
  LK_SKINNY_PAIR=$v TAG=pair$v timeout -k 10 120 python tools/skinny_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
done
