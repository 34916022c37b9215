#!/bin/bash
# skinny GEMM A/B: parity tests on the default build, lab timelines of the variants, probe timings.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread -k "skinny or batched or mul_mat_vs" > gpurun_out/ab_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/ab_pytest.log; [ $rc -eq 0 ] || exit $rc
for b in skinny_trace_old skinny_trace; do
  echo "== $b"; timeout -k 10 60 tools/lab/$b 11008 4096 32 | grep -E "untraced|unit0 landed|unit0 done|loop done" || exit 1
  timeout -k 10 60 tools/lab/$b 11008 4096 4 | grep -E "untraced" || exit 1
done
timeout -k 10 120 python tools/skinny_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
