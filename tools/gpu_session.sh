#!/bin/bash
# One GPU session: the selected GPU tests (PYTEST_K; "all" = every -m gpu test), then an optional
# A/B of library builds (AB_LIBS, AB_SECTIONS; tools/ab.sh). Each step under its own time limit,
# chained so the first failure ends the session.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
K=${PYTEST_K:-all}
if [ "$K" != none ]; then
  if [ "$K" = all ]; then KARG=(); else KARG=(-k "$K"); fi
  timeout -k 10 ${PYTEST_TIMEOUT:-900} python -u -m pytest tests -v -m gpu -x --timeout 150 --timeout-method thread "${KARG[@]}" > gpurun_out/session_pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/session_pytest.log | tail -n 3
  [ $rc -eq 0 ] || { tail -n 40 gpurun_out/session_pytest.log; exit $rc; }
fi
if [ -n "$AB_LIBS" ]; then
  ROUNDS=${ROUNDS:-2} bash tools/ab.sh "$AB_LIBS" $AB_SECTIONS
  rc=$?; echo "ab rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$AB_ENV" ]; then
  ROUNDS=${ROUNDS:-2} bash tools/ab_env.sh "$AB_ENV" $AB_SECTIONS
  rc=$?; echo "ab_env rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
exit 0
