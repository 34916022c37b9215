#!/bin/bash
# One GPU session (round 6: replaces the per-session tools/r5_* scripts). Every GPU step runs under a
# time limit of its own; the first failing step ends the session.
#   TESTS     pytest targets, or "all" (= tests/ -m gpu); empty: no tests. TESTS_K: optional -k expression
#   BENCH     bench.py arguments; empty: no bench. TAG names the outputs (default s)
#   PROF      1: the bench command once more under rocprofv3 --kernel-trace --stats (gpurun_out/prof_<tag>/)
#   PMC       counter sets for separate --pmc passes of PMC_CMD (e.g. "FETCH_SIZE|WRITE_SIZE"), one pass each
#   AB_ENV / AB_LIBS / AB_SECTIONS / ROUNDS   A/B through tools/ab_env.sh / tools/ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-s}
if [ -n "$TESTS" ]; then
  if [ "$TESTS" = all ]; then T=(tests); else read -r -a T <<< "$TESTS"; fi
  KARG=(); [ -n "$TESTS_K" ] && KARG=(-k "$TESTS_K")
  timeout -k 10 ${TESTS_TIMEOUT:-900} python -u -m pytest "${T[@]}" -v -m gpu -x --timeout 150 --timeout-method thread \
    -p no:cacheprovider "${KARG[@]}" > gpurun_out/tests_$TAG.log 2>&1
  rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|error" gpurun_out/tests_$TAG.log | tail -n 3
  [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/tests_$TAG.log | tail -n 30; exit $rc; }
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-600} python -u bench.py $BENCH > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
  rc=$?; echo "bench rc=$rc"; tail -c 3000 gpurun_out/bench_$TAG.json; echo
  [ $rc -eq 0 ] || { tail -n 30 gpurun_out/bench_$TAG.err; exit $rc; }
  if [ "$PROF" = 1 ]; then
    timeout -k 10 ${PROF_TIMEOUT:-600} rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run -- python3 bench.py $BENCH \
      > gpurun_out/prof_$TAG.log 2>&1
    rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || { tail -n 20 gpurun_out/prof_$TAG.log; exit $rc; }
  fi
fi
if [ -n "$PMC" ]; then
  IFS='|' read -r -a SETS <<< "$PMC"
  i=0
  for c in "${SETS[@]}"; do
    timeout -s KILL ${PMC_TIMEOUT:-120} rocprofv3 --pmc $c -d gpurun_out/pmc_${TAG}_$i -o run -- ${PMC_CMD:-python3 bench.py --steps 3 --warmup 1} \
      > gpurun_out/pmc_${TAG}_$i.log 2>&1
    rc=$?; echo "pmc[$c] rc=$rc"; [ $rc -eq 0 ] || { tail -n 20 gpurun_out/pmc_${TAG}_$i.log; exit $rc; }
    i=$((i + 1))
  done
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
