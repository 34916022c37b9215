#!/bin/bash
# One GPU session: parity tests, smoke, bench, kernel trace. Each GPU step has its own time
# limit; a fault/abort/timeout (anything but exit 0/1) ends the session.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "== $name" ; date
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -n ${TAIL:-6} "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping after rc=$rc"; exit $rc; fi
  return 0
}
[ -z "$NO_TESTS" ] && step pytest_gpu 900 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread
[ -n "$SMOKE" ] && step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py --steps 20 --warmup 5
[ -n "$PROF" ] && step prof_trace 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_trace -o run -- python3 bench.py --steps 20 --warmup 5 --no-headline --no-chain --no-batched --no-cpu-baseline
[ -n "$PROF" ] && grep -h "gemv\|Name" gpurun_out/prof_trace/run_kernel_stats.csv
exit 0
