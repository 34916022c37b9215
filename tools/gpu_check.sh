#!/bin/bash
# One GPU session: parity tests, smoke, a short bench. Each GPU step has its own time
# limit; a fault/abort/timeout (anything but exit 0/1) ends the session.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "== $name" ; date
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
  return 0
}
step pytest_gpu 900 python -m pytest tests -q -m gpu -x
#step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
#step bench 600 python bench.py --steps 10 --warmup 3
