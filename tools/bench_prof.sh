#!/bin/bash
# One GPU session: bench (full JSON line), then a rocprofv3 kernel trace of the timed step only.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.log; tail -5 gpurun_out/bench.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_trace -o run -- python3 bench.py --steps 20 --warmup 5 --no-headline --no-chain --no-cpu-baseline > gpurun_out/prof_trace.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -3 gpurun_out/prof_trace.log
find gpurun_out/prof_trace -name "*stats*.csv" -exec cat {} \;
exit $rc
