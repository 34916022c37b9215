#!/bin/bash
# Kernel-trace stats of the batched configs (C3 N=32, C5 N=512) through tools/gemm_probe.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_gemm
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 tools/gemm_probe.py > $OUT/run.log 2>&1
rc=$?; tail -3 $OUT/run.log
find $OUT -name "*kernel_stats.csv" -exec cat {} \;
exit $rc
