#!/bin/bash
# lab: gemm_wide2_kernel on C5 with 4 / 8 consumers, whole kernel vs its skeletons (LDS reads only,
# compute only): per-wave wait shares from the tracer, kernel durations from rocprofv3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/w2m
for w in ${W2S:-1 2}; do
  for b in ${BINS:-w2_trace w2_trace_m1 w2_trace_m2}; do
    echo "== LK_WIDE2=$w $b"
    LK_WIDE2=$w timeout -k 10 60 tools/lab/$b || exit 1
    LK_WIDE2=$w timeout -k 10 60 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/w2m/$w$b -o run -- tools/lab/$b > /dev/null 2>&1 || exit 1
    python3 -c "
import csv,glob
for f in glob.glob('gpurun_out/w2m/$w$b/**/*kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'gemm_wide2' in r['Name'] or 'xsplit' in r['Name'] or 'splitk' in r['Name']: print('  ', r['Name'][:40], r['Calls'], 'avg us', round(float(r['AverageNs'])/1e3, 2), 'min us', round(float(r['MinNs'])/1e3, 2))
"
  done
done
