#!/bin/bash
# lab: L2 hit rate and LDS activity of gemm_wide2_kernel (tracer binaries, LK_WIDE2=1) and of
# gemm_wide_kernel (LK_WIDE2=0), one counter pass per run
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/w2pmc; rm -rf $OUT; mkdir -p $OUT
i=0
for cfg in "1 w2_trace" "1 w2_trace_m1" "0 w2_trace"; do
  set -- $cfg
  for set in "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES"; do
    i=$((i+1))
    LK_WIDE2=$1 timeout -s KILL 60 rocprofv3 --pmc $set --output-format csv -d $OUT/p$i -o run -- tools/lab/$2 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 $OUT/p$i.log; exit 1; }
    echo "== LK_WIDE2=$1 $2: $set"
    python3 - $OUT/p$i <<'PY'
import csv, glob, collections, sys
agg = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "gemm_wide" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    print(f"  {k:24s} mean over {len(v)} launches {sum(v) / len(v):16.1f}")
PY
  done
done
