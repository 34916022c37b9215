#!/bin/bash
# PMC passes over the wide-GEMM lab binary (data movement only): HBM fetch, L2 hit/miss.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
BIN=${1:-tools/lab/wide_lab_nc}
i=0
for set in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc_wide/p$i -o run -- $BIN > gpurun_out/pmc_wide_p$i.log 2>&1 || { echo "pass $i failed"; tail -3 gpurun_out/pmc_wide_p$i.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(list)
for f in glob.glob("gpurun_out/pmc_wide/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "wide" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    print(f"{k:20s} {sum(v)/len(v):16.1f}  (n={len(v)})")
PY
