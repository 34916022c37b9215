#!/bin/bash
# SQ counters of the C3 skinny kernel through the bench's batched configs (tools/gemm_probe.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_sq; rm -rf $OUT; mkdir -p $OUT
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $OUT/p$i -o run -- python3 tools/gemm_probe.py > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 $OUT/p$i.log; exit 1; }
done
for PAT in ${PATS:-"gemm_q32_kernel<2>" "gemm_wide_kernel<2>"}; do
echo "== $PAT"
PAT="$PAT" python3 - <<'PY'
import csv, glob, collections, os
agg = collections.defaultdict(list)
for f in glob.glob("gpurun_out/pmc_sq/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if os.environ["PAT"] in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
w = sum(agg["SQ_WAVES"]) / len(agg["SQ_WAVES"]) if agg.get("SQ_WAVES") else 1
for k, v in sorted(agg.items()):
    m = sum(v) / len(v)
    print(f"{k:28s} {m:16.1f}   per wave {m / w:12.1f}")
PY
done
