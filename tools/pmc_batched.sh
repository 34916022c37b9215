#!/bin/bash
# SQ counters (instruction mix, waits, MFMA busy) of the batched kernels on the bench's batched
# configs (tools/gemm_probe.py: C3 Q4_0 / Q4_1 N = 32, C5, C1), per kernel name, one pass per
# counter set; per-wave averages. Output: gpurun_out/pmc_batched/summary.txt
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_batched; rm -rf $OUT; mkdir -p $OUT
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $OUT/p$i -o run -- python3 tools/gemm_probe.py > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 $OUT/p$i.log; exit 1; }
done
python3 - <<'PY' > $OUT/summary.txt
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/pmc_batched/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        if "lk::" in k:
            agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in sorted(agg.items()):
    w = sum(cs["SQ_WAVES"]) / len(cs["SQ_WAVES"]) if cs.get("SQ_WAVES") else 1
    print(f"== {k}  (dispatches {len(cs.get('SQ_WAVES', []))}, waves per dispatch {w:.0f}; per-wave averages; SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_* in quad-cycles)")
    for c, v in sorted(cs.items()):
        m = sum(v) / len(v)
        if c in ("FETCH_SIZE", "WRITE_SIZE"):  # KB per dispatch; HBM bytes = FETCH_SIZE x 2 (gfx950) + WRITE_SIZE
            mb = m * (2 if c == "FETCH_SIZE" else 1) / 1e3
            print(f"  {c:28s} {m:16.1f} KB   per dispatch {mb:10.2f} MB{' (x2, gfx950)' if c == 'FETCH_SIZE' else ''}")
        else:
            print(f"  {c:28s} {m:16.1f}   per wave {m / w:12.1f}")
PY
cat $OUT/summary.txt
