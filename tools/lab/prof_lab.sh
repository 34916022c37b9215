#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
LIB=llama.kotlin_amd/ggml_hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/lab/lab.hip -o tools/lab/lab -L$LIB -llk_hip -Wl,-rpath,$PWD/$LIB || exit 1
OUT=gpurun_out/labprof; rm -rf $OUT; mkdir -p $OUT
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS TA_BUSY_avr TCP_TCC_READ_REQ_sum SQ_INSTS_SMEM SQ_ACTIVE_INST_MISC" ; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $OUT/p$i -o run -- tools/lab/lab 48 1 prof > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; }
done
python3 - <<'PY'
import csv, collections, glob
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/labprof/*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"][:36]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    if "fill" in k: continue
    print(k)
    print("   ", {c: round(sum(v) / len(v)) for c, v in sorted(d.items())})
PY
