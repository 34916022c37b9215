#!/bin/bash
# lab: stream kernel with rows handed out per wave from an LDS counter (LK_STREAM_DYN=1) against
# the fixed eighth per wave (0): per-wave timelines of the layer launch and of single launches
# (binaries cross-compiled beforehand: tools/lab/trace_dyn{0,1}), then the GPU suite and a bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for args in "8" "16 0" "8 4" "8 6" "8 0123"; do
  for d in 0 1 0 1; do
    echo "== dyn=$d args=$args"
    timeout -k 10 120 tools/lab/trace_dyn$d $args || exit $?
  done
done > gpurun_out/dyn_trace.log 2>&1
rc=$?; grep -E "^==|layer launch|single launch|span inside|mean wave exit|exit by wave|workgroup last" gpurun_out/dyn_trace.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/dyn_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 5 gpurun_out/dyn_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/dyn_bench.json 2> gpurun_out/dyn_bench.err
rc=$?; echo "bench rc=$rc"; python3 -c "
import json; d=json.loads(open('gpurun_out/dyn_bench.json').read().strip().splitlines()[-1])
print(d['value'], d['tokens_per_s'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['decode_chain']['tokens_per_s'], d['headline_q4_0_4096x4096_n1']['avg_launch_us'], {k:v['avg_launch_us'] for k,v in d['n1_configs'].items()})"
exit $rc
