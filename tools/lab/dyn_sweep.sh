#!/bin/bash
# lab: LK_STREAM_DYN sweep (0 = fixed eighth per wave; c = rows handed out c units at a time)
# on the layer launch and the 4-matrix attention group (binaries: tools/lab/trace_dyn<c>)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for args in "8" "8 0123" "8 6"; do
  for rep in 1 2; do
    for d in ${DYNS:-0 1 2 4 8}; do
      echo "== dyn=$d args=$args"
      timeout -k 10 120 tools/lab/trace_dyn$d $args || exit $?
    done
  done
done > gpurun_out/dyn_sweep.log 2>&1
rc=$?; grep -E "^==|layer launch|mean wave exit|exit by wave" gpurun_out/dyn_sweep.log; exit $rc
