#!/bin/bash
# A/B of liblk_hip.so builds on the GPU box: tools/ab.sh "<lib1> <lib2> ..." [probe sections...]
# ("default" = the in-tree build). Rounds alternate the builds (A B A B ...) so clock drift
# spreads over all of them. One JSON line per run in gpurun_out/ab.jsonl.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
LIBS=$1; shift
ROUNDS=${ROUNDS:-2}
: > gpurun_out/ab.jsonl
for r in $(seq 1 $ROUNDS); do
  for lib in $LIBS; do
    if [ "$lib" = default ]; then unset LK_HIP_LIB; else export LK_HIP_LIB=$PWD/$lib; fi
    timeout -k 10 300 python tools/probe.py "$@" >> gpurun_out/ab.jsonl 2> gpurun_out/ab_err.log
    rc=$?
    if [ $rc -ne 0 ]; then echo "probe rc=$rc ($lib)"; tail -5 gpurun_out/ab_err.log; exit $rc; fi
    tail -n 1 gpurun_out/ab.jsonl
  done
done
