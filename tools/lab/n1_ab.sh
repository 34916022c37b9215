#!/bin/bash
# lab: batch-1 single launches on the product build and lab builds ($@)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
for lib in "" "$@" ""; do
  echo "== ${lib:-product}"
  LK_HIP_LIB=${lib:+$PWD/$lib} timeout -k 10 180 python tools/lab/n1_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
done
