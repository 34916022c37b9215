#!/bin/bash
# usage: run_trace.sh "<defines>" "<args>" ["<args>" ...]  (defines e.g. "-DLK_WEIGHT_AUX=0")
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
DEFS=$1; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 $DEFS -I include tools/lab/trace.hip -o tools/lab/trace || exit 1
for a in "$@"; do echo "== trace [$DEFS] $a"; timeout -k 10 120 tools/lab/trace $a || exit $?; done
