#!/bin/bash
# usage: run_q32_trace.sh "<defines>" "<args>" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
DEFS=$1; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize $DEFS -I include tools/lab/q32_trace.hip -o tools/lab/q32_trace -L/opt/rocm/lib -lrccl || exit 1
for a in "$@"; do echo "== q32 trace [$DEFS] $a"; timeout -k 10 120 tools/lab/q32_trace $a || exit $?; done
