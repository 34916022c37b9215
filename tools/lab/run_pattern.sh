#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/lab/pattern.hip -o tools/lab/pattern || exit 1
for c in "$@"; do timeout -k 10 120 tools/lab/pattern $c || exit $?; done
