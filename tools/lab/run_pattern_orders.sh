#!/bin/bash
# pattern lab built with each LK_PROLOGUE_ORDER (production kernel line) - lab helper
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
for o in 0; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -DLK_PROLOGUE_ORDER=$o -I include tools/lab/pattern.hip -o tools/lab/pattern || exit 1
  for c in "$@"; do echo "== order $o"; timeout -k 10 120 tools/lab/pattern $c | grep -E "launch =|production|NW=8|X0" || exit 1; done
done
