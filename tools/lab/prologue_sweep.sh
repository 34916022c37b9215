#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"
for defs in "-DLK_PROLOGUE_ORDER=0" "-DLK_PROLOGUE_ORDER=1" "-DLK_PROLOGUE_ORDER=2" "-DLK_PROLOGUE_ORDER=0 -DLK_STREAM_D=4" "-DLK_PROLOGUE_ORDER=2 -DLK_STREAM_D=4"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -DNO_TRACE $defs -I include tools/lab/trace.hip -o /tmp/tr -L/opt/rocm/lib -lrccl 2>/dev/null || exit 1
  echo "== $defs"; timeout -k 10 60 /tmp/tr 8 | grep "layer launch" || exit 1; timeout -k 10 60 /tmp/tr 8 3 | grep "layer launch\|single" || exit 1
done
