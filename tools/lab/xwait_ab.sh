#!/bin/bash
# lab: the layer launch with and without waiting for the activation image (LK_NO_XWAIT: wrong
# results, timing only) — how much of the per-launch cost the x latency is
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
for defs in "" "-DLK_NO_XWAIT" "" "-DLK_NO_XWAIT"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -DNO_TRACE $defs -I include tools/lab/trace.hip -o /tmp/tr -L/opt/rocm/lib -lrccl 2>/dev/null || exit 1
  echo "== [$defs]"; timeout -k 10 60 /tmp/tr 8 | grep "layer launch" || exit 1; timeout -k 10 60 /tmp/tr 8 3 | grep "layer launch\|single" || exit 1
done
