#!/bin/bash
# 8 vs 16 waves per workgroup on CPL-1 (K <= 4096) launches only
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
for s in 0 0000 000000000000 0123; do
  for b in sw_d3 sw_w16; do echo "== $b $s"; timeout -k 10 60 tools/lab/$b 32 $s | grep -E "launch" || exit 1; done
done
