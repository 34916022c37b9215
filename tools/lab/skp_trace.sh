#!/bin/bash
# lab: per-wave timeline of gemm_skinny_pair_kernel on C3 (Q4_0 11008 x 4096, N = 32): product
# build and the no-compute skeleton (LK_SKP_SKEL=5)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
for b in sk_ptrace sk_ptrace5; do
  echo "== $b"; PAIR=1 timeout -k 10 60 tools/lab/$b 11008 4096 32 || exit 1
done
