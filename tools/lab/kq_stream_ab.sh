#!/bin/bash
# lab: Q4_K batch-1 per-launch times, kquant_n1_kernel (LK_KQ_STREAM=0) vs the stream kernel (1)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
for v in 0 1 0 1; do
  LK_KQ_STREAM=$v timeout -k 10 180 python tools/lab/kq_stream_probe.py 2>&1 | grep LK_KQ_STREAM || exit 1
done
