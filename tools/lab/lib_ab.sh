#!/bin/bash
# lab: batched probe (C3 / C5 per-call times) on the product library and on a lab build ($1)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
for lib in "" "$1" "" "$1"; do
  echo "== ${lib:-product}"
  LK_HIP_LIB=$lib timeout -k 10 120 python tools/gemm_probe.py 2>&1 | grep -v amdgpu.ids | python3 -c "import sys,ast; d=ast.literal_eval(sys.stdin.read().strip()); print({k: v['avg_launch_us'] for k, v in d.items()})" || exit 1
done
