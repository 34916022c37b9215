#!/bin/bash
# lab: C3 per call with and without the split-K reduce launch (LK_LAB_SKIP_REDUCE, wrong results)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
for v in 0 1 0 1; do
  echo "== skip reduce $v"
  if [ $v = 1 ]; then export LK_LAB_SKIP_REDUCE=1; else unset LK_LAB_SKIP_REDUCE; fi
  timeout -k 10 120 python tools/gemm_probe.py 2>&1 | grep -v amdgpu.ids | python3 -c "import sys,ast; d=ast.literal_eval(sys.stdin.read().strip()); print({k: v['avg_launch_us'] for k, v in d.items() if k.startswith('c3')})" || exit 1
done
