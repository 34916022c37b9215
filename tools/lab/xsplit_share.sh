#!/bin/bash
# lab: C5 per call with and without the xsplit launch (LK_LAB_SKIP_XSPLIT, wrong results)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
for v in 0 1 0 1; do
  echo "== skip xsplit $v"
  if [ $v = 1 ]; then export LK_LAB_SKIP_XSPLIT=1; else unset LK_LAB_SKIP_XSPLIT; fi
  timeout -k 10 120 python tools/gemm_probe.py 2>&1 | grep -v amdgpu.ids | python3 -c "import sys,ast; d=ast.literal_eval(sys.stdin.read().strip()); print({k: v['avg_launch_us'] for k, v in d.items() if k.startswith('c5')})" || exit 1
done
