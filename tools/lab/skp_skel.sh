#!/bin/bash
# lab: C3 per-call time of the skinny pair kernel's skeleton builds (LK_SKP_SKEL 1-5, wrong
# results) against the product build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
for lib in ${LIBS:-"" tools/lab/liblk_skel1.so tools/lab/liblk_skel2.so tools/lab/liblk_skel3.so tools/lab/liblk_skel4.so tools/lab/liblk_skel5.so ""}; do
  [ "$lib" = product ] && lib=""; echo "== ${lib:-product}"
  LK_HIP_LIB=${lib:+$PWD/$lib} timeout -k 10 120 python tools/gemm_probe.py 2>&1 | grep -v amdgpu.ids | python3 -c "import sys,ast; d=ast.literal_eval(sys.stdin.read().strip()); print({k: v['avg_launch_us'] for k, v in d.items() if k.startswith('c3')})" || exit 1
done
