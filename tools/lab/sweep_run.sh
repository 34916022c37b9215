#!/bin/bash
# usage: sweep_run.sh "<layer shapes>" bin1 bin2 ... — prebuilt trace-lab binaries, NO_TRACE timing only
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
S=$1; shift
for b in "$@"; do echo "== $b $S"; timeout -k 10 60 tools/lab/$b 32 $S || exit $?; done
