#!/bin/bash
# A/B of run-time switches on the GPU box: tools/ab_env.sh "<VAR=val,...> <VAR=val,...> ..." [probe sections...]
# ("-" = no switch). Rounds alternate the settings so clock drift spreads over all of them. One JSON
# line per run in gpurun_out/ab_env.jsonl.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
SETS=$1; shift
ROUNDS=${ROUNDS:-2}
: > gpurun_out/ab_env.jsonl
for r in $(seq 1 $ROUNDS); do
  for set in $SETS; do
    envs=()
    [ "$set" = - ] || IFS=, read -ra envs <<< "$set"
    echo -n "{\"set\": \"$set\", \"probe\": " >> gpurun_out/ab_env.jsonl
    env "${envs[@]}" timeout -k 10 300 python tools/probe.py "$@" >> gpurun_out/ab_env.jsonl 2> gpurun_out/ab_env_err.log
    rc=$?
    echo "}" >> gpurun_out/ab_env.jsonl
    if [ $rc -ne 0 ]; then echo "probe rc=$rc ($set)"; tail -5 gpurun_out/ab_env_err.log; exit $rc; fi
    tail -n 1 gpurun_out/ab_env.jsonl
  done
done
