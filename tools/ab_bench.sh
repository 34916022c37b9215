#!/bin/bash
# A/B of run-time switches on bench.py's own lines (value, decode_chain): tools/ab_bench.sh "<VAR=val,...> ..."
# ("-" = no switch); rounds alternate the settings. Lines in gpurun_out/ab_bench.jsonl.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
SETS=$1; shift
ROUNDS=${ROUNDS:-2}
: > gpurun_out/ab_bench.jsonl
for r in $(seq 1 $ROUNDS); do
  for set in $SETS; do
    envs=()
    [ "$set" = - ] || IFS=, read -ra envs <<< "$set"
    env "${envs[@]}" timeout -k 10 300 python bench.py --no-batched --no-host-path --no-cpu-baseline --no-multi-gpu-cost "$@" \
      > gpurun_out/ab_bench_run.log 2> gpurun_out/ab_bench_err.log
    rc=$?
    if [ $rc -ne 0 ]; then echo "bench rc=$rc ($set)"; tail -5 gpurun_out/ab_bench_err.log; exit $rc; fi
    python - "$set" >> gpurun_out/ab_bench.jsonl <<'PY'
import json, sys
line = [l for l in open("gpurun_out/ab_bench_run.log") if l.startswith("{")][-1]
b = json.loads(line)
pc = b.get("persistent_chain", {})
print(json.dumps({"set": sys.argv[1], "value": b["value"], "decode_tok_s": b["tokens_per_s"],
                  "layer_us": b["roofline"]["avg_launch_us"], "chain32": pc.get("layer_stages", {}).get("tokens_per_s"),
                  "chain128": pc.get("decode_stages", {}).get("tokens_per_s")}))
PY
    tail -n 1 gpurun_out/ab_bench.jsonl
  done
done
