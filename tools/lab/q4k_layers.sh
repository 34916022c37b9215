#!/bin/bash
# lab: the bench's next_rows lines (incl. the Q4_K layer lines) alone, plus their kernel trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-headline --no-chain --no-cpu-baseline --no-host-path > gpurun_out/q4k_bench.json 2> gpurun_out/q4k_bench.err || exit $?
python3 -c "
import json; d=json.loads(open('gpurun_out/q4k_bench.json').read().strip().splitlines()[-1])
print(json.dumps({k: v for k, v in d['next_rows'].items() if 'layer' in k}, indent=1)); print({k:v.get('avg_launch_us') for k,v in d['next_rows'].items()})"
