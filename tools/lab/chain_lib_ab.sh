#!/bin/bash
# lab: bench chain lines (decode_chain, persistent_chain) on the product library and a lab build ($1)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
for lib in "" "$1"; do
  echo "== ${lib:-product}"
  LK_HIP_LIB=$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-batched --no-host-path --no-cpu-baseline --no-headline > gpurun_out/clab.log 2>&1 || { tail -5 gpurun_out/clab.log; exit 1; }
  python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/clab.log') if l.startswith('{')][-1])
print('value', d['value'], 'decode_chain', d['decode_chain']['tokens_per_s'], 'persistent', {k: v['tokens_per_s'] for k, v in d['persistent_chain'].items()})"
done
