#!/bin/bash
# persistent chain change: chain / plan parity tests, then the bench line (decode_chain and
# persistent_chain figures)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_chain_gpu.py tests/test_graph_gpu.py -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/chain_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/chain_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-batched --no-host-path --no-cpu-baseline > gpurun_out/chain_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/chain_bench.log; exit $rc; }
python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/chain_bench.log') if l.startswith('{')][-1])
print('value', d['value'], 'tok/s', d['tokens_per_s'], 'decode_chain', d['decode_chain']['tokens_per_s'])
print('persistent', {k: (v['tokens_per_s'], v['barrier_timeout']) for k, v in d['persistent_chain'].items()})"
