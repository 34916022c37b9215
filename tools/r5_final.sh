#!/bin/bash
# Round-5 end-of-round GPU evidence, part A: every -m gpu test, smoke, the bench line, and the bench
# started by torchrun at world size 1 on the sharded (RCCL C-ABI) path. Outputs under
# gpurun_out/r5/ (copied into profiles/r05/ afterwards). Each step under its own limit, chained.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r5; mkdir -p $O
step() {  # step <name> <secs> <cmd...>: stdout to $O/<name>.log
  local name=$1 secs=$2; shift 2
  echo "== $name"; timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
  local rc=$?; echo "rc=$rc"; tail -n 3 "$O/$name.log"
  [ $rc -eq 0 ] || { echo "stop at $name"; exit $rc; }
}
if [ -z "$SKIP_TESTS" ]; then
  step pytest_gpu 900 python -u -m pytest tests -v -m gpu -x --timeout 200 --timeout-method thread
fi
step smoke 300 python -c "import __graft_entry__ as g; g.build() if False else None; g.smoke(); print('smoke ok')"
step bench 600 python bench.py
grep '^{' $O/bench.log | tail -n 1 > $O/bench_line.json
step bench_sharded 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531 bench.py --sharded --no-cpu-baseline --no-host-path
grep '^{' $O/bench_sharded.log | tail -n 1 > $O/bench_sharded_line.json
echo done
