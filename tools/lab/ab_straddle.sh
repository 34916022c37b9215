cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread -k "plan or chain or graph" > gpurun_out/t.log 2>&1; echo pytest rc=$?; tail -2 gpurun_out/t.log
bash tools/lab/run_trace.sh "" "16 0123456" > gpurun_out/trace2.log 2>&1; echo rc=$?; head -12 gpurun_out/trace2.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-headline --no-batched --no-cpu-baseline --no-host-path > gpurun_out/b.log 2>&1; echo bench rc=$?
python -c "import json;d=json.loads(open('gpurun_out/b.log').read().strip().splitlines()[-1]);print(d['value'],d['tokens_per_s'],d['roofline']['avg_launch_us'],d['roofline']['frac'],d['decode_chain'], d['persistent_chain'])"
LK_STRADDLE=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-headline --no-batched --no-cpu-baseline --no-host-path > gpurun_out/b2.log 2>&1; echo bench rc=$?
python -c "import json;d=json.loads(open('gpurun_out/b2.log').read().strip().splitlines()[-1]);print(d['value'],d['tokens_per_s'],d['roofline']['avg_launch_us'],d['roofline']['frac'],d['decode_chain'])"
