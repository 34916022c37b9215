# lab diagnostic: test_graph_gpu after test_gpu_parity under switches
cd $GRAFT_REPO_ROOT
for v in "" "LK_GRAPH_NO_DIRECT=1" "LK_KPART_OFF=1"; do
  echo "== parity + graph [$v]"
  env $v timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_graph_gpu.py -q -m gpu --timeout 100 --timeout-method thread 2>&1 | grep -E "passed|failed|FAILED" | tail -3
done
