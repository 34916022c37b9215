# lab diagnostic: test_graph_gpu after test_gpu_parity, default and with kpart off
cd $GRAFT_REPO_ROOT
echo "== parity + graph"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_graph_gpu.py -x -q -m gpu --timeout 100 --timeout-method thread 2>&1 | tail -2
echo "== parity + graph, LK_KPART_OFF=1"
LK_KPART_OFF=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_graph_gpu.py -x -q -m gpu --timeout 100 --timeout-method thread 2>&1 | tail -2
