"""Repeats tests/test_graph_gpu.py::test_layer_graph_equals_sequential[N=4]'s scenario and
reports which node's bytes differ between runs (sequential vs sequential, graph vs sequential)."""
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path[:0] = [os.path.join(ROOT, "llama.kotlin_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import ggml_hip as G  # noqa: E402
import oracle as O  # noqa: E402
from test_graph_gpu import _layer, _sequential  # noqa: E402

G.load_library()
names = ["q", "k", "v", "o", "g", "u", "d"]
bad_seq, bad_graph = {}, {}
for it in range(int(sys.argv[1]) if len(sys.argv) > 1 else 20):
    ga = G.GGMLGraphAllocator(device="host", defaultBufferSize=1 << 20)
    x, nodes = _layer(ga, O, N=4, seed=it % 3)
    want = _sequential(ga, nodes)
    again = _sequential(ga, nodes)
    for j in range(7):
        if want[j] != again[j]:
            bad_seq[names[j]] = bad_seq.get(names[j], 0) + 1
    for _, _, d in nodes:
        ga.setTensorBytes(d, np.zeros(4 * d.ne[0] * d.ne[1], np.uint8))
    g = G.ResidentGraph(ga, nodes)
    g.compute()
    got = [bytes(ga.tensorBytes(d)) for _, _, d in nodes]
    for j in range(7):
        if got[j] != want[j]:
            a = np.frombuffer(got[j], np.float32); b = np.frombuffer(want[j], np.float32)
            nd = int((a != b).sum())
            bad_graph[names[j]] = bad_graph.get(names[j], 0) + 1
            print(f"iter {it} node {names[j]}: {nd}/{a.size} differ, max|diff| {np.abs(a - b).max():.3e}, first at {int(np.argmax(a != b))}", flush=True)
    g.close()
print("seq-vs-seq mismatches", bad_seq, "graph-vs-seq mismatches", bad_graph, flush=True)
