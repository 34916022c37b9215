"""Lab diagnostic (not collected by pytest): test_graph_gpu.py::test_layer_graph_equals_sequential[4]
repeated in one process. Per round: are per-node computeMatMul reruns bit-stable, and which nodes'
resident-graph bytes differ from them (count of differing floats, max abs diff)."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [HERE, ROOT, os.path.join(ROOT, "llama.kotlin_amd"), os.path.join(ROOT, "oracle")]


def main(rounds=int(sys.argv[1]) if len(sys.argv) > 1 else 20):
    import torch
    import oracle as O
    import ggml_hip as G
    from test_graph_gpu import _layer, _sequential
    O.lib()
    G.load_library()
    torch.cuda.set_device(0)
    names = ["q", "k", "v", "o", "g", "u", "d"]
    for r in range(rounds):
        ga = G.GGMLGraphAllocator(device="host", defaultBufferSize=1 << 20)
        x, nodes = _layer(ga, O, N=4, seed=r)
        want = _sequential(ga, nodes)
        again = _sequential(ga, nodes)
        seq_diff = [names[i] for i in range(7) if want[i] != again[i]]
        for _, _, d in nodes:
            ga.setTensorBytes(d, np.zeros(4 * d.ne[0] * d.ne[1], np.uint8))
        g = G.ResidentGraph(ga, nodes)
        g.compute()
        got = [bytes(ga.tensorBytes(d)) for _, _, d in nodes]
        bad = []
        for i in range(7):
            if got[i] != want[i]:
                a = np.frombuffer(got[i], np.float32); b = np.frombuffer(want[i], np.float32)
                bad.append((names[i], int((a != b).sum()), float(np.abs(a - b).max())))
        print(f"round {r}: seq rerun differs {seq_diff}; graph vs seq {bad}", flush=True)
        g.close() if hasattr(g, "close") else None


if __name__ == "__main__":
    main()
