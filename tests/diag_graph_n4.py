"""Lab diagnostic (not collected by pytest): test_graph_gpu.py::test_layer_graph_equals_sequential[4]
after the GPU parity tests (in-process, as in the full suite). Reports which nodes' graph bytes
differ from the node-by-node bytes, and each side's error against the oracle for those nodes."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [HERE, ROOT, os.path.join(ROOT, "llama.kotlin_amd"), os.path.join(ROOT, "oracle")]


def main():
    import pytest
    if len(sys.argv) > 1:
        pytest.main(["-q", "-m", "gpu", "-x", "-p", "no:cacheprovider"] + sys.argv[1:])
    import torch
    import oracle as O
    import ggml_hip as G
    from test_graph_gpu import _layer, _sequential
    O.lib()
    G.load_library()
    torch.cuda.set_device(0)
    names = ["q", "k", "v", "o", "g", "u", "d"]
    for r in range(3):
        for N in (1, 4):
            ga = G.GGMLGraphAllocator(device="host", defaultBufferSize=1 << 20)
            x, nodes = _layer(ga, O, N=N)
            want = _sequential(ga, nodes)
            for _, _, d in nodes:
                ga.setTensorBytes(d, np.zeros(4 * d.ne[0] * d.ne[1], np.uint8))
            g = G.ResidentGraph(ga, nodes)
            g.compute()
            got = [bytes(ga.tensorBytes(d)) for _, _, d in nodes]
            for i in range(7):
                if got[i] != want[i]:
                    a, b, dd = nodes[i]
                    ref = np.frombuffer(bytes(ga.tensorBytes(dd)), np.float32)
                    gg = np.frombuffer(got[i], np.float32); ww = np.frombuffer(want[i], np.float32)
                    # oracle on the node's own inputs as the graph saw them (host bytes now hold graph outputs)
                    ob = O.compute_mat_mul(ga, a, b, dd) if hasattr(O, "compute_mat_mul") else None
                    print(f"r{r} N={N} node {names[i]}: {int((gg != ww).sum())} of {gg.size} differ; "
                          f"max|got-want| {float(np.abs(gg - ww).max()):.3e}; got nan {int(np.isnan(gg).sum())}, want nan {int(np.isnan(ww).sum())}; "
                          f"got zeros {int((gg == 0).sum())}, want zeros {int((ww == 0).sum())}", flush=True)
            print(f"r{r} N={N} done", flush=True)


if __name__ == "__main__":
    main()
