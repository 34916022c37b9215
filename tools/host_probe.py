"""Host-path probe (lab tool): the bench's host_path token (Llama-7B Q4_0 layers on host buffers,
weights pinned) with several write-back masks, ms per token (x 32 / layers).
Usage: python tools/host_probe.py [layers]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "llama.kotlin_amd")]

import bench  # noqa: E402


def main():
    import numpy as np
    import torch
    import ggml_hip as G
    layers = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    G.load_library()
    T = G.GGMLType
    total = layers * sum(bench.alg_bytes(M, K) + 64 for (_, M, K) in bench.LAYER_MATS) + 4 * bench.HIDDEN + 64
    ga = G.GGMLGraphAllocator(device="host", defaultBufferSize=total)
    gen = torch.Generator(device=dev)
    gen.manual_seed(7)
    nodes, outs = [], []
    x = ga.allocateTensor(T.F32, [1, bench.HIDDEN], bufferId=0)
    ga.setTensorBytes(x, np.random.default_rng(1).standard_normal(bench.HIDDEN).astype(np.float32))
    act = {"h": x}
    for _ in range(layers):
        for grp in bench.CHAIN:
            for name in grp:
                M, K = next((m, k) for (n, m, k) in bench.LAYER_MATS if n == name)
                a = ga.allocateTensor(T.Q4_0, [K, M])
                w = torch.randn(M * K, generator=gen, device=dev) * 0.02
                ga.setTensorBytes(a, G.quantizeTensor(w, T.Q4_0).cpu().numpy())
                d = ga.allocateTensor(T.F32, [1, M])
                nodes.append((a, act[bench.X_OF[name]], d))
                outs.append(name == "down")
                if name in ("q", "o", "up", "down"):
                    act[{"q": "attn", "o": "h2", "up": "ffn", "down": "h"}[name]] = d
    for a, _, _ in nodes:
        G.weightsPin(ga, a)
    lay = 32 / layers
    dsts = []
    for a, b, d in nodes:
        d.op, d.src = G.GGMLOp.MUL_MAT, [a, b]
        dsts.append(d)
    be_mask = G.backend.writeBackMask(dsts, wholeGraph=True)
    last = [False] * (len(nodes) - 1) + [True]
    res = {"layers": layers}

    def timeit(fn, reps=20):
        fn()
        fn()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        return round((time.perf_counter() - t0) / reps * lay * 1e3, 3)

    for key, mask in (("last_only", last), ("down_outs", outs), ("backend_mask", be_mask), ("all", None)):
        g = G.ResidentGraph(ga, nodes, outputs=mask)
        res[key] = {"ms_per_token": timeit(g.compute), "d2h_per_token": int(g.transferBytes(False) * lay)}
        g.close()
    be = G.GGMLHipBackend(ga, wholeGraphs=True)
    cg = G.GGMLCGraph(dsts, ga)
    res["backend"] = {"ms_per_token": timeit(lambda: be.graphCompute(cg))}
    be.free()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
