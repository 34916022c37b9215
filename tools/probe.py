"""A/B probe of the kernels the bench times, one JSON line per run (for comparing builds of
liblk_hip.so: LK_HIP_LIB=<path> python tools/probe.py [sections]).

Sections (default: all):
  layer    one grouped launch of a Llama-7B layer's 7 Q4_0 matrices, 8 distinct layers (> MALL)
  chain    the dependent decode order {q,k,v} -> o -> {gate,up} -> down over the same layers
  n1       Q4_0 4096^2 / 11008x4096 / 4096x11008 single launches at batch 1 (rotating copies)
  c3       Q4_0 / Q4_1 11008x4096 at N = 32
  c5       Q4_0 4096^2 at N = 512
  c1       F32 512^3 (the general F32 path on the f32 MFMA)
  skinny   Q4_0 11008x4096 at N = 8 and 16 (gemm_skinny_kernel)
Every time is the mean over a HIP-graph replay (bench._graph_time)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "llama.kotlin_amd")]

import bench  # noqa: E402


def main():
    import torch
    import ggml_hip as G
    want = set(sys.argv[1:]) or {"layer", "chain", "n1", "c3", "c5", "c1"}
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    G.load_library()
    T = G.GGMLType
    out = {"lib": os.environ.get("LK_HIP_LIB", "default")}
    s = torch.cuda.Stream(device=dev)
    if want & {"layer", "chain"}:
        layers = 8
        g = G.GGMLGraphAllocator(device=str(dev), defaultBufferSize=16)
        xs = {}
        for kind, n in bench.X_LEN.items():
            xs[kind] = G.GGMLTensor(T.F32, [1, n], bufferId=g.addBuffer(4 * n + 256))
            g.buffers[xs[kind].bufferId][: 4 * n].copy_(torch.randn(n, device=dev).view(torch.uint8))
        by_layer, lbytes = [], 0
        for _ in range(layers):
            n = {}
            for (name, M, K) in bench.LAYER_MATS:
                nb = M * K // 32 * 18
                wb = g.addBuffer(nb + 256)
                g.buffers[wb][:nb].copy_(G.quantizeTensor(torch.randn(M * K, device=dev) * 0.02, T.Q4_0))
                d = G.GGMLTensor(T.F32, [1, M], bufferId=g.addBuffer(4 * M + 256))
                n[name] = (G.GGMLTensor(T.Q4_0, [K, M], bufferId=wb), xs[bench.X_OF[name]], d)
                lbytes += bench.alg_bytes(M, K)
            by_layer.append(n)
        lbytes /= layers
        for sec, groups in (("layer", [tuple(m for (m, _, _) in bench.LAYER_MATS)]), ("chain", bench.CHAIN)):
            if sec not in want:
                continue
            plans = [[G.MulMatPlan(g, [n[k] for k in grp]) for grp in groups] for n in by_layer]

            def run_all():
                for lp in plans:
                    for p in lp:
                        p.launch(stream=s)

            per, _ = bench._graph_time(torch, run_all, s, 20)
            per /= layers
            out[sec] = {"us_per_layer": round(per * 1e6, 2), "frac": round(lbytes / per / 1e9 / 8000, 4),
                        "tok_s_32": round(1 / (32 * per), 1)}
        del g
    if "n1" in want:
        for name, M, K, copies in (("q4_0_4096x4096", 4096, 4096, 48), ("q4_0_11008x4096", 11008, 4096, 16),
                                   ("q4_0_4096x11008", 4096, 11008, 16)):
            out["n1_" + name] = _single(torch, G, dev, s, T.Q4_0, M, K, 1, copies)
    if "c3" in want:
        out["c3_q4_0"] = _single(torch, G, dev, s, T.Q4_0, 11008, 4096, 32, 16)
        out["c3_q4_1"] = _single(torch, G, dev, s, T.Q4_1, 11008, 4096, 32, 16)
    if "c5" in want:
        out["c5_q4_0"] = _single(torch, G, dev, s, T.Q4_0, 4096, 4096, 512, 32)
    if "skinny" in want:
        out["q4_0_n8"] = _single(torch, G, dev, s, T.Q4_0, 11008, 4096, 8, 16)
        out["q4_0_n16"] = _single(torch, G, dev, s, T.Q4_0, 11008, 4096, 16, 16)
    if "skinny41" in want:
        out["q4_1_n16"] = _single(torch, G, dev, s, T.Q4_1, 11008, 4096, 16, 16)
    if "c1" in want:
        out["c1_f32"] = _single(torch, G, dev, s, T.F32, 512, 512, 512, 4)
    if "down32" in want:
        out["q4_0_4096x11008_n32"] = _single(torch, G, dev, s, T.Q4_0, 4096, 11008, 32, 16)
    if "q80" in want:
        out["q8_0_n32"] = _single(torch, G, dev, s, T.Q8_0, 11008, 4096, 32, 8)
    if "q4k" in want:
        out["q4_k_n32"] = _q4k(torch, G, dev, s, 11008, 4096, 32, 16)
    print(json.dumps(out), flush=True)


def _single(torch, G, dev, s, qt, M, K, N, copies):
    T = G.GGMLType
    nb = M * K * 4 if qt == T.F32 else M * K // 32 * G.GGMLType(qt).byteSize
    g = G.GGMLGraphAllocator(device=str(dev), defaultBufferSize=16)
    wb, xb, db = g.addBuffer(copies * nb + 256), g.addBuffer(4 * K * N + 256), g.addBuffer(4 * M * N * copies + 256)
    src = torch.randn(M * K, device=dev) * 0.02
    for c in range(copies):
        g.buffers[wb][c * nb:(c + 1) * nb].copy_((src * (1 + 0.01 * c)).view(torch.uint8) if qt == T.F32
                                                 else G.quantizeTensor(src * (1 + 0.01 * c), qt))
    g.buffers[xb][: 4 * K * N].copy_(torch.randn(K * N, device=dev).view(torch.uint8))
    nodes = [(G.GGMLTensor(qt, [K, M], bufferId=wb, dataOffset=c * nb), G.GGMLTensor(T.F32, [N, K], bufferId=xb),
              G.GGMLTensor(T.F32, [N, M], bufferId=db, dataOffset=4 * M * N * c)) for c in range(copies)]

    def run_all():
        for (a, b, d) in nodes:
            G.computeMatMul(g, None, a, b, d, stream=s)

    per, _ = bench._graph_time(torch, run_all, s, 10)
    per /= copies
    nbytes = nb + 4 * K * N + 4 * M * N
    del g
    return {"us": round(per * 1e6, 2), "frac": round(nbytes / per / 1e9 / 8000, 4),
            "tflops": round(2 * M * N * K / per / 1e12, 1)}


def _q4k(torch, G, dev, s, M, K, N, copies):
    """Q4_K x F32 (bench.next_rows' synthetic super-blocks: random code bytes, d = 0.01, dmin = 0.001)."""
    T = G.GGMLType
    bb, so, _ = bench.KQ_BLOCK["Q4_K"]
    nblk = M * K // 256
    nb = nblk * bb
    g = G.GGMLGraphAllocator(device=str(dev), defaultBufferSize=16)
    wb, xb, db = g.addBuffer(copies * nb + 256), g.addBuffer(4 * K * N + 256), g.addBuffer(4 * M * N * copies + 256)
    w = g.buffers[wb][: copies * nb].view(copies * nblk, bb)
    w.copy_(torch.randint(0, 256, w.shape, dtype=torch.uint8, device=dev))
    w[:, so:so + 4].copy_(torch.tensor([0.01, 0.001], dtype=torch.float16).view(torch.uint8).to(dev))
    g.buffers[xb][: 4 * K * N].copy_(torch.randn(K * N, device=dev).view(torch.uint8))
    nodes = [(G.GGMLTensor(T.Q4_K, [K, M], bufferId=wb, dataOffset=c * nb), G.GGMLTensor(T.F32, [N, K], bufferId=xb),
              G.GGMLTensor(T.F32, [N, M], bufferId=db, dataOffset=4 * M * N * c)) for c in range(copies)]

    def run_all():
        for (a, b, d) in nodes:
            G.computeMatMul(g, None, a, b, d, stream=s)

    per, _ = bench._graph_time(torch, run_all, s, 10)
    per /= copies
    del g
    return {"us": round(per * 1e6, 2), "frac": round((nb + 4 * K * N + 4 * M * N) / per / 1e9 / 8000, 4),
            "tflops": round(2 * M * N * K / per / 1e12, 1)}


if __name__ == "__main__":
    main()
