"""Lab probe (lab build -DLK_PF=<units>, `lk_plan_prefetch_next`): the decode chain (32 Llama-7B
layers, {q,k,v} -> o -> {gate,up} -> down, one plan per stage, captured in a HIP graph) with and
without each plan's last launch prefetching its successor's first weight units per wave. Rounds
alternate the two forms on one box; outputs must be bit-equal (prefetch only reads).
Usage: LK_HIP_LIB=<lab .so> python tools/pf_probe.py [rounds]"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "llama.kotlin_amd")]

import bench  # noqa: E402


def main():
    import torch
    import ggml_hip as G
    from ggml_hip import _lib
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    L = _lib.load()
    link = getattr(L, "lk_plan_prefetch_next", None)
    if link is None:
        print(json.dumps({"error": "library has no lk_plan_prefetch_next (build with -DLK_PF=<units>)"}))
        sys.exit(1)
    link.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    T = G.GGMLType
    layers = 32
    ga = G.GGMLGraphAllocator(device=str(dev), defaultBufferSize=16)
    wbytes = sum(layers * ((M * K // 32 * 18 + 255) // 256 * 256) for (_, M, K) in bench.LAYER_MATS)
    wbuf = ga.addBuffer(wbytes + 256)
    w, off = [], 0
    for _ in range(layers):
        d = {}
        for (name, M, K) in bench.LAYER_MATS:
            t = G.GGMLTensor(T.Q4_0, [K, M], bufferId=wbuf, dataOffset=off)
            ga.buffers[wbuf][off:off + M * K // 32 * 18].copy_(G.quantizeTensor(torch.randn(M * K, device=dev) * 0.02, T.Q4_0))
            off += (M * K // 32 * 18 + 255) // 256 * 256
            d[name] = t
        w.append(d)
    src = {"q": "x", "k": "x", "v": "x", "o": "q", "gate": "o", "up": "o", "down": "up"}
    act = ga.addBuffer(4 * bench.HIDDEN + layers * sum((4 * M + 255) // 256 * 256 for (_, M, _) in bench.LAYER_MATS) + 256)
    t, o = {"x": G.GGMLTensor(T.F32, [1, bench.HIDDEN], bufferId=act, dataOffset=0)}, 4 * bench.HIDDEN
    for Ly in range(layers):
        for (name, M, _) in bench.LAYER_MATS:
            t[(Ly, name)] = G.GGMLTensor(T.F32, [1, M], bufferId=act, dataOffset=o)
            o += (4 * M + 255) // 256 * 256
    ga.buffers[act][: 4 * bench.HIDDEN].copy_((torch.randn(bench.HIDDEN, device=dev)).view(torch.uint8))
    groups = [("q", "k", "v"), ("o",), ("gate", "up"), ("down",)]
    plans = []
    for Ly in range(layers):
        for grp in groups:
            nodes = []
            for name in grp:
                s = src[name]
                b = (t["x"] if Ly == 0 else t[(Ly - 1, "down")]) if s == "x" else t[(Ly, s)]
                nodes.append((w[Ly][name], b, t[(Ly, name)]))
            plans.append(G.MulMatPlan(ga, nodes))
    st = torch.cuda.Stream(device=dev)

    def token():
        for p in plans:
            p.launch(stream=st)

    def set_links(on):
        for i, p in enumerate(plans):
            nxt = plans[(i + 1) % len(plans)] if on else None
            _lib.check(link(p._handle, nxt._handle if nxt is not None else None))

    out = {"layers": layers, "pf_units": os.environ.get("LK_PF_UNITS", "?")}
    res = {False: [], True: []}
    outputs = {}
    for r in range(rounds):
        for on in (False, True):
            set_links(on)  # before the capture: the launches' arguments are baked into the graph
            per, _ = bench._graph_time(torch, token, st, 20)
            res[on].append(round(per * 1e6, 1))
            outputs[on] = bytes(ga.tensorBytes(t[(layers - 1, "down")]).cpu().numpy().tobytes())
    out["us_per_token_plain"] = res[False]
    out["us_per_token_prefetch"] = res[True]
    out["tok_s_plain"] = round(1e6 / min(res[False]), 1)
    out["tok_s_prefetch"] = round(1e6 / min(res[True]), 1)
    out["bit_equal"] = outputs[False] == outputs[True]
    set_links(False)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
