"""Phase stamps of gemv_stream_kernel (lab tool): needs a lab build of liblk_hip.so whose stream
kernel holds s_memrealtime stamps per (workgroup, wave) in registers and stores them at exit —
S0 entry, S8 work count read, S9 node parameters resolved, S6 activation DMAs issued, S7 first weight unit issued, S5 prologue DMAs issued, S1 activation image landed (after the barrier), S2
activations in VGPRs, S3 first weight unit landed, S4 exit — and exports
lk_lab_stamps / lk_lab_stamps_clear. Usage: LK_HIP_LIB=<lab .so> python tools/stamp_probe.py
Prints per phase the median / max over waves of the time since the earliest entry (µs)."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "llama.kotlin_amd")]

import bench  # noqa: E402


def summarize(st, grid):
    import numpy as np
    a = np.array(st[: grid * 8 * 10], dtype=np.int64).reshape(grid, 8, 10)
    live = a[:, :, 0] > 0
    t0 = a[:, :, 0][live].min()
    rel = (a - t0) / 100.0  # 100 MHz ticks -> µs
    out = {}
    for k, name in enumerate(("entry", "x_landed", "x_in_vgprs", "unit0_landed", "exit", "issued", "x_issued", "unit0_issued", "work_count", "node_params")):
        v = rel[:, :, k][live & (a[:, :, k] > 0)]
        if v.size:
            out[name] = {"med": round(float(np.median(v)), 2), "p10": round(float(np.percentile(v, 10)), 2),
                         "max": round(float(v.max()), 2)}
    # per workgroup exit (last wave) spread
    ex = rel[:, :, 4].max(axis=1)
    out["wg_exit"] = {"min": round(float(ex.min()), 2), "med": round(float(np.median(ex)), 2), "max": round(float(ex.max()), 2)}
    # by XCD (workgroup b on XCD b % 8) and by workgroup range (plans: nodes hold contiguous ranges)
    out["exit_by_xcd"] = [round(float(np.median(ex[x::8])), 2) for x in range(8)]
    out["exit_by_range"] = [round(float(np.median(ex[r * grid // 16:(r + 1) * grid // 16])), 2) for r in range(16)]
    out["entry_by_xcd"] = [round(float(np.median(rel[x::8, :, 0])), 2) for x in range(8)]
    return out


def main():
    import torch
    import ggml_hip as G
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    G.load_library()
    lib = ctypes.CDLL(os.environ["LK_HIP_LIB"])
    buf = (ctypes.c_uint64 * (1024 * 8 * 10))()
    T = G.GGMLType
    s = torch.cuda.Stream(device=dev)
    res = {}
    for name, M, K, copies in (("q4_0_4096x4096", 4096, 4096, 48), ("q4_0_11008x4096", 11008, 4096, 16)):
        nb = M * K // 32 * 18
        g = G.GGMLGraphAllocator(device=str(dev), defaultBufferSize=16)
        wb, xb, db = g.addBuffer(copies * nb + 256), g.addBuffer(4 * K + 256), g.addBuffer(4 * M * copies + 256)
        src = torch.randn(M * K, device=dev) * 0.02
        for c in range(copies):
            g.buffers[wb][c * nb:(c + 1) * nb].copy_(G.quantizeTensor(src * (1 + 0.01 * c), T.Q4_0))
        g.buffers[xb][: 4 * K].copy_(torch.randn(K, device=dev).view(torch.uint8))
        nodes = [(G.GGMLTensor(T.Q4_0, [K, M], bufferId=wb, dataOffset=c * nb), G.GGMLTensor(T.F32, [1, K], bufferId=xb),
                  G.GGMLTensor(T.F32, [1, M], bufferId=db, dataOffset=4 * M * c)) for c in range(copies)]

        def run_all():
            for (a, b, d) in nodes:
                G.computeMatMul(g, None, a, b, d, stream=s)

        per, _ = bench._graph_time(torch, run_all, s, 10)
        lib.lk_lab_stamps_clear()
        torch.cuda.synchronize()
        with torch.cuda.stream(s):
            run_all()  # the stamps keep the last launch's (copy copies-1, after copies-1 others)
        torch.cuda.synchronize()
        lib.lk_lab_stamps(buf, len(buf))
        res[name] = {"graph_us": round(per / copies * 1e6, 2), "phases": summarize(list(buf), 256)}
        del g
    # one Llama-7B layer's 7 matrices in one grouped launch (8 distinct layers, stamps of the last)
    g = G.GGMLGraphAllocator(device=str(dev), defaultBufferSize=16)
    xs = {}
    for kind, n in bench.X_LEN.items():
        xs[kind] = G.GGMLTensor(T.F32, [1, n], bufferId=g.addBuffer(4 * n + 256))
        g.buffers[xs[kind].bufferId][: 4 * n].copy_(torch.randn(n, device=dev).view(torch.uint8))
    plans = []
    for _ in range(8):
        nodes = []
        for (nm, M, K) in bench.LAYER_MATS:
            nb = M * K // 32 * 18
            wb = g.addBuffer(nb + 256)
            g.buffers[wb][:nb].copy_(G.quantizeTensor(torch.randn(M * K, device=dev) * 0.02, T.Q4_0))
            d = G.GGMLTensor(T.F32, [1, M], bufferId=g.addBuffer(4 * M + 256))
            nodes.append((G.GGMLTensor(T.Q4_0, [K, M], bufferId=wb), xs[bench.X_OF[nm]], d))
        plans.append(G.MulMatPlan(g, nodes))

    def run_layers():
        for p in plans:
            p.launch(stream=s)

    per, _ = bench._graph_time(torch, run_layers, s, 10)
    lib.lk_lab_stamps_clear()
    torch.cuda.synchronize()
    with torch.cuda.stream(s):
        run_layers()
    torch.cuda.synchronize()
    lib.lk_lab_stamps(buf, len(buf))
    res["layer"] = {"graph_us": round(per / 8 * 1e6, 2), "phases": summarize(list(buf), 256)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
