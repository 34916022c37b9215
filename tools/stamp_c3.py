"""Timeline of gemm_skinny_pair_kernel on C3 (lab tool): needs a lab build whose pair kernel keeps
per-wave s_memrealtime stamps — S0 entry, S1 activation split done, S2 fragments in VGPRs (loop
start), S3 first unit landed, S4 loop end, S5 exit (after the fused reduction) — and per-wave sums
over its units of the data wait, the compute (LDS reads, decode, MFMAs, refill) and the pair
hand-off, exported by lk_lab_stamps / lk_lab_stamps_clear.
Usage: LK_HIP_LIB=<lab .so> python tools/stamp_c3.py"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "llama.kotlin_amd")]

import bench  # noqa: E402


def main():
    import numpy as np
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
    for qt, name in ((T.Q4_0, "c3_q4_0"), (T.Q4_1, "c3_q4_1")):
        M, K, N, copies = 11008, 4096, 32, 16
        nb = M * K // 32 * G.GGMLType(qt).byteSize
        g = G.GGMLGraphAllocator(device=str(dev), defaultBufferSize=16)
        wb, xb, db = g.addBuffer(copies * nb + 256), g.addBuffer(4 * K * N + 256), g.addBuffer(4 * M * N * copies + 256)
        src = torch.randn(M * K, device=dev) * 0.02
        for c in range(copies):
            g.buffers[wb][c * nb:(c + 1) * nb].copy_(G.quantizeTensor(src * (1 + 0.01 * c), qt))
        g.buffers[xb][: 4 * K * N].copy_(torch.randn(K * N, device=dev).view(torch.uint8))
        nodes = [(G.GGMLTensor(qt, [K, M], bufferId=wb, dataOffset=c * nb), G.GGMLTensor(T.F32, [N, K], bufferId=xb),
                  G.GGMLTensor(T.F32, [N, M], bufferId=db, dataOffset=4 * M * N * c)) for c in range(copies)]

        def run_all():
            for (a, b, d) in nodes:
                G.computeMatMul(g, None, a, b, d, stream=s)

        per, _ = bench._graph_time(torch, run_all, s, 10)
        lib.lk_lab_stamps_clear()
        torch.cuda.synchronize()
        with torch.cuda.stream(s):
            run_all()
        torch.cuda.synchronize()
        lib.lk_lab_stamps(buf, len(buf))
        a = np.array(list(buf), dtype=np.int64).reshape(1024, 8, 10)
        live = a[:, :, 0] > 0
        t0 = a[:, :, 0][live].min()
        out = {"graph_us": round(per / copies * 1e6, 2), "workgroups": int(live.any(axis=1).sum())}
        for k, ph in enumerate(("entry", "split_done", "loop_start", "unit0_landed", "loop_end", "exit")):
            v = (a[:, :, k][live] - t0) / 100.0
            out[ph] = {"med": round(float(np.median(v)), 2), "p10": round(float(np.percentile(v, 10)), 2),
                       "max": round(float(v.max()), 2)}
        units = a[:, :, 9][live]
        for k, ph in ((6, "wait_per_unit"), (7, "compute_per_unit"), (8, "handoff_per_unit")):
            v = a[:, :, k][live] / 100.0 / np.maximum(units, 1)
            out[ph] = round(float(np.median(v)), 3)
        out["units_med"] = float(np.median(units))
        for h in (0, 1):
            v = a[:, 4 * h:4 * h + 4, :][live[:, 4 * h:4 * h + 4]]
            u = np.maximum(v[:, 9], 1)
            out[f"half{h}"] = {"wait": round(float(np.median(v[:, 6] / 100.0 / u)), 3),
                               "compute": round(float(np.median(v[:, 7] / 100.0 / u)), 3),
                               "handoff": round(float(np.median(v[:, 8] / 100.0 / u)), 3)}
        res[name] = out
        del g
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
