"""Timelines of the split-K kernels (lab tool): needs a lab build with -DLK_LAB_STAMPS
(tools/build_lab.sh stamps -DLK_LAB_STAMPS), which keeps per-wave s_memrealtime stamps.
Usage: LK_HIP_LIB=<lab .so> [LK_KPART_OFF=1] python tools/stamp_kpart.py [N ...]   (default N = 32 and 8)
gemm_kpart_kernel slots: 0 entry, 1 activations in registers, 2 loop start, 3 loop end, 4 exit,
5 ring wait / 6 compute / 7 tile sum (sums over units), 8 units. gemm_skinny_pair_kernel (LK_KPART_OFF=1):
0 entry, 2 loop start, 3 loop end, 4 exit, 5 arrivals done, 6 after the fix-up barrier, 7 tiles
this stream was last for, 8 units."""
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
    ns = [int(a) for a in sys.argv[1:]] or [32, 8]
    for N in ns:
        for qt, qn in ((T.Q4_0, "q4_0"), (T.Q4_1, "q4_1")):
            M, K, copies = 11008, 4096, 16
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
                G.computeMatMul(g, None, *nodes[0], stream=s)
            torch.cuda.synchronize()
            lib.lk_lab_stamps(buf, len(buf))
            a = np.array(list(buf), dtype=np.int64).reshape(1024, 8, 10)
            live = a[:, :, 0] > 0
            t0 = a[:, :, 0][live].min()
            out = {"graph_us": round(per / copies * 1e6, 2), "workgroups": int(live.any(axis=1).sum())}
            pair = os.environ.get("LK_KPART_OFF") == "1"
            phases = ((0, "entry"), (2, "loop_start"), (3, "loop_end"), (5, "arrived"), (6, "fixup_barrier"), (4, "exit")) if pair \
                else ((0, "entry"), (1, "x_in_regs"), (2, "loop_start"), (3, "loop_end"), (4, "exit"))
            for k, ph in phases:
                sel = live & (a[:, :, k] > 0)
                if not sel.any():
                    continue
                v = (a[:, :, k][sel] - t0) / 100.0
                out[ph] = {"med": round(float(np.median(v)), 2), "p10": round(float(np.percentile(v, 10)), 2),
                           "max": round(float(v.max()), 2)}
            units = a[:, :, 8][live]
            if pair:
                out["last_tiles_per_stream"] = {"med": float(np.median(a[:, :4, 7][live[:, :4]])),
                                                "max": float(a[:, :4, 7][live[:, :4]].max())}
            else:
                for k, ph in ((5, "wait_per_unit"), (6, "compute_per_unit"), (7, "tilesum_per_unit")):
                    v = a[:, :, k][live] / 100.0 / np.maximum(units, 1)
                    out[ph] = round(float(np.median(v)), 3)
            out["units_med"] = float(np.median(units))
            if not pair:  # per workgroup: who ends the loop late, and why (entry, start or compute)
                wgs = np.nonzero(live.any(axis=1))[0]
                grid = (len(wgs) + 7) // 8 * 8
                rows = []
                for b in wgs:
                    lv = live[b]
                    rows.append({"bid": int(b), "xcd": int(b % 8), "task": int((b % 8) * (grid // 8) + b // 8),
                                 "entry": round(float((a[b, lv, 0].min() - t0) / 100), 2),
                                 "loop_start": round(float((a[b, lv, 2].max() - t0) / 100), 2),
                                 "loop_end": round(float((a[b, lv, 3].max() - t0) / 100), 2),
                                 "comp_per_unit": round(float(np.median(a[b, lv, 6] / np.maximum(a[b, lv, 8], 1))) / 100, 3),
                                 "wait_per_unit": round(float(np.median(a[b, lv, 5] / np.maximum(a[b, lv, 8], 1))) / 100, 3),
                                 "red_per_unit": round(float(np.median(a[b, lv, 7] / np.maximum(a[b, lv, 8], 1))) / 100, 3)})
                rows.sort(key=lambda r: -r["loop_end"])
                out["slowest_wgs"] = rows[:10]
                b = rows[0]["bid"]
                out["slowest_wg_waves"] = [{"wave": w, "loop_start": round(float((a[b, w, 2] - t0) / 100), 2),
                                            "loop_end": round(float((a[b, w, 3] - t0) / 100), 2),
                                            "wait": round(float(a[b, w, 5] / 100), 2), "comp": round(float(a[b, w, 6] / 100), 2),
                                            "red": round(float(a[b, w, 7] / 100), 2), "units": int(a[b, w, 8])}
                                           for w in range(8) if live[b, w]]
                out["fastest_wgs"] = rows[-3:]
                out["loop_end_by_xcd"] = {x: round(float(np.median([r["loop_end"] for r in rows if r["xcd"] == x])), 2)
                                          for x in range(8)}
            res[f"{qn}_11008x4096_n{N}"] = out
            del g
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
