"""Where a chain plan's stage transitions go (lab build: tools/build_lab.sh cstamps -DLK_LAB_CHAIN_STAMPS).
The decode chain (Llama-7B layers, {q,k,v} -> o -> {gate,up} -> down, one chain plan = one launch)
launched warm, then once with stamps: per (workgroup, segment) wave 0 records segment start, stores
drained, released from the grid barrier, image ready, x in VGPRs, first unit landed and done. For
each stage kind, medians over stages of (median / max over workgroups) µs after the previous stage's
last workgroup was done (T0). Usage: LK_HIP_LIB=<lab .so> python tools/chain_stamps.py [layers]"""
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
    layers = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    G.load_library()
    lib = ctypes.CDLL(os.environ["LK_HIP_LIB"])
    T = G.GGMLType
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
    stage_of = {"q": 0, "k": 0, "v": 0, "o": 1, "gate": 2, "up": 2, "down": 3}
    act = ga.addBuffer(4 * bench.HIDDEN + layers * sum((4 * M + 255) // 256 * 256 for (_, M, _) in bench.LAYER_MATS) + 256)
    t, o = {"x": G.GGMLTensor(T.F32, [1, bench.HIDDEN], bufferId=act, dataOffset=0)}, 4 * bench.HIDDEN
    for Ly in range(layers):
        for (name, M, _) in bench.LAYER_MATS:
            t[(Ly, name)] = G.GGMLTensor(T.F32, [1, M], bufferId=act, dataOffset=o)
            o += (4 * M + 255) // 256 * 256
    ga.buffers[act][: 4 * bench.HIDDEN].copy_(torch.randn(bench.HIDDEN, device=dev).view(torch.uint8))
    nodes, stages = [], []
    for Ly in range(layers):
        for (name, M, K) in bench.LAYER_MATS:
            s = src[name]
            b = (t["x"] if Ly == 0 else t[(Ly - 1, "down")]) if s == "x" else t[(Ly, s)]
            nodes.append((w[Ly][name], b, t[(Ly, name)]))
            stages.append(4 * Ly + stage_of[name])
    chain = G.MulMatPlan(ga, nodes, stages=stages)
    st = torch.cuda.Stream(device=dev)
    kinds = ["q+k+v", "o", "gate+up", "down"]
    buf = (ctypes.c_uint64 * (256 * 256 * 8))()
    reps = []
    for rep in range(3):
        for _ in range(3):
            chain.launch(stream=st)
        torch.cuda.synchronize()
        lib.lk_lab_chain_stamps_clear()
        torch.cuda.synchronize()
        chain.launch(stream=st)
        torch.cuda.synchronize()
        lib.lk_lab_chain_stamps(buf, len(buf))
        a = np.array(list(buf), dtype=np.int64).reshape(256, 256, 8)
        live_wg = np.nonzero(a[:, 0, 0] > 0)[0]
        # stage of each (wg, segment): the running barrier count (slot 7 = barrier number, 0 = none)
        per_stage = {}
        for g in live_wg:
            cur = 0
            for si in range(256):
                if a[g, si, 0] == 0:
                    break
                if a[g, si, 7] > 0:
                    cur = int(a[g, si, 7])
                per_stage.setdefault(cur, []).append(a[g, si])
        t_first = min(int(r[0]) for r in per_stage[0])
        res = {k: [] for k in kinds}
        prev_done = None
        for sidx in sorted(per_stage):
            rows = np.array(per_stage[sidx])
            done = rows[:, 6].max()
            if prev_done is not None:
                first = rows[rows[:, 7] > 0] if (rows[:, 7] > 0).any() else rows

                def rel(col, fn, r=first):
                    v = r[:, col]
                    v = v[v > 0]
                    return round(float(fn(v) - prev_done) / 100, 2) if len(v) else None
                res[kinds[sidx % 4]].append({
                    "drained_med": rel(1, np.median), "drained_max": rel(1, np.max),
                    "released_min": rel(2, np.min), "released_med": rel(2, np.median), "released_max": rel(2, np.max),
                    "image_med": rel(3, np.median), "x_med": rel(4, np.median), "u0_med": rel(5, np.median),
                    "u0_max": rel(5, np.max), "done_med": rel(6, np.median, rows), "done_max": rel(6, np.max, rows)})
            prev_done = done
        summ = {}
        for k, lst in res.items():
            if not lst:
                continue
            summ[k] = {f: round(float(np.median([d[f] for d in lst if d[f] is not None])), 2) for f in lst[0]}
            summ[k]["n"] = len(lst)
        reps.append({"token_us": round(float(prev_done - t_first) / 100, 2), "per_layer_us": round(float(prev_done - t_first) / 100 / layers, 2),
                     "stages": summ})
    chain.close()
    print(json.dumps({"layers": layers, "reps": reps}), flush=True)


if __name__ == "__main__":
    main()
