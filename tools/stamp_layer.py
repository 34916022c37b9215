"""Where a grouped launch's tail comes from (lab tool; build with tools/build_lab.sh stamps
-DLK_LAB_STAMPS): one Llama-7B layer (7 Q4_0 matrices, one MulMatPlan = the bench's layer launch)
and the decode chain's four stage plans, each launched warm and stamped. Per XCD (workgroup
blockIdx % 8, the observed round-robin dispatch): median entry, median and last exit (µs after the
launch's first entry), and the units its waves ran. Usage: LK_HIP_LIB=<lab .so> python tools/stamp_layer.py"""
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
    g = G.GGMLGraphAllocator(device=str(dev), defaultBufferSize=16)
    xs = {}
    for kind, n in bench.X_LEN.items():
        xs[kind] = G.GGMLTensor(T.F32, [1, n], bufferId=g.addBuffer(4 * n + 256))
        g.buffers[xs[kind].bufferId][: 4 * n].copy_(torch.randn(n, device=dev).view(torch.uint8))
    nodes = {}
    for (name, M, K) in bench.LAYER_MATS:
        nb = M * K // 32 * 18
        wb = g.addBuffer(nb + 256)
        g.buffers[wb][:nb].copy_(G.quantizeTensor(torch.randn(M * K, device=dev) * 0.02, T.Q4_0))
        d = G.GGMLTensor(T.F32, [1, M], bufferId=g.addBuffer(4 * M + 256))
        nodes[name] = (G.GGMLTensor(T.Q4_0, [K, M], bufferId=wb), xs[bench.X_OF[name]], d)
    s = torch.cuda.Stream(device=dev)
    forms = {"layer": [tuple(m for (m, _, _) in bench.LAYER_MATS)]}
    for i, grp in enumerate(bench.CHAIN):
        forms["stage_" + "+".join(grp)] = [grp]
    out = {}
    # back to back: a token's four stage plans in stream order, no synchronisation between them; the
    # stamps are the last launch's (every launch overwrites the slots of its workgroups)
    chain = [G.MulMatPlan(g, [nodes[k] for k in grp]) for grp in bench.CHAIN]
    for last in range(4):
        reps = []
        for rep in range(3):
            for _ in range(3):
                for p in chain:
                    p.launch(stream=s)
            torch.cuda.synchronize()
            lib.lk_lab_stamps_clear()
            torch.cuda.synchronize()
            for _ in range(2):
                for p in chain:
                    p.launch(stream=s)
            for p in chain[: last + 1]:
                p.launch(stream=s)
            torch.cuda.synchronize()
            lib.lk_lab_stamps(buf, len(buf))
            st = np.array(list(buf), dtype=np.int64).reshape(1024, 8, 10)
            live = st[:, :, 0] > 0
            wgs = np.nonzero(live.any(axis=1))[0]
            t0 = st[:, :, 0][live].min()
            entry = {w: (st[w, live[w], 0].min() - t0) / 100 for w in wgs}
            exit_ = {w: (st[w, live[w], 4].max() - t0) / 100 for w in wgs}
            by = {x: {"entry_med": round(float(np.median([entry[w] for w in wgs if w % 8 == x])), 2),
                      "exit_med": round(float(np.median([exit_[w] for w in wgs if w % 8 == x])), 2)} for x in range(8)}
            ex = np.array(list(exit_.values()))
            units = {w: int(st[w, live[w], 8].sum()) for w in wgs}
            late = sorted(wgs, key=lambda w: -exit_[w])[:8]
            # within a workgroup: its last wave's exit against its waves' mean and earliest exit
            wex = {w: (st[w, live[w], 4] - t0) / 100 for w in wgs}
            intra = np.array([wex[w].max() - wex[w].mean() for w in wgs])
            intra_first = np.array([wex[w].max() - wex[w].min() for w in wgs])
            reps.append({"exit_med": round(float(np.median(ex)), 2), "exit_max": round(float(ex.max()), 2), "by_xcd": by,
                         "latest": [[int(w), round(float(exit_[w]), 2), round(float(entry[w]), 2), units[w]] for w in late],
                         "intra_wg_last_minus_mean_med": round(float(np.median(intra)), 2),
                         "intra_wg_last_minus_first_med": round(float(np.median(intra_first)), 2),
                         "latest_wg_last_minus_mean": [round(float(wex[w].max() - wex[w].mean()), 2) for w in late],
                         "units_med": int(np.median(list(units.values())))})
        out["b2b_" + "+".join(bench.CHAIN[last])] = reps
    for p in chain:
        p.close()
    for fname, groups in forms.items():
        plan = G.MulMatPlan(g, [nodes[k] for k in groups[0]])
        reps = []
        for rep in range(3):
            for _ in range(3):
                plan.launch(stream=s)
            torch.cuda.synchronize()
            lib.lk_lab_stamps_clear()
            torch.cuda.synchronize()
            plan.launch(stream=s)
            torch.cuda.synchronize()
            lib.lk_lab_stamps(buf, len(buf))
            st = np.array(list(buf), dtype=np.int64).reshape(1024, 8, 10)
            live = st[:, :, 0] > 0
            wgs = np.nonzero(live.any(axis=1))[0]
            t0 = st[:, :, 0][live].min()
            entry = {w: (st[w, live[w], 0].min() - t0) / 100 for w in wgs}
            exit_ = {w: (st[w, live[w], 4].max() - t0) / 100 for w in wgs}
            units = {w: int(st[w, live[w], 8].sum()) for w in wgs}
            by = {}
            for x in range(8):
                ws = [w for w in wgs if w % 8 == x]
                if not ws:
                    continue
                by[x] = {"entry_med": round(float(np.median([entry[w] for w in ws])), 2),
                         "exit_med": round(float(np.median([exit_[w] for w in ws])), 2),
                         "exit_max": round(float(max(exit_[w] for w in ws)), 2),
                         "units": int(sum(units[w] for w in ws))}
            ex = np.array(list(exit_.values()))
            reps.append({"workgroups": int(len(wgs)), "exit_med": round(float(np.median(ex)), 2),
                         "exit_p90": round(float(np.percentile(ex, 90)), 2), "exit_max": round(float(ex.max()), 2),
                         "by_xcd": by})
        out[fname] = reps
        plan.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
