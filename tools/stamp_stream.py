"""Entry / exit of gemv_stream_kernel's workgroups against blockIdx (lab tool): needs a lab build
with -DLK_LAB_STAMPS (tools/build_lab.sh stamps -DLK_LAB_STAMPS). One computeMatMul of a Q4_0
M x K matrix at N = 1; prints, per group of 16 consecutive workgroups, the median entry and the
last wave's exit (µs after the earliest entry), and the units per wave.
Usage: LK_HIP_LIB=<lab .so> python tools/stamp_stream.py [M K]"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "llama.kotlin_amd")]


def main():
    import numpy as np
    import torch
    import ggml_hip as G
    M, K = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (4096, 4096)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    G.load_library()
    lib = ctypes.CDLL(os.environ["LK_HIP_LIB"])
    buf = (ctypes.c_uint64 * (1024 * 8 * 10))()
    T = G.GGMLType
    nb = M * K // 32 * 18
    g = G.GGMLGraphAllocator(device=str(dev), defaultBufferSize=16)
    wb, xb, db = g.addBuffer(nb + 256), g.addBuffer(4 * K + 256), g.addBuffer(4 * M + 256)
    g.buffers[wb][:nb].copy_(G.quantizeTensor(torch.randn(M * K, device=dev) * 0.02, T.Q4_0))
    g.buffers[xb][: 4 * K].copy_(torch.randn(K, device=dev).view(torch.uint8))
    a, b, d = G.GGMLTensor(T.Q4_0, [K, M], bufferId=wb), G.GGMLTensor(T.F32, [1, K], bufferId=xb), G.GGMLTensor(T.F32, [1, M], bufferId=db)
    s = torch.cuda.Stream(device=dev)
    out = {}
    for rep in range(3):
        for _ in range(3):
            G.computeMatMul(g, None, a, b, d, stream=s)
        torch.cuda.synchronize()
        lib.lk_lab_stamps_clear()
        torch.cuda.synchronize()
        G.computeMatMul(g, None, a, b, d, stream=s)
        torch.cuda.synchronize()
        lib.lk_lab_stamps(buf, len(buf))
        st = np.array(list(buf), dtype=np.int64).reshape(1024, 8, 10)
        live = st[:, :, 0] > 0
        wgs = np.nonzero(live.any(axis=1))[0]
        t0 = st[:, :, 0][live].min()
        entry = np.array([(st[w, live[w], 0].min() - t0) / 100 for w in wgs])
        exit_ = np.array([(st[w, live[w], 4].max() - t0) / 100 for w in wgs])
        units = np.array([st[w, live[w], 8].max() for w in wgs])
        # per-wave phases (slots 1-3, 5, 6 of the stream kernel's lab build): median over waves,
        # µs after the earliest entry and after the wave's own entry
        names = {1: "record", 2: "dma_issued", 3: "image_barrier", 5: "x_in_vgprs", 6: "unit0_landed", 4: "exit"}
        ph, ph_own = {}, {}
        wl = st[live]
        for i, nm in names.items():
            ok = wl[:, i] > 0
            ph[nm] = round(float(np.median((wl[ok, i] - t0) / 100)), 2)
            ph_own[nm] = round(float(np.median((wl[ok, i] - wl[ok, 0]) / 100)), 2)
        ph["entry"] = round(float(np.median((wl[:, 0] - t0) / 100)), 2)
        grp = 16
        out[f"rep{rep}"] = {
            "workgroups": int(len(wgs)),
            "entry_by_group": [round(float(np.median(entry[i:i + grp])), 2) for i in range(0, len(wgs), grp)],
            "exit_by_group": [round(float(np.median(exit_[i:i + grp])), 2) for i in range(0, len(wgs), grp)],
            "exit_max": round(float(exit_.max()), 2), "exit_med": round(float(np.median(exit_)), 2),
            "entry_by_xcd": [round(float(np.median(entry[x::8])), 2) for x in range(8)],
            "units_per_wave_max": int(units.max()), "phases_from_first_entry": ph, "phases_from_own_entry": ph_own}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
