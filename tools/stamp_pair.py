"""Phases of gemm_skinny_pair_kernel on C3 (lab tool; tools/build_lab.sh stamps -DLK_LAB_STAMPS): per-wave
stamps of the current kernel (slot 0 entry, 1 split done, 5 ring issued, 6 barrier, 2 loop start = fragments in VGPRs, 9 first unit landed, 3 loop end = its stores
drained, 4 exit, 8 units). One warm graph-free call of Q4_0 / Q4_1 11008 x 4096 at N = 32; medians
and maxima in µs after the launch's first entry, and the reduce launch's share by wall clock.
Usage: LK_HIP_LIB=<lab .so> python tools/stamp_pair.py"""
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
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    G.load_library()
    lib = ctypes.CDLL(os.environ["LK_HIP_LIB"])
    buf = (ctypes.c_uint64 * (1024 * 8 * 10))()
    T = G.GGMLType
    s = torch.cuda.Stream(device=dev)
    M, K, N = 11008, 4096, 32
    out = {}
    for qt, name in ((T.Q4_0, "c3_q4_0"), (T.Q4_1, "c3_q4_1")):
        bb = 18 if qt == T.Q4_0 else 20
        nb = M * K // 32 * bb
        g = G.GGMLGraphAllocator(device=str(dev), defaultBufferSize=16)
        wb, xb, db = g.addBuffer(nb + 256), g.addBuffer(4 * K * N + 256), g.addBuffer(4 * M * N + 256)
        g.buffers[wb][:nb].copy_(G.quantizeTensor(torch.randn(M * K, device=dev) * 0.02, qt))
        g.buffers[xb][: 4 * K * N].copy_(torch.randn(K * N, device=dev).view(torch.uint8))
        a = G.GGMLTensor(qt, [K, M], bufferId=wb)
        b = G.GGMLTensor(T.F32, [N, K], bufferId=xb)
        d = G.GGMLTensor(T.F32, [N, M], bufferId=db)
        reps = []
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
            t0 = st[:, :, 0][live].min()
            w = st[live]
            ph = {}
            for slot, nm in ((0, "entry"), (1, "split"), (5, "ring_issued"), (6, "barrier"), (2, "loop_start"), (9, "unit0"),
                             (3, "loop_end"), (4, "exit")):
                ok = w[:, slot] > 0
                v = (w[ok, slot] - t0) / 100
                ph[nm] = [round(float(np.median(v)), 2), round(float(v.max()), 2)]
            ph["units_per_wave"] = [int(np.median(w[:, 8])), int(w[:, 8].max())]
            reps.append(ph)
        out[name] = reps
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
