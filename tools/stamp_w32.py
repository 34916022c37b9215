"""Where gemm_w32_kernel's main loop waits (lab tool; tools/build_lab.sh w32st -DLK_LAB_W32_STAMPS):
per wave, cycles (s_memtime) of the whole loop, of its waits for the wave's own DMAs (vmcnt) and of the
stage barriers; medians over waves of the last of several warm calls, for C5 and C3.
Usage: LK_HIP_LIB=<lab .so> python tools/stamp_w32.py"""
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
    buf = (ctypes.c_uint64 * (1024 * 4 * 8))()
    T = G.GGMLType
    s = torch.cuda.Stream(device=dev)
    out = {}
    for name, qt, M, K, N in (("c5", T.Q4_0, 4096, 4096, 512), ("c3", T.Q4_0, 11008, 4096, 32)):
        nb = M * K // 32 * 18
        g = G.GGMLGraphAllocator(device=str(dev), defaultBufferSize=16)
        wb, xb, db = g.addBuffer(nb + 256), g.addBuffer(4 * K * N + 256), g.addBuffer(4 * M * N + 256)
        g.buffers[wb][:nb].copy_(G.quantizeTensor(torch.randn(M * K, device=dev) * 0.02, qt))
        g.buffers[xb][: 4 * K * N].copy_(torch.randn(K * N, device=dev).view(torch.uint8))
        a, b, d = G.GGMLTensor(qt, [K, M], bufferId=wb), G.GGMLTensor(T.F32, [N, K], bufferId=xb), G.GGMLTensor(T.F32, [N, M], bufferId=db)
        for _ in range(5):
            G.computeMatMul(g, None, a, b, d, stream=s)
        s.synchronize()
        G.debugRoute()
        G.computeMatMul(g, None, a, b, d, stream=s)
        s.synchronize()
        route = G.debugRoute()
        assert lib.lk_lab_w32_stamps(buf, len(buf)) == 0
        st = np.frombuffer(buf, np.uint64).reshape(1024, 4, 8).astype(np.int64)
        live = st[:, :, 4] > 0
        loop = (st[:, :, 1] - st[:, :, 0])[live]
        wait = st[:, :, 2][live]
        bar = st[:, :, 3][live]
        nst = st[:, :, 4][live]
        iss = st[:, :, 5][live]
        out[name] = {"route": route, "waves": int(live.sum()), "stages_per_wave": float(np.median(nst)),
                     "loop_cycles_median": float(np.median(loop)), "loop_cycles_max": float(loop.max()),
                     "vmcnt_wait_median": float(np.median(wait)), "barrier_wait_median": float(np.median(bar)),
                     "per_stage_cycles": float(np.median(loop / np.maximum(nst, 1))),
                     "per_stage_wait": float(np.median(wait / np.maximum(nst, 1))),
                     "per_stage_barrier": float(np.median(bar / np.maximum(nst, 1))),
                     "per_stage_dma_issue": float(np.median(iss / np.maximum(nst, 1)))}
        del g
    print(json.dumps(out))


if __name__ == "__main__":
    main()
