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
    buf = (ctypes.c_uint64 * (1024 * 8 * 8))()
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
        st = np.frombuffer(buf, np.uint64).reshape(1024, 8, 8).astype(np.int64)
        res = {"route": route}
        # slots: w32_main 2 vmcnt wait, 3 barrier, 5 DMA issue; w32_main_pp 2 operand phase, 3 waits + barriers,
        # 5 DMA issue, 6 matrix phase (cycles per stage, medians over waves of each row half)
        for half, ws in (("half0", slice(0, 4)), ("half1", slice(4, 8))):
            sub = st[:, ws, :]
            live = sub[:, :, 4] > 0
            if not live.any():
                continue
            nst = np.maximum(sub[:, :, 4][live], 1)
            per = lambda k: float(np.median(sub[:, :, k][live] / nst))  # noqa: E731
            res[half] = {"waves": int(live.sum()), "stages": float(np.median(nst)),
                         "loop_per_stage": float(np.median((sub[:, :, 1] - sub[:, :, 0])[live] / nst)),
                         "slot2": per(2), "slot3": per(3), "slot5_issue": per(5), "slot6": per(6)}
        out[name] = res
        del g
    print(json.dumps(out))


if __name__ == "__main__":
    main()
