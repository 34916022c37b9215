"""Launch floors for the batch-1 stream kernel (lab tool): mean µs per launch in HIP-graph replay
of an empty kernel and of a bare LDS-DMA read of a Q4_0 matrix's bytes (tools/floor.hip), at the
stream kernel's grid, over rotating copies larger than the Infinity Cache.
Usage: python tools/floor.py (after building tools/libfloor.so)."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]

import bench  # noqa: E402


def main():
    import numpy as np
    import torch
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libfloor.so"))
    lib.floor_empty.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    lib.floor_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.floor_read.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                               ctypes.c_void_p, ctypes.c_void_p]
    s = torch.cuda.Stream(device=dev)
    sp = ctypes.c_void_p(s.cuda_stream)
    out = torch.zeros(4096, device=dev)
    res = {}
    n = 256
    for lds in (0, 160 * 1024):
        def run_empty():
            for _ in range(48):
                lib.floor_empty(n, lds, ctypes.c_void_p(out.data_ptr()), sp)
        per, _ = bench._graph_time(torch, run_empty, s, 20)
        res[f"empty_lds{lds // 1024}k"] = round(per / 48 * 1e6, 3)
    for name, nbytes, copies, xb in (("q4_0_4096x4096", 4096 * 4096 // 32 * 18, 48, 16384),
                                     ("q4_0_11008x4096", 11008 * 4096 // 32 * 18, 16, 16384),
                                     ("layer", 114148352, 8, 16384)):
        bufs = torch.empty(copies * nbytes + 4096, dtype=torch.uint8, device=dev)
        bufs.random_(0, 255)
        x = torch.randn(xb // 4, device=dev)
        for depth in (6, 12):
            for with_x in (False, True):
                def run_read():
                    for c in range(copies):
                        lib.floor_read(ctypes.c_void_p(bufs.data_ptr() + c * nbytes), nbytes,
                                       ctypes.c_void_p(x.data_ptr() if with_x else 0), xb, n, depth,
                                       ctypes.c_void_p(out.data_ptr()), sp)
                per, _ = bench._graph_time(torch, run_read, s, 10)
                us = per / copies * 1e6
                rec = {"us": round(us, 3), "GBps": round(nbytes / us / 1e3, 1)}
                if depth == 6 and with_x:  # stamps of the last launch: first piece landed / exit after entry
                    st = (ctypes.c_uint64 * (1024 * 8 * 4))()
                    lib.floor_stamps(st, len(st))
                    a = np.array(list(st), dtype=np.int64).reshape(1024, 8, 4)[:n]
                    t0 = a[:, :, 0].min()
                    rel = (a - t0) / 100.0
                    rec["entry_med"] = round(float(np.median(rel[:, :, 0])), 2)
                    rec["first_landed_med"] = round(float(np.median(rel[:, :, 1])), 2)
                    rec["exit_med"] = round(float(np.median(rel[:, :, 2])), 2)
                    rec["exit_max"] = round(float(rel[:, :, 2].max()), 2)
                res[f"read_{name}_d{depth}{'_x' if with_x else ''}"] = rec
        del bufs
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
