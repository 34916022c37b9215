import sys, os
sys.path[:0] = ["tests", "oracle", "llama.kotlin_amd"]
import numpy as np, torch
import oracle as O
torch.cuda.set_device(0)
import ggml_hip as G
G.load_library()
from test_gpu_parity import make_inputs
from _util import parity_ok

def run(q, x, M, K, mode):
    ga = G.GGMLGraphAllocator(device="cuda", defaultBufferSize=16)
    ia = ga.addBuffer(q.size + 64); ib = ga.addBuffer(4 * K + 64); idd = ga.addBuffer(4 * M + 64)
    ga.buffers[idd].fill_(0x7F)
    a = G.GGMLTensor(G.GGMLType.Q4_0, [K, M], bufferId=ia)
    b = G.GGMLTensor(G.GGMLType.F32, [1, K], bufferId=ib)
    d = G.GGMLTensor(G.GGMLType.F32, [1, M], bufferId=idd)
    ga.setTensorBytes(a, q); ga.setTensorBytes(b, x.reshape(-1).view(np.uint8))
    if mode == "sync_before": torch.cuda.synchronize()
    G.computeMatMul(ga, None, a, b, d)
    if mode == "sync_after": torch.cuda.synchronize()
    return ga.buffers[idd][:4 * M].cpu().numpy().view(np.float32).reshape(M, 1).copy()

for mode in ["none", "sync_before", "sync_after", "none"]:
    bad = {"zero": 0, "sentinel": 0, "other": 0}
    for it in range(60):
        q, x = make_inputs(O, 2, 64, 4096, 1, "random", seed=it)
        ref = O.mat_mul_q(2, q, 64, 4096, x)
        got = run(q, x, 64, 4096, mode)
        ok, msg = parity_ok(got, ref)
        if not ok:
            if np.all(got == 0): bad["zero"] += 1
            elif np.all(got.view(np.uint32) == 0x7F7F7F7F): bad["sentinel"] += 1
            else:
                bad["other"] += 1
                print("other", msg, got[:4, 0], ref[:4, 0])
    print(mode, bad, flush=True)
