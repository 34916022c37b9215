import sys, os
sys.path[:0] = ["tests", "oracle", "llama.kotlin_amd"]
import numpy as np, torch
import oracle as O
torch.cuda.set_device(0)
import ggml_hip as G
G.load_library()
from test_gpu_parity import make_inputs
from _util import parity_ok
side = torch.cuda.Stream()

def run(q, x, M, K, mode):
    ga = G.GGMLGraphAllocator(device="cuda", defaultBufferSize=16)
    ia = ga.addBuffer(q.size + 64); ib = ga.addBuffer(4 * K + 64); idd = ga.addBuffer(4 * M + 64)
    ga.buffers[idd].fill_(0x7F)
    a = G.GGMLTensor(G.GGMLType.Q4_0, [K, M], bufferId=ia)
    b = G.GGMLTensor(G.GGMLType.F32, [1, K], bufferId=ib)
    d = G.GGMLTensor(G.GGMLType.F32, [1, M], bufferId=idd)
    ga.setTensorBytes(a, q); ga.setTensorBytes(b, x.reshape(-1).view(np.uint8))
    if mode == "null":
        G.computeMatMul(ga, None, a, b, d)
    elif mode == "null+streamsync":
        G.computeMatMul(ga, None, a, b, d)
        torch.cuda.current_stream().synchronize()
    elif mode == "side+waits":
        side.wait_stream(torch.cuda.current_stream())
        G.computeMatMul(ga, None, a, b, d, stream=side)
        torch.cuda.current_stream().wait_stream(side)
    elif mode == "all_on_side":
        pass
    return ga.buffers[idd][:4 * M].cpu().numpy().view(np.float32).reshape(M, 1).copy()

def run_all_side(q, x, M, K):
    with torch.cuda.stream(side):
        ga = G.GGMLGraphAllocator(device="cuda", defaultBufferSize=16)
        ia = ga.addBuffer(q.size + 64); ib = ga.addBuffer(4 * K + 64); idd = ga.addBuffer(4 * M + 64)
        ga.buffers[idd].fill_(0x7F)
        a = G.GGMLTensor(G.GGMLType.Q4_0, [K, M], bufferId=ia)
        b = G.GGMLTensor(G.GGMLType.F32, [1, K], bufferId=ib)
        d = G.GGMLTensor(G.GGMLType.F32, [1, M], bufferId=idd)
        ga.setTensorBytes(a, q); ga.setTensorBytes(b, x.reshape(-1).view(np.uint8))
        G.computeMatMul(ga, None, a, b, d)
        return ga.buffers[idd][:4 * M].cpu().numpy().view(np.float32).reshape(M, 1).copy()

for mode in ["null", "null+streamsync", "side+waits", "all_on_side", "null"]:
    bad = 0
    for it in range(60):
        q, x = make_inputs(O, 2, 64, 4096, 1, "random", seed=it)
        ref = O.mat_mul_q(2, q, 64, 4096, x)
        got = run_all_side(q, x, 64, 4096) if mode == "all_on_side" else run(q, x, 64, 4096, mode)
        ok, msg = parity_ok(got, ref)
        bad += not ok
    print(mode, "bad", bad, "/60", flush=True)
