import sys, os
sys.path[:0] = ["tests", "oracle", "llama.kotlin_amd"]
import numpy as np, torch
import oracle as O
from test_gpu_parity import gpu_matmul, make_inputs
from _util import parity_ok
torch.cuda.set_device(0)
for kind in ["pattern", "random"]:
    for (qt, M, K, N) in [(2, 64, 128, 1), (2, 64, 4096, 1), (2, 256, 4096, 1), (2, 64, 256, 1), (2, 16, 96, 1), (6, 64, 128, 1)]:
        q, x = make_inputs(O, qt, M, K, N, kind)
        ref = O.mat_mul_q(qt, q, M, K, x)
        got = gpu_matmul(qt, q, M, K, N, x)
        ok, msg = parity_ok(got, ref)
        print(kind, qt, M, K, N, ok, msg, "got", got[:3, 0], "ref", ref[:3, 0], flush=True)
