import sys, os
sys.path[:0] = ["tests", "oracle", "llama.kotlin_amd"]
import numpy as np, torch
import oracle as O
torch.cuda.set_device(0)
import ggml_hip as G
G.load_library()
print("current stream", torch.cuda.current_stream(), torch.cuda.current_stream().cuda_stream)
maps = open("/proc/self/maps").read().splitlines()
print(sorted({l.split()[-1] for l in maps if "amdhip64" in l or "hsa-runtime" in l}))
from test_gpu_parity import gpu_matmul, make_inputs
from _util import parity_ok
bad = 0
for it in range(40):
    q, x = make_inputs(O, 2, 64, 4096, 1, "random", seed=it)
    ref = O.mat_mul_q(2, q, 64, 4096, x)
    got = gpu_matmul(2, q, 64, 4096, 1, x)
    ok, msg = parity_ok(got, ref)
    bad += (not ok)
print("no-sync failures", bad, "/ 40")
