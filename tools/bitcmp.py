"""Lab: outputs of a fixed set of batched calls (seeded inputs) saved to an .npz, so two library builds
can be compared bit for bit: LK_HIP_LIB=<a> python tools/bitcmp.py out_a.npz; ... out_b.npz;
python tools/bitcmp.py --cmp out_a.npz out_b.npz"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "llama.kotlin_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]

CASES = [(2, 11008, 4096, 32), (3, 11008, 4096, 32), (2, 4096, 11008, 32), (2, 11008, 4096, 24), (2, 4096, 4096, 512),
         (2, 11008, 4096, 16), (3, 4096, 4096, 8), (6, 4096, 4096, 32),
         (3, 4096, 4096, 512), (2, 4096, 11008, 64), (3, 2048, 4096, 48), (2, 1024, 4096, 80), (6, 1024, 4096, 96)]


def main():
    import numpy as np
    if sys.argv[1] == "--cmp":
        a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
        bad = [k for k in a.files if a[k].tobytes() != b[k].tobytes()]
        print("bit-identical" if not bad else f"differ: {bad}")
        sys.exit(1 if bad else 0)
    import torch
    import oracle as O
    from _util import random_acts, random_weights
    from test_gpu_parity import gpu_matmul
    torch.cuda.set_device(0)
    out = {}
    for (qt, M, K, N) in CASES:
        q = O.quantize(qt, random_weights(M * K, M + K + N))
        x = random_acts(K * N, K + N).reshape(K, N)
        out[f"q{qt}_{M}x{K}_n{N}"] = gpu_matmul(qt, q, M, K, N, x)
    np.savez(sys.argv[1], **out)
    print("saved", sys.argv[1])


if __name__ == "__main__":
    main()
