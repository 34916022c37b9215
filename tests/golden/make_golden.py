"""Generate tests/golden/*.npz — fixed input/output vectors for the MUL_MAT path.

Inputs follow SURVEY §8d: the reference benchmark's pattern generators
(T/core/GGMLMatMulBenchmarkTest.kt:51-82, seeds 42 for A and 84 for B) and a seeded
normal set (weights N(0, 0.02^2), activations N(0, 1)). Block bytes come from the
restated quantizeTensor; expected outputs from the restated computeMatMul (oracle/).
The reference itself cannot run here, so these vectors are pinned by the
KATs in tests/test_oracle_kats.py; they freeze the oracle and give the GPU a fixed
target. Run:  python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.dirname(HERE)]

import oracle as O  # noqa: E402
from _util import pattern_f32, pattern_src, random_acts, random_weights  # noqa: E402

CASES = [
    # name, type, M, K, N, kind
    ("q4_0_pattern_64x128x1", O.Q4_0, 64, 128, 1, "pattern"),
    ("q4_0_random_96x256x1", O.Q4_0, 96, 256, 1, "random"),
    ("q4_0_random_40x96x3", O.Q4_0, 40, 96, 3, "random"),
    ("q4_0_ragged_8x40x2", O.Q4_0, 8, 40, 2, "random"),
    ("q4_1_pattern_64x128x1", O.Q4_1, 64, 128, 1, "pattern"),
    ("q4_1_random_96x256x2", O.Q4_1, 96, 256, 2, "random"),
    ("q8_0_pattern_64x128x1", O.Q8_0, 64, 128, 1, "pattern"),
    ("q8_0_random_48x512x1", O.Q8_0, 48, 512, 1, "random"),
    ("q8_0_kat_2x32x2", O.Q8_0, 2, 32, 2, "kat"),
    ("f32_kat_2x3x2", O.F32, 2, 3, 2, "kat"),
    ("f32_pattern_16x64x8", O.F32, 16, 64, 8, "pattern"),
]


def inputs(qt, M, K, N, kind, name):
    if kind == "kat" and qt == O.F32:
        return np.array([1, 2, 3, 4, 5, 6], np.float32), np.array([7, 8, 9, 10, 11, 12], np.float32).reshape(K, N)
    if kind == "kat":
        a = np.zeros((M, K), np.float32)
        a[0, :3] = [1, 2, 3]
        a[1, :3] = [4, 5, 60]
        b = np.zeros((K, N), np.float32)
        b[:3] = [[7, 8], [9, 10], [11, 12]]
        return a.reshape(-1), b
    if kind == "pattern":
        src = pattern_f32(M * K, 42) if qt == O.F32 else pattern_src(qt, M * K, 42) * np.float32(0.25)
        return src, pattern_f32(K * N, 84).reshape(K, N)
    seed = sum(map(ord, name))
    return random_weights(M * K, seed), random_acts(K * N, seed + 1).reshape(K, N)


def build_case(name, qt, M, K, N, kind):
    src, x = inputs(qt, M, K, N, kind, name)
    a_bytes = src.view(np.uint8).copy() if qt == O.F32 else O.quantize(qt, src)
    dst = O.mat_mul_q(qt, a_bytes, M, K, x)
    return dict(type=np.int32(qt), M=np.int64(M), K=np.int64(K), N=np.int64(N), a=a_bytes,
                b=np.ascontiguousarray(x, np.float32), dst=dst, src=src)


def main():
    for case in CASES:
        d = build_case(*case)
        np.savez_compressed(os.path.join(HERE, case[0] + ".npz"), **d)
        print(case[0], d["a"].size, "bytes of A")


if __name__ == "__main__":
    main()
