"""Lab diagnostic (not collected by pytest): split-K tile-counter growth in a fresh process.

Host-path calls (lk_mul_mat, the library's non-blocking stream) of the down-projection shape of
tests/test_graph_gpu.py (Q4_0, K = 384: 216-B rows, so gemm_q_mfma_kernel with 12 K slices and one
arrival counter per 128-row tile) with the row count growing call by call, so every call needs more
tile counters than exist: round 4's library reallocated them each time (hipFree + hipMalloc + a
hipMemset on the null stream, which nothing orders before a launch on a non-blocking stream); round 5
zeroes them with hipMemsetAsync on the launch stream. BUSY=1 first queues ~10 ms of torch matmuls on torch's default
stream — the legacy null stream, behind which round 4's hipMemset waits while the library's
non-blocking stream runs the kernel at once. Every result against the oracle; prints one line
per call that misses the parity bar and a summary.
Usage: [LK_HIP_LIB=...] [BUSY=1] python tests/diag_counter_growth.py"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [HERE, ROOT, os.path.join(ROOT, "llama.kotlin_amd"), os.path.join(ROOT, "oracle")]


def main():
    import torch
    import oracle as O
    import ggml_hip as G
    from _util import parity_ok, random_acts, random_weights
    from test_gpu_parity import gpu_matmul, noise_for
    O.lib()
    G.load_library()
    torch.cuda.set_device(0)
    K, N = 384, 4
    bad = 0
    busy = os.environ.get("BUSY") == "1"
    sq = torch.randn(2048, 2048, device="cuda") / 64
    torch.cuda.synchronize()
    for rep in range(int(os.environ.get("REPS", "3"))):
        for t in range(1, 41):
            M = 128 * t + 128 * 40 * rep  # more tiles than any call before
            q = O.quantize(2, random_weights(M * K, t))
            x = random_acts(K * N, 100 + t).reshape(K, N)
            # garbage in recently freed device memory, so a counter buffer recycled from it is not zero
            junk = torch.full((1 << 18,), -1, dtype=torch.int32, device="cuda")
            del junk
            torch.cuda.empty_cache()
            if busy:  # the null stream busy for ~10 ms (not waited for)
                y = sq
                for _ in range(60):
                    y = y @ sq
            got = gpu_matmul(2, q, M, K, N, x, host=True)
            ref = O.mat_mul_q(2, q, M, K, x)
            ok, msg = parity_ok(got, ref, noise=noise_for(O, 2, q, M, K, x))
            if not ok:
                bad += 1
                err = np.abs(got - ref).max(axis=1)
                rows = np.nonzero(err > 1e-3 * np.abs(ref).max())[0]
                zeros = int((got == 0).sum())
                print(f"rep {rep} M {M}: {msg}; wrong rows {rows.min()}..{rows.max()} ({rows.size}) "
                      f"tiles {sorted(set((rows // 128).tolist()))[:8]} exact zeros {zeros} of {got.size}", flush=True)
    print(f"calls off the oracle: {bad} of {40 * int(os.environ.get('REPS', '3'))}", flush=True)


if __name__ == "__main__":
    main()
