"""The in-launch split-K fix-up (round 4) and the failure contract of the remaining waits.

The batched kernels (skinny, pair, sk, wide) split K over workgroups and sum the slices inside the
launch by the LAST ARRIVER per output tile (lk_kernels.hpp splitk_arrive): nobody waits for another
workgroup, so a grid larger than the CUs that are free, or CUs held by another stream's kernel,
changes nothing but the time. The per-tile counters re-arm inside every launch (zero between
launches, lk_sync_counters_sum). Only the opt-in chain plans still wait (grid barriers); a wait that
gives up there is counted (lk_sync_timeouts) and reported (plan.timedOut), never silently taken as
success (core/GGMLCpuBackend.kt:167-176: failure is FAILED, never wrong bytes)."""
import os

import numpy as np
import pytest

from _util import parity_ok, random_acts, random_weights
from test_gpu_parity import gpu_matmul, noise_for

pytestmark = pytest.mark.gpu

DEFAULT_BOUND = 20000000  # 200 ms at 100 MHz


@pytest.mark.parametrize("qt,M,K,N", [(2, 11008, 4096, 32), (2, 4096, 11008, 32), (3, 4096, 4096, 8), (2, 4096, 4096, 512)])
def test_split_k_counters_rearm_every_launch(gpu, oracle, qt, M, K, N):
    import ggml_hip as G
    q = oracle.quantize(qt, random_weights(M * K, 5))
    x = random_acts(K * N, 6).reshape(K, N)
    first = gpu_matmul(qt, q, M, K, N, x)
    assert G.syncCountersSum() == 0
    for _ in range(3):
        again = gpu_matmul(qt, q, M, K, N, x)
        assert np.array_equal(again.view(np.uint32), first.view(np.uint32))
        assert G.syncCountersSum() == 0
    assert G.syncTimeouts() == 0


@pytest.mark.parametrize("qt,M,K,N", [
    (2, 64, 153600, 8),    # 300 K slices over one row range: 300 workgroups on 256 CUs (skinny, one wave per stream)
    (3, 48, 153600, 20),   # the same on wave pairs (Q4_1)
    (2, 6400, 512, 512),   # wide: 200 tiles x 2 slices = 400 workgroups
])
def test_split_k_grid_larger_than_the_gpu(gpu, oracle, qt, M, K, N):
    """Grids the old co-resident design could not run in-launch (it waited for every slice of a row
    range, so it needed every workgroup resident at once): now fixed up in the launch, against the
    oracle, bit-equal on a rerun, counters re-armed."""
    import ggml_hip as G
    q = oracle.quantize(qt, random_weights(M * K, M + N))
    x = random_acts(K * N, K + N).reshape(K, N)
    got = gpu_matmul(qt, q, M, K, N, x)
    ref = oracle.mat_mul_q(qt, q, M, K, x, tight=True, threads=min(16, os.cpu_count() or 1))
    ok, msg = parity_ok(got, ref, noise=noise_for(oracle, qt, q, M, K, x))
    assert ok, msg
    again = gpu_matmul(qt, q, M, K, N, x)
    assert np.array_equal(got.view(np.uint32), again.view(np.uint32))
    assert G.syncCountersSum() == 0 and G.syncTimeouts() == 0


def test_split_k_beside_a_kernel_holding_the_cus(gpu, oracle):
    """C3 (Q4_0 11008 x 4096, N = 32) and C5 (Q4_0 4096^2, N = 512) issued on one stream while a
    long GEMM on another stream holds CUs: the same bytes as the quiet runs, no wait given up."""
    import torch
    import ggml_hip as G
    cases = []
    ga = G.GGMLGraphAllocator(defaultBufferSize=16)
    for (M, K, N, seed) in [(11008, 4096, 32, 1), (4096, 4096, 512, 2)]:
        q = oracle.quantize(2, random_weights(M * K, seed))
        x = random_acts(K * N, seed + 10).reshape(K, N)
        a = G.GGMLTensor(G.GGMLType.Q4_0, [K, M], bufferId=ga.addBuffer(q.size + 64))
        b = G.GGMLTensor(G.GGMLType.F32, [N, K], bufferId=ga.addBuffer(4 * K * N + 64))
        d = G.GGMLTensor(G.GGMLType.F32, [N, M], bufferId=ga.addBuffer(4 * M * N + 64))
        ga.setTensorBytes(a, q)
        ga.setTensorBytes(b, np.ascontiguousarray(x))
        cases.append((a, b, d))
    ours, other = torch.cuda.Stream(), torch.cuda.Stream()
    quiet = []
    for (a, b, d) in cases:
        G.computeMatMul(ga, None, a, b, d, stream=ours)
        torch.cuda.synchronize()
        quiet.append(ga.tensorBytes(d).cpu().numpy().copy())
    big = torch.randn(8192, 8192, device="cuda")
    for rep in range(3):
        for (_, _, d) in cases:
            ga.tensorBytes(d).fill_(0xFF)
        torch.cuda.synchronize()
        with torch.cuda.stream(other):
            for _ in range(4):
                big = torch.tanh(big @ big * 1e-4)  # ~tens of ms of work that occupies every CU
        for (a, b, d) in cases:
            G.computeMatMul(ga, None, a, b, d, stream=ours)
        torch.cuda.synchronize()
        for i, (_, _, d) in enumerate(cases):
            assert np.array_equal(ga.tensorBytes(d).cpu().numpy(), quiet[i]), (rep, i)
    assert G.syncCountersSum() == 0 and G.syncTimeouts() == 0


def test_batched_paths_have_no_wait_to_give_up(gpu, oracle):
    """With the wait bound at 0 (every wait gives up at once) the batched host operator and a resident
    graph still return the original bytes: the split-K fix-up never waits. The bound is restored."""
    import ggml_hip as G
    qt, M, K, N = 2, 11008, 4096, 32
    q = oracle.quantize(qt, random_weights(M * K, 7))
    x = random_acts(K * N, 8).reshape(K, N)
    want = gpu_matmul(qt, q, M, K, N, x, host=True)
    ga = G.GGMLGraphAllocator(device="host", defaultBufferSize=q.size + 4 * (K * N + M * N) + 4096)
    a = ga.allocateTensor(G.GGMLType.Q4_0, [K, M]); ga.setTensorBytes(a, q)
    b = ga.allocateTensor(G.GGMLType.F32, [N, K]); ga.setTensorBytes(b, np.ascontiguousarray(x))
    d = ga.allocateTensor(G.GGMLType.F32, [N, M])
    g = G.ResidentGraph(ga, [(a, b, d)])
    try:
        G.setSyncWaitBound(0)
        G.computeMatMul(ga, ga.context, a, b, d)
        got = np.frombuffer(bytes(ga.tensorBytes(d)), np.float32).reshape(M, N)
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
        ga.setTensorBytes(d, np.zeros(4 * M * N, np.uint8))
        g.compute()
        assert bytes(ga.tensorBytes(d)) == want.tobytes()
    finally:
        G.setSyncWaitBound(DEFAULT_BOUND)
    assert G.syncTimeouts() == 0 and G.syncCountersSum() == 0
    g.close()


def test_chain_wait_that_gives_up_is_reported(gpu):
    """The chain plans' grid barriers are the waits left. Bound 0: the launch gives up at its first
    barrier — plan.timedOut() says so and lk_sync_timeouts counts it — and with the bound restored the
    same plan runs clean again, bit-identical to stage-by-stage launches."""
    import torch
    import ggml_hip as G
    from test_chain_gpu import _chain
    ga = G.GGMLGraphAllocator(device="cuda", defaultBufferSize=16)
    nodes, stages, *_ = _chain(G, ga, 2, [4096, 4096, 4096], [1, 1], seed=11)
    for (a, b, d) in nodes:
        G.computeMatMul(ga, ga.context, a, b, d)
    torch.cuda.synchronize()
    ref = [ga.tensorBytes(d).cpu().numpy().copy() for (_, _, d) in nodes]
    plan = G.MulMatPlan(ga, nodes, stages=stages)
    assert G.syncTimeouts() == 0
    try:
        G.setSyncWaitBound(0)
        plan.launch()
        torch.cuda.synchronize()
        assert plan.timedOut()
    finally:
        G.setSyncWaitBound(DEFAULT_BOUND)
    assert G.syncTimeouts() > 0
    assert G.syncTimeouts() == 0  # reported once
    plan.launch()
    torch.cuda.synchronize()
    assert not plan.timedOut()
    for i, (_, _, d) in enumerate(nodes):
        assert np.array_equal(ga.tensorBytes(d).cpu().numpy(), ref[i]), i
