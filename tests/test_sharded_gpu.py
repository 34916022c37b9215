"""lk_mul_mat_sharded: computeMatMul over host buffers with A's rows split over
the GPUs of one process. On a one-GPU box every shard maps to device 0 (shard r runs on
device r mod device count), which exercises the row split, the per-shard staging offsets
and the disjoint dst write-back exactly as on eight devices."""
import numpy as np
import pytest

from _util import parity_ok, random_acts, random_weights
from test_gpu_parity import gpu_matmul, noise_for

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("qt,M,K,N,P", [
    (2, 4096, 4096, 1, 8), (3, 70, 256, 1, 3), (6, 33, 320, 2, 2), (2, 5, 64, 1, 8),
    (2, 130, 512, 17, 4), (3, 11008, 4096, 1, 8), (6, 37, 11008, 1, 3),
])
def test_sharded_matches_single_and_oracle(gpu, oracle, qt, M, K, N, P):
    q = oracle.quantize(qt, random_weights(M * K, 0x5EED + M))
    x = random_acts(K * N, 0x5EED + K).reshape(K, N)
    single = gpu_matmul(qt, q, M, K, N, x, host=True)
    for pin in (False, True):
        got = gpu_matmul(qt, q, M, K, N, x, host=True, n_shards=P, pin=pin)
        if N == 1:  # one wave per row, sequential in k: the split cannot change a bit
            assert np.array_equal(got.view(np.uint32), single.view(np.uint32)), pin
        ref = oracle.mat_mul_q(qt, q, M, K, x, tight=True)
        ok, msg = parity_ok(got, ref, noise=noise_for(oracle, qt, q, M, K, x))
        assert ok, (pin, msg)


def test_sharded_strided_dst_and_offsets(gpu, oracle):
    qt, M, K, N = 2, 96, 256, 3
    q = oracle.quantize(qt, random_weights(M * K, 3))
    x = random_acts(K * N, 4).reshape(K, N)
    ref = oracle.mat_mul_q(qt, q, M, K, x)
    got = gpu_matmul(qt, q, M, K, N, x, a_off=36, b_off=20, d_off=8, dst_row_pad=5, host=True, n_shards=4)
    ok, msg = parity_ok(got, ref, noise=noise_for(oracle, qt, q, M, K, x))
    assert ok, msg


def test_sharded_falls_back_when_rows_straddle_blocks(gpu, oracle):
    """K % 32 != 0: rows are not byte ranges of A (flat-index blocks), so one device runs it."""
    qt, M, K, N = 2, 8, 40, 2
    q = oracle.quantize(qt, random_weights(M * K, 5))
    x = random_acts(K * N, 6).reshape(K, N)
    got = gpu_matmul(qt, q, M, K, N, x, host=True, n_shards=4)
    single = gpu_matmul(qt, q, M, K, N, x, host=True)
    assert np.array_equal(got.view(np.uint32), single.view(np.uint32))


def test_sharded_errors_and_pins(gpu, oracle):
    import ggml_hip as G
    ga = G.GGMLGraphAllocator(device="host", defaultBufferSize=1 << 16)
    a = ga.allocateTensor(G.GGMLType.Q4_0, [64, 8])
    b = ga.allocateTensor(G.GGMLType.F32, [1, 64])
    d = ga.allocateTensor(G.GGMLType.F32, [1, 8])
    with pytest.raises(G.IllegalArgumentException):
        G.computeMatMulSharded(ga, ga.context, a, b, d, 0)
    bad = ga.allocateTensor(G.GGMLType.F32, [1, 9])
    with pytest.raises(G.IllegalArgumentException):
        G.computeMatMulSharded(ga, ga.context, a, b, bad, 2)
    G.weightsEvictAll()
    G.weightsPinSharded(ga, a, 3)
    from ggml_hip import _lib
    assert _lib.load().lk_weights_cached_bytes() == 8 * 2 * 18
    G.weightsEvictAll()
    assert _lib.load().lk_weights_cached_bytes() == 0


def test_rccl_sharded_plan_world1_equals_plan(gpu, oracle):
    """The C-ABI RCCL path (lk_comm + lk_sharded_plan) at world size 1 on the one GPU of the box:
    bit-equal to lk_plan over the same nodes, and a second plan reading the first one's dst."""
    import torch
    import ggml_hip as G
    from _util import random_acts, random_weights
    comm = G.Comm.single()
    assert comm.nranks == 1
    K, F = 256, 384
    ga = G.GGMLGraphAllocator(defaultBufferSize=1 << 20)
    specs = [("q", 2, K, K), ("k", 3, K, K), ("v", 6, K, K), ("gate", 2, K, F), ("up", 2, K, F)]
    x = ga.allocateTensor(G.GGMLType.F32, [1, K]); ga.setTensorBytes(x, random_acts(K, 1))
    nodes, ref_nodes = [], []
    for i, (name, qt, k, m) in enumerate(specs):
        a = ga.allocateTensor(G.GGMLType(qt), [k, m]); ga.setTensorBytes(a, oracle.quantize(qt, random_weights(k * m, 10 + i)))
        d = ga.allocateTensor(G.GGMLType.F32, [1, m])
        dr = ga.allocateTensor(G.GGMLType.F32, [1, m])
        nodes.append((G.shard_view(a, 1, 0), x, d))
        ref_nodes.append((a, x, dr))
    plan = G.ShardedMulMatPlan(comm, ga, nodes)
    assert plan.numGathers == len(nodes)
    ref = G.MulMatPlan(ga, ref_nodes)
    # level 2 reads level 1's (gathered) outputs
    wd = ga.allocateTensor(G.GGMLType.Q4_0, [F, K]); ga.setTensorBytes(wd, oracle.quantize(2, random_weights(F * K, 99)))
    d2 = ga.allocateTensor(G.GGMLType.F32, [1, K])
    d2r = ga.allocateTensor(G.GGMLType.F32, [1, K])
    plan2 = G.ShardedMulMatPlan(comm, ga, [(G.shard_view(wd, 1, 0), nodes[4][2], d2)])
    ref2 = G.MulMatPlan(ga, [(wd, ref_nodes[4][2], d2r)])
    s = torch.cuda.Stream()
    for _ in range(2):
        plan.launch(stream=s); plan2.launch(stream=s)
        ref.launch(stream=s); ref2.launch(stream=s)
    torch.cuda.synchronize()
    for (_, _, d), (_, _, dr) in zip(nodes + [(None, None, d2)], ref_nodes + [(None, None, d2r)]):
        assert bytes(ga.tensorBytes(d).cpu().numpy()) == bytes(ga.tensorBytes(dr).cpu().numpy())
    plan.close(); plan2.close(); comm.close()


def test_rccl_sharded_plan_rejects_uneven_rows(gpu):
    import ggml_hip as G
    comm = G.Comm.single()
    ga = G.GGMLGraphAllocator(defaultBufferSize=1 << 16)
    a = ga.allocateTensor(G.GGMLType.Q4_0, [64, 8])
    b = ga.allocateTensor(G.GGMLType.F32, [1, 64])
    d = ga.allocateTensor(G.GGMLType.F32, [1, 16])  # A holds 8 rows of a 16-row dst at P = 1
    with pytest.raises(G.IllegalArgumentException):
        G.ShardedMulMatPlan(comm, ga, [(a, b, d)])
    comm.close()
