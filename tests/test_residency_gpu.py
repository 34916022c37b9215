"""The weight-residency contract of the host (ByteArray) path (include/lk_hip.h, SURVEY §7.3.6,
A14): a device mirror is current for (ByteArray base, byte range, generation). The Kotlin
caller rewrites bytes in place — GGMLGraphAllocator.allocateGraph re-places tensors
(K/core/GGMLAlloc.kt:404-480), reserve replaces buffers (:392, :638) — and then bumps the
generation or evicts. These tests rewrite host bytes the way the caller does (straight into
the ByteArray, no library call) and check that a re-pin with a new generation, an eviction of
the tensor, of its buffer, or of everything is honoured by lk_mul_mat, lk_mul_mat_sharded and a
live lk_graph, without the cache growing across generations."""
import numpy as np
import pytest

from _util import parity_ok, random_acts, random_weights

pytestmark = pytest.mark.gpu

M, K = 96, 256


def _setup(oracle, qt=2, seed=0):
    import ggml_hip as G
    ga = G.GGMLGraphAllocator(device="host", defaultBufferSize=1 << 18)
    a = ga.allocateTensor(G.GGMLType(qt), [K, M], name="w")
    q0 = oracle.quantize(qt, random_weights(M * K, seed + 1))
    ga.setTensorBytes(a, q0)
    b = ga.allocateTensor(G.GGMLType.F32, [1, K], name="x")
    x = random_acts(K, seed + 2)
    ga.setTensorBytes(b, x)
    d = ga.allocateTensor(G.GGMLType.F32, [1, M], name="y")
    return ga, a, b, d, x


def _rewrite(ga, a, q):
    """The caller's in-place rewrite of the weight bytes (no library call)."""
    buf = ga.buffers[a.bufferId]
    buf[a.dataOffset:a.dataOffset + q.size] = q


def _result(ga, d):
    return np.frombuffer(bytes(ga.tensorBytes(d)), np.float32).reshape(-1, 1).copy()


def _check(oracle, qt, q, x, got):
    ref = oracle.mat_mul_q(qt, q, M, K, x.reshape(K, 1))
    ok, msg = parity_ok(got, ref)
    assert ok, msg


def test_repin_with_new_generation_serves_new_bytes(gpu, oracle):
    import ggml_hip as G
    ga, a, b, d, x = _setup(oracle)
    q0 = np.frombuffer(bytes(ga.tensorBytes(a)), np.uint8).copy()
    G.weightsPin(ga, a, 0)
    base_bytes, base_count = G.weightsCachedBytes(), G.weightsCachedCount()
    G.computeMatMul(ga, ga.context, a, b, d)
    _check(oracle, 2, q0, x, _result(ga, d))
    for gen in range(1, 4):
        q = oracle.quantize(2, random_weights(M * K, 100 + gen))
        _rewrite(ga, a, q)
        G.weightsPin(ga, a, gen)
        G.computeMatMul(ga, ga.context, a, b, d)
        _check(oracle, 2, q, x, _result(ga, d))
        # the superseded mirror is gone: the cache does not grow across generations
        assert G.weightsCachedBytes() == base_bytes
        assert G.weightsCachedCount() == base_count
    # the same generation again is a no-op (no re-copy, no growth)
    G.weightsPin(ga, a, 3)
    assert G.weightsCachedCount() == base_count


def test_repin_same_generation_keeps_the_mirror(gpu, oracle):
    """The contract, pinned: bytes rewritten WITHOUT a generation bump or eviction are not seen
    (the mirror is current for that generation) — the caller's duty is to bump or evict."""
    import ggml_hip as G
    ga, a, b, d, x = _setup(oracle, seed=10)
    q0 = np.frombuffer(bytes(ga.tensorBytes(a)), np.uint8).copy()
    G.weightsPin(ga, a, 7)
    q1 = oracle.quantize(2, random_weights(M * K, 11))
    _rewrite(ga, a, q1)
    G.weightsPin(ga, a, 7)
    G.computeMatMul(ga, ga.context, a, b, d)
    _check(oracle, 2, q0, x, _result(ga, d))
    G.weightsEvict(ga, a)
    G.computeMatMul(ga, ga.context, a, b, d)
    _check(oracle, 2, q1, x, _result(ga, d))


@pytest.mark.parametrize("how", ["evict", "evict_buffer", "evict_all"])
def test_eviction_stages_fresh_bytes(gpu, oracle, how):
    import ggml_hip as G
    ga, a, b, d, x = _setup(oracle, qt=6, seed=20)
    G.weightsPin(ga, a, 0)
    assert G.weightsCachedBytes() >= M * K // 32 * 34
    q1 = oracle.quantize(6, random_weights(M * K, 21))
    _rewrite(ga, a, q1)
    if how == "evict":
        G.weightsEvict(ga, a)
    elif how == "evict_buffer":
        G.weightsEvictBuffer(ga, a.bufferId)
    else:
        G.weightsEvictAll()
    assert G.weightsCachedBytes() == 0
    G.computeMatMul(ga, ga.context, a, b, d)
    _check(oracle, 6, q1, x, _result(ga, d))


def test_evict_leaves_other_ranges(gpu, oracle):
    import ggml_hip as G
    ga, a, b, d, x = _setup(oracle, seed=30)
    a2 = ga.allocateTensor(G.GGMLType.Q4_0, [K, M], name="w2")
    ga.setTensorBytes(a2, oracle.quantize(2, random_weights(M * K, 31)))
    G.weightsPin(ga, a, 0)
    G.weightsPin(ga, a2, 0)
    assert G.weightsCachedCount() == 2
    G.weightsEvict(ga, a)
    assert G.weightsCachedCount() == 1
    assert G.weightsCachedBytes() == M * K // 32 * 18


@pytest.mark.parametrize("how", ["repin", "evict", "evict_all"])
def test_resident_graph_rebinds_after_rewrite(gpu, oracle, how):
    import ggml_hip as G
    ga, a, b, d, x = _setup(oracle, seed=40)
    q0 = np.frombuffer(bytes(ga.tensorBytes(a)), np.uint8).copy()
    g = G.ResidentGraph(ga, [(a, b, d)], weightGeneration=0)
    g.compute()
    g.compute()  # second compute: captured as a HIP graph (raw mirror pointers inside)
    _check(oracle, 2, q0, x, _result(ga, d))
    assert g.numRebinds == 0
    count = G.weightsCachedCount()
    q1 = oracle.quantize(2, random_weights(M * K, 41))
    _rewrite(ga, a, q1)
    if how == "repin":
        G.weightsPin(ga, a, 1)
    elif how == "evict":
        G.weightsEvict(ga, a)
    else:
        G.weightsEvictAll()
    for _ in range(3):  # the rebind compute, its eager successor, then a captured replay
        g.compute()
        _check(oracle, 2, q1, x, _result(ga, d))
    assert g.numRebinds == 1
    assert G.weightsCachedCount() == count


def test_two_graphs_share_and_follow_a_repin(gpu, oracle):
    import ggml_hip as G
    ga, a, b, d, x = _setup(oracle, seed=50)
    d2 = ga.allocateTensor(G.GGMLType.F32, [1, M], name="y2")
    g1 = G.ResidentGraph(ga, [(a, b, d)], weightGeneration=0)
    g2 = G.ResidentGraph(ga, [(a, b, d2)], weightGeneration=0)
    assert G.weightsCachedCount() == 1  # one mirror, two holders
    g1.compute(); g2.compute()
    q1 = oracle.quantize(2, random_weights(M * K, 51))
    _rewrite(ga, a, q1)
    G.weightsPin(ga, a, 1)
    g1.compute(); g2.compute()
    _check(oracle, 2, q1, x, _result(ga, d))
    _check(oracle, 2, q1, x, _result(ga, d2))
    assert G.weightsCachedCount() == 1


def test_sharded_repin(gpu, oracle):
    import ggml_hip as G
    ga, a, b, d, x = _setup(oracle, seed=60)
    G.weightsPinSharded(ga, a, 3, 0)
    G.computeMatMulSharded(ga, ga.context, a, b, d, 3)
    _check(oracle, 2, np.frombuffer(bytes(ga.tensorBytes(a)), np.uint8).copy(), x, _result(ga, d))
    n0 = G.weightsCachedBytes()
    q1 = oracle.quantize(2, random_weights(M * K, 61))
    _rewrite(ga, a, q1)
    G.weightsPinSharded(ga, a, 3, 1)
    G.computeMatMulSharded(ga, ga.context, a, b, d, 3)
    _check(oracle, 2, q1, x, _result(ga, d))
    assert G.weightsCachedBytes() == n0


def test_freed_buffer_address_reuse(gpu, oracle):
    """A ByteArray freed and another allocated at the same address: the allocator mirror evicts
    a buffer's mirrors when the buffer goes away (tensor.py), so the new bytes are read."""
    import gc
    import ggml_hip as G
    seen = set()
    for i in range(6):
        ga, a, b, d, x = _setup(oracle, seed=70 + i)
        q = np.frombuffer(bytes(ga.tensorBytes(a)), np.uint8).copy()
        seen.add(ga.dataPtr(a.bufferId))
        G.weightsPin(ga, a, 0)  # generation 0 every time, as a careless caller would
        G.computeMatMul(ga, ga.context, a, b, d)
        _check(oracle, 2, q, x, _result(ga, d))
        del ga, a, b, d
        gc.collect()
        assert G.weightsCachedCount() == 0
