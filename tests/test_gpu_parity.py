"""GPU parity: the HIP backend (through the C-ABI) against the oracle on the same inputs.

Bar (BASELINE.json north_star): F32 results within 1e-3 relative —
normwise ||g-r||_inf/||r||_inf <= 1e-3 and per element |g-r| <= 1e-3*max(|r|, 1e-3*||r||_inf)
(_util.parity_ok) — and bit-exact bytes for dequantize/quantize.
"""
import os

import numpy as np
import pytest

from _util import acc_noise, parity_ok, pattern_f32, pattern_src, random_acts, random_weights

pytestmark = pytest.mark.gpu

Q_TYPES = [2, 3, 6]  # Q4_0, Q4_1, Q8_0 (lk_type ids)
QNAME = {2: "Q4_0", 3: "Q4_1", 6: "Q8_0"}


def make_inputs(O, qt, M, K, N, kind="random", seed=0):
    if kind == "pattern":
        src = pattern_src(qt, M * K, 42) * np.float32(0.25)
        x = pattern_f32(K * N, 84).reshape(K, N)
    else:
        src = random_weights(M * K, 0x5EED + seed)
        x = random_acts(K * N, 0x5EED + 1000 + seed).reshape(K, N)
    if (M * K) % 32:
        raise ValueError("quantizeTensor needs numElements % 32 == 0")
    q = O.quantize(qt, src)
    return q, x


def noise_for(O, qt, q, M, K, x):
    """acc_noise for A = q (M x K blocks, flat-index layout) against x [K, N]; N > 1 runs on the
    batched MFMA path and gets its activation-split bound too."""
    w = np.abs(O.dequantize(qt, q, M * K)).reshape(M, K)
    x = np.asarray(x).reshape(K, -1)
    return acc_noise(w, np.abs(x), split=x.shape[1] > 1)


def gpu_matmul(qt, q, M, K, N, x, a_off=0, b_off=0, d_off=0, dst_row_pad=0, b_stride=None, host=False,
               n_shards=0, pin=False):
    """Run computeMatMul through the ggml_hip mirror; returns dst as [M, N] float32.
    n_shards > 0: computeMatMulSharded over host buffers (pin: weightsPinSharded first)."""
    import ggml_hip as G
    ga = G.GGMLGraphAllocator(device="host" if host else "cuda", defaultBufferSize=16)
    a_bytes = q.size
    bcol = N if b_stride is None else b_stride
    b_bytes = 4 * K * bcol
    d_row = N + dst_row_pad
    d_bytes = 4 * M * d_row
    ia = ga.addBuffer(a_off + a_bytes + 64)
    ib = ga.addBuffer(b_off + b_bytes + 64)
    idd = ga.addBuffer(d_off + d_bytes + 64)
    a = G.GGMLTensor(G.GGMLType(qt), [K, M, 1, 1], bufferId=ia, dataOffset=a_off, name="a")
    b = G.GGMLTensor(G.GGMLType.F32, [N, K, 1, 1], nb=[4, 4 * bcol, 4 * bcol * K, 4 * bcol * K],
                     bufferId=ib, dataOffset=b_off, name="b")
    d = G.GGMLTensor(G.GGMLType.F32, [N, M, 1, 1], nb=[4, 4 * d_row, 4 * d_row * M, 4 * d_row * M],
                     bufferId=idd, dataOffset=d_off, name="dst")
    ga.setTensorBytes(a, q)
    xb = np.zeros((K, bcol), np.float32)
    xb[:, :N] = x
    ga.setTensorBytes(b, xb.view(np.uint8).reshape(-1))
    if n_shards:
        if pin:
            G.weightsPinSharded(ga, a, n_shards)
        G.computeMatMulSharded(ga, ga.context, a, b, d, n_shards)
    else:
        G.computeMatMul(ga, ga.context, a, b, d)
    raw = ga.buffers[idd]
    raw = raw if isinstance(raw, np.ndarray) else raw.cpu().numpy()
    out = raw[d_off:d_off + d_bytes].view(np.float32).reshape(M, d_row)[:, :N]
    return np.ascontiguousarray(out)


SHAPES = [
    (64, 64, 1),      # one pair per row: register-streaming GEMV (row bytes not a 16 B multiple)
    (256, 4096, 1),   # LDS-DMA GEMV, one unit (64 pairs) per row
    (100, 4096, 1),   # rows not a multiple of the waves
    (37, 11008, 1),   # 172 pairs per row: three units, the last one partial
    (70, 4352, 1),    # 68 pairs: two units, 4 pairs in the second
    (9, 16384, 1),    # 256 pairs per row: beyond the LDS-DMA kernel's VGPR-held activations
    (33, 320, 1),     # 5 pairs per row: odd pair count
    (17, 384, 1),     # 6 pairs per row (Q4_1 streams it: rows of 240 B)
    (16, 96, 1),      # K % 64 != 0 -> generic kernel
    (8, 40, 1),       # K % 32 != 0: blocks straddle rows (flat-index semantics)
    (32, 128, 3),     # N > 1: MFMA GEMM (16-column tiles)
    (5, 256, 7),
    (70, 96, 5),      # three blocks per row: a half K-stage
    (100, 4096, 32),  # C3's batch: 32-column tiles
    (33, 4352, 17),   # ragged rows and columns
    (130, 512, 100),  # 64-column tiles, ragged
    (8, 40, 3),       # K % 32 != 0 with N > 1: generic kernel
]


@pytest.mark.parametrize("qt", Q_TYPES, ids=lambda t: QNAME[t])
@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "x".join(map(str, s)))
@pytest.mark.parametrize("kind", ["random", "pattern"])
def test_mul_mat_vs_oracle(gpu, oracle, qt, shape, kind):
    M, K, N = shape
    q, x = make_inputs(oracle, qt, M, K, N, kind)
    ref = oracle.mat_mul_q(qt, q, M, K, x)
    got = gpu_matmul(qt, q, M, K, N, x)
    ok, msg = parity_ok(got, ref, noise=noise_for(oracle, qt, q, M, K, x))
    assert ok, msg


@pytest.mark.parametrize("qt", Q_TYPES, ids=lambda t: QNAME[t])
def test_offsets_strides_and_host_path(gpu, oracle, qt):
    M, K, N = 48, 256, 1
    q, x = make_inputs(oracle, qt, M, K, N, seed=3)
    ref = oracle.mat_mul_q(qt, q, M, K, x)
    for kw in [dict(a_off=16, b_off=32, d_off=48), dict(a_off=2), dict(b_off=4), dict(dst_row_pad=3),
               dict(b_stride=2), dict(host=True), dict(host=True, a_off=16, dst_row_pad=1)]:
        got = gpu_matmul(qt, q, M, K, N, x, **kw)
        ok, msg = parity_ok(got, ref)
        assert ok, (kw, msg)


def test_empty_and_k0(gpu, oracle):
    import ggml_hip as G
    # M = 0 and N = 0: nothing read or written
    for (M, N) in [(0, 1), (4, 0)]:
        ga = G.GGMLGraphAllocator(defaultBufferSize=1024)
        a = ga.allocateTensor(G.GGMLType.Q4_0, [64, M])
        b = ga.allocateTensor(G.GGMLType.F32, [N, 64])
        d = ga.allocateTensor(G.GGMLType.F32, [N, M])
        G.computeMatMul(ga, ga.context, a, b, d)
    # K = 0: every dot product is the empty sum -> dst := 0 (GGMLComputeOps.kt:132-144 with no iterations)
    ga = G.GGMLGraphAllocator(defaultBufferSize=1024)
    a = ga.allocateTensor(G.GGMLType.Q8_0, [0, 3])
    b = ga.allocateTensor(G.GGMLType.F32, [2, 0])
    d = ga.allocateTensor(G.GGMLType.F32, [2, 3])
    ga.buffers[0].fill_(0xFF)
    G.computeMatMul(ga, ga.context, a, b, d)
    out = ga.buffers[0][d.dataOffset:d.dataOffset + 24].cpu().numpy().view(np.float32)
    assert np.all(out == 0)


def test_errors_raise_like_kotlin(gpu, oracle):
    import ggml_hip as G
    ga = G.GGMLGraphAllocator(defaultBufferSize=1 << 16)
    a = ga.allocateTensor(G.GGMLType.Q4_0, [64, 4])
    b = ga.allocateTensor(G.GGMLType.F32, [1, 64])
    d = ga.allocateTensor(G.GGMLType.F32, [1, 4])
    with pytest.raises(G.IllegalArgumentException):
        G.computeMatMul(ga, ga.context, a, ga.allocateTensor(G.GGMLType.F32, [1, 32]), d)
    with pytest.raises(G.IllegalArgumentException):
        G.computeMatMul(ga, ga.context, a, b, ga.allocateTensor(G.GGMLType.F16, [1, 4]))
    with pytest.raises(NotImplementedError):
        G.computeMatMul(ga, ga.context, ga.allocateTensor(G.GGMLType.I32, [64, 4]),
                        ga.allocateTensor(G.GGMLType.I32, [1, 64]), ga.allocateTensor(G.GGMLType.I32, [1, 4]))
    bad = G.GGMLTensor(G.GGMLType.Q4_0, [64, 4], bufferId=0, dataOffset=ga.bufferSize(0) - 8)
    with pytest.raises(G.IndexOutOfBoundsException):
        G.computeMatMul(ga, ga.context, bad, b, d)
    missing = G.GGMLTensor(G.GGMLType.Q4_0, [64, 4], bufferId=7)
    with pytest.raises(G.IllegalStateException):
        G.computeMatMul(ga, ga.context, missing, b, d)


def test_f32_and_f16_general_path(gpu, oracle):
    """General fallback (GGMLComputeOps.kt:1530-1556) on the device."""
    O = oracle
    import ggml_hip as G
    for (M, K, N) in [(2, 3, 2), (4, 4, 4), (33, 70, 5), (64, 512, 64)]:
        a = pattern_f32(M * K, 1)
        x = pattern_f32(K * N, 2)
        ref = O.mat_mul_q(O.F32, a.view(np.uint8), M, K, x.reshape(K, N))
        ga = G.GGMLGraphAllocator(defaultBufferSize=1 << 20)
        ta = ga.allocateTensor(G.GGMLType.F32, [K, M]); ga.setTensorBytes(ta, a)
        tb = ga.allocateTensor(G.GGMLType.F32, [N, K]); ga.setTensorBytes(tb, x)
        td = ga.allocateTensor(G.GGMLType.F32, [N, M])
        G.computeMatMul(ga, ga.context, ta, tb, td)
        got = ga.tensorBytes(td).cpu().numpy().view(np.float32).reshape(M, N)
        ok, msg = parity_ok(got, ref)
        assert ok, msg
    # F16 x F16 -> F16 (sum in f32, stored through Kotlin floatToHalf)
    M, K, N = 12, 40, 3
    ah = (pattern_f32(M * K, 5) * np.float32(0.1)).astype(np.float16)
    bh = (pattern_f32(K * N, 6) * np.float32(0.1)).astype(np.float16)
    abuf, bbuf = ah.view(np.uint8).copy(), bh.view(np.uint8).copy()
    dbuf = np.zeros(M * N * 2, np.uint8)
    st = O.compute_mat_mul(O.make_tensor(O.F16, [K, M], abuf), O.make_tensor(O.F16, [N, K], bbuf),
                           O.make_tensor(O.F16, [N, M], dbuf))
    assert st == 0
    ref = dbuf.view(np.float16).astype(np.float32).reshape(M, N)
    ga = G.GGMLGraphAllocator(defaultBufferSize=1 << 16)
    ta = ga.allocateTensor(G.GGMLType.F16, [K, M]); ga.setTensorBytes(ta, abuf)
    tb = ga.allocateTensor(G.GGMLType.F16, [N, K]); ga.setTensorBytes(tb, bbuf)
    td = ga.allocateTensor(G.GGMLType.F16, [N, M])
    G.computeMatMul(ga, ga.context, ta, tb, td)
    got = ga.tensorBytes(td).cpu().numpy().view(np.float16).astype(np.float32).reshape(M, N)
    np.testing.assert_allclose(got, ref, rtol=2e-3, atol=2e-3)


@pytest.mark.parametrize("qt", Q_TYPES, ids=lambda t: QNAME[t])
def test_dequantize_bit_exact(gpu, oracle, qt):
    import torch
    import ggml_hip as G
    n = 32 * 4096
    src = random_weights(n, 11) * np.float32(50.0)
    src[:64] = 0.0
    src[64:96] = np.float32(1e-7)
    q = oracle.quantize(qt, src)
    ga = G.GGMLGraphAllocator(defaultBufferSize=q.size + 64)
    t = ga.allocateTensor(G.GGMLType(qt), [n])
    ga.setTensorBytes(t, q)
    got = G.dequantizeTensor(ga, t).cpu().numpy()
    torch.cuda.synchronize()
    ref = oracle.dequantize(qt, q, n)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    # blocks at an odd byte offset take the one-thread-per-block kernel: same bits
    t1 = G.GGMLTensor(G.GGMLType(qt), [n], bufferId=ga.addBuffer(q.size + 64), dataOffset=1)
    ga.setTensorBytes(t1, q)
    got = G.dequantizeTensor(ga, t1).cpu().numpy()
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


@pytest.mark.parametrize("qt", Q_TYPES, ids=lambda t: QNAME[t])
def test_quantize_bit_exact(gpu, oracle, qt):
    import torch
    import ggml_hip as G
    rng = np.random.default_rng(7)
    parts = [random_weights(32 * 512, 3), random_acts(32 * 512, 4) * np.float32(1e3),
             np.zeros(64, np.float32), np.full(32, 1e-30, np.float32),
             (rng.standard_normal(32 * 64) * np.exp2(rng.uniform(-30, 10, 32 * 64))).astype(np.float32),
             np.repeat(np.float32([0.5, -0.5, 1.5, 2.5]), 8),
             # NaN / inf / signed zeros: maxOf / minOf propagate NaN and order -0.0 < +0.0, so the
             # eight-lane butterfly of quantize_coop_kernel must give the sequential fold's value
             np.float32([np.nan] + [1.0] * 31), np.float32([2.0] * 17 + [np.inf] + [0.5] * 14),
             np.float32([-0.0, 0.0] * 16), np.float32([0.0] * 31 + [-0.0]), np.float32([-np.inf] + [3.0] * 31)]
    x = np.concatenate(parts).astype(np.float32)
    ref = oracle.quantize(qt, x)
    got = G.quantizeTensor(torch.from_numpy(x).cuda(), G.GGMLType(qt)).cpu().numpy()
    assert np.array_equal(got, ref)
    # a source off 16-byte alignment takes the one-thread-per-block kernel: same bytes
    buf = torch.from_numpy(np.concatenate([np.zeros(1, np.float32), x])).cuda()
    got = G.quantizeTensor(buf[1:], G.GGMLType(qt)).cpu().numpy()
    assert np.array_equal(got, ref)


def test_plan_equals_single_launches(gpu, oracle):
    """Independent MUL_MAT nodes in one grouped launch give the same bits as one launch each."""
    import torch
    import ggml_hip as G
    O = oracle
    ga = G.GGMLGraphAllocator(defaultBufferSize=1 << 26)
    nodes, refs = [], []
    for i, (qt, M, K) in enumerate([(2, 96, 256), (2, 40, 512), (3, 64, 256), (6, 16, 1024), (2, 8, 96),
                                    (2, 3000, 4096), (2, 5, 4096), (2, 700, 11008), (2, 1, 8192)]):
        q, x = make_inputs(O, qt, M, K, 1, seed=20 + i)
        a = ga.allocateTensor(G.GGMLType(qt), [K, M]); ga.setTensorBytes(a, q)
        b = ga.allocateTensor(G.GGMLType.F32, [1, K]); ga.setTensorBytes(b, x)
        d = ga.allocateTensor(G.GGMLType.F32, [1, M])
        nodes.append((a, b, d))
        refs.append(O.mat_mul_q(qt, q, M, K, x))
    plan = G.MulMatPlan(ga, nodes)
    # launches: Q4_0 (one-, two- and three-unit rows together), Q4_1, Q8_0, + the K=96 generic node
    assert plan.numLaunches == 4
    plan.launch()
    torch.cuda.synchronize()
    grouped = [ga.tensorBytes(d).cpu().numpy().view(np.float32).copy() for (_, _, d) in nodes]
    for (a, b, d) in nodes:
        G.computeMatMul(ga, ga.context, a, b, d)
    torch.cuda.synchronize()
    for (a, b, d), gr, ref in zip(nodes, grouped, refs):
        single = ga.tensorBytes(d).cpu().numpy().view(np.float32)
        assert np.array_equal(gr.view(np.uint32), single.view(np.uint32))
        ok, msg = parity_ok(single.reshape(-1, 1), ref)
        assert ok, msg


def test_plan_groups_pair_nodes(gpu, oracle):
    """Round 6: a plan's independent 17 <= N <= 32 Q4_0 / Q4_1 nodes run as ONE grouped pair-kernel launch
    per type plus one grouped slab-sum launch (lk_plan_launch) — the same bits as one launch each, on the
    oracle; one slice, several slices, ragged rows and columns, K = 11008; a second plan launch reuses the
    plan's slabs bit-equal."""
    import torch
    import ggml_hip as G
    O = oracle
    ga = G.GGMLGraphAllocator(defaultBufferSize=1 << 26)
    specs = [(2, 256, 4096, 32), (2, 200, 1024, 24), (2, 64, 512, 32), (2, 1000, 11008, 17),
             (3, 300, 2048, 32), (3, 48, 4096, 20), (2, 96, 256, 8)]  # the last (N = 8) stays a single launch
    nodes, refs, noises = [], [], []
    for i, (qt, M, K, N) in enumerate(specs):
        q, x = make_inputs(O, qt, M, K, N, seed=40 + i)
        a = ga.allocateTensor(G.GGMLType(qt), [K, M]); ga.setTensorBytes(a, q)
        b = ga.allocateTensor(G.GGMLType.F32, [N, K]); ga.setTensorBytes(b, np.ascontiguousarray(x, np.float32).view(np.uint8).reshape(-1))
        d = ga.allocateTensor(G.GGMLType.F32, [N, M])
        nodes.append((a, b, d))
        refs.append(O.mat_mul_q(qt, q, M, K, x))
        noises.append(noise_for(O, qt, q, M, K, x))
    plan = G.MulMatPlan(ga, nodes)
    assert plan.numLaunches == 3  # the Q4_0 group, the Q4_1 group, the N = 8 node
    G.debugRoute()
    plan.launch()
    torch.cuda.synchronize()
    route = G.debugRoute()
    assert "pairgroup<2,2>:n4" in route and "pairgroup<3,2>:n2" in route, route

    def outs():
        return [ga.tensorBytes(d).cpu().numpy().view(np.float32).copy() for (_, _, d) in nodes]

    grouped = outs()
    plan.launch()
    torch.cuda.synchronize()
    again = outs()
    for (a, b, d) in nodes:
        G.computeMatMul(ga, ga.context, a, b, d)
    torch.cuda.synchronize()
    single = outs()
    for (qt, M, K, N), gr, ag, sg, ref, nz in zip(specs, grouped, again, single, refs, noises):
        assert np.array_equal(gr.view(np.uint32), sg.view(np.uint32)), (qt, M, K, N)
        assert np.array_equal(ag.view(np.uint32), sg.view(np.uint32)), (qt, M, K, N)
        ok, msg = parity_ok(sg.reshape(M, N), ref, noise=nz)
        assert ok, ((qt, M, K, N), msg)
    plan.close()


def test_backend_graph_compute(gpu, oracle):
    import ggml_hip as G
    O = oracle
    be = G.GGMLBackendRegistry.initBackend("HIP")
    assert be.getName() == "HIP"
    ga = G.GGMLGraphAllocator(defaultBufferSize=1 << 20)
    q, x = make_inputs(O, 2, 64, 128, 1)
    a = ga.allocateTensor(G.GGMLType.Q4_0, [128, 64]); ga.setTensorBytes(a, q)
    b = ga.allocateTensor(G.GGMLType.F32, [1, 128]); ga.setTensorBytes(b, x)
    d = ga.allocateTensor(G.GGMLType.F32, [1, 64])
    d.op, d.src = G.GGMLOp.MUL_MAT, [a, b]
    assert be.supportsOp(d)
    assert be.graphCompute(G.GGMLCGraph([d], ga)) == G.GGMLStatus.SUCCESS
    be.synchronize()
    ok, msg = parity_ok(ga.tensorBytes(d).cpu().numpy().view(np.float32).reshape(64, 1), O.mat_mul_q(2, q, 64, 128, x))
    assert ok, msg
    bad = G.GGMLTensor(G.GGMLType.F32, [1, 64], op=G.GGMLOp.MUL_MAT, src=[a, ga.allocateTensor(G.GGMLType.F32, [1, 64])])
    bad.bufferId = 0
    assert be.graphCompute(G.GGMLCGraph([bad], ga)) == G.GGMLStatus.FAILED


@pytest.mark.parametrize("qt,M,K", [(6, 4096, 4096), (2, 11008, 4096), (2, 4096, 11008), (3, 11008, 4096),
                                    (3, 4096, 11008), (2, 4096, 4096)])
def test_full_size_batch1_vs_oracle(gpu, oracle, qt, M, K):
    """BASELINE configs C2/C3 and the Q4_0 4096^2 headline shape at full size, N = 1."""
    q, x = make_inputs(oracle, qt, M, K, 1, seed=M + K)
    ref = oracle.mat_mul_q(qt, q, M, K, x, tight=True)
    got = gpu_matmul(qt, q, M, K, 1, x)
    ok, msg = parity_ok(got, ref, noise=noise_for(oracle, qt, q, M, K, x))
    assert ok, msg


@pytest.mark.parametrize("qt,M,K,N", [(2, 11008, 4096, 32), (3, 11008, 4096, 32), (2, 4096, 11008, 32),
                                      (3, 4096, 11008, 32), (6, 4096, 4096, 32)])
def test_full_size_batched_vs_oracle(gpu, oracle, qt, M, K, N):
    """BASELINE config C3 at batch 32 (and Q8_0 4096^2 at batch 32), full size."""
    q, x = make_inputs(oracle, qt, M, K, N, seed=M + K + N)
    ref = oracle.mat_mul_q(qt, q, M, K, x, tight=True)
    got = gpu_matmul(qt, q, M, K, N, x)
    ok, msg = parity_ok(got, ref, noise=noise_for(oracle, qt, q, M, K, x))
    assert ok, msg


def test_c5_prefill_full(gpu, oracle):
    """Config C5: Q4_0 4096 x 4096 x 512 on the GPU, every row and column against the oracle —
    the tight restatement on up to 16 host threads (its row split is bit-identical to one
    thread, tests/test_oracle_threads.py)."""
    qt, M, K, N = 2, 4096, 4096, 512
    q, x = make_inputs(oracle, qt, M, K, N, seed=5)
    got = gpu_matmul(qt, q, M, K, N, x)
    ref = oracle.mat_mul_q(qt, q, M, K, x, tight=True, threads=min(16, os.cpu_count() or 1))
    ok, msg = parity_ok(got, ref, noise=noise_for(oracle, qt, q, M, K, x))
    assert ok, msg


def test_full_size_linearity(gpu, oracle):
    """Size-independent property: A(x1 + x2) == A x1 + A x2 (within the F32 bar)."""
    qt, M, K = 2, 11008, 4096
    q, x1 = make_inputs(oracle, qt, M, K, 1, seed=1)
    x2 = random_acts(K, 99).reshape(K, 1)
    y1 = gpu_matmul(qt, q, M, K, 1, x1)
    y2 = gpu_matmul(qt, q, M, K, 1, x2)
    y12 = gpu_matmul(qt, q, M, K, 1, (x1 + x2).astype(np.float32))
    ok, msg = parity_ok(y12, (y1.astype(np.float64) + y2))
    assert ok, msg


# Skinny split-K GEMM (2 <= N <= 32, 16-byte-aligned rows): ragged K slices, ragged tiles,
# one-slice direct stores, strided operands; misaligned weights fall back to the LDS GEMM.
SKINNY = [
    (1000, 11008, 2),   # 344 blocks: 21 full K slices and a half one
    (4096, 4096, 16),   # exactly one 16-column x-tile
    (257, 4096, 31),    # ragged rows (a 1-row tile) and columns (two x-tiles)
    (40, 512, 5),       # one K slice: outputs stored without the reduce kernel
    (3000, 2048, 32),
    (50, 384, 20),      # 12 blocks: the second half-slice has 4 blocks (Q4_1; Q4_0 rows are not 16-B)
    (300, 1280, 24),    # 40 blocks: the last slice has no second half
    # the in-launch split-K reduction at its limits: 64 slices (the largest counter row) over one
    # row range; 128 slices (past it: the reduce launch instead); many tiles per range at N <= 16
    (16, 32768, 20),
    (64, 65536, 8),
    (5000, 4096, 3),
]


@pytest.mark.parametrize("qt", Q_TYPES, ids=lambda t: QNAME[t])
@pytest.mark.parametrize("shape", SKINNY, ids=lambda s: "x".join(map(str, s)))
def test_skinny_gemm_vs_oracle(gpu, oracle, qt, shape):
    M, K, N = shape
    q, x = make_inputs(oracle, qt, M, K, N, seed=M + N)
    ref = oracle.mat_mul_q(qt, q, M, K, x, tight=True)
    noise = noise_for(oracle, qt, q, M, K, x)
    got = gpu_matmul(qt, q, M, K, N, x)
    ok, msg = parity_ok(got, ref, noise=noise)
    assert ok, msg
    again = gpu_matmul(qt, q, M, K, N, x)
    assert np.array_equal(got.view(np.uint32), again.view(np.uint32)), "split-K reduction is not deterministic"


@pytest.mark.parametrize("qt", Q_TYPES, ids=lambda t: QNAME[t])
def test_skinny_gemm_offsets_strides(gpu, oracle, qt):
    M, K, N = 100, 1024, 9
    q, x = make_inputs(oracle, qt, M, K, N, seed=11)
    ref = oracle.mat_mul_q(qt, q, M, K, x)
    noise = noise_for(oracle, qt, q, M, K, x)
    for kw in [dict(a_off=16, b_off=32, d_off=48), dict(a_off=2), dict(b_off=4), dict(dst_row_pad=3),
               dict(b_stride=11), dict(host=True, a_off=32, dst_row_pad=1)]:
        got = gpu_matmul(qt, q, M, K, N, x, **kw)
        ok, msg = parity_ok(got, ref, noise=noise)
        assert ok, (kw, msg)


# Wide GEMM (N > 32, K % 128 == 0): 256-row x 64-column tiles, K split over slices when the
# tiles do not fill the chip, ragged rows / columns, strided outputs.
WIDE = [
    (300, 4096, 64),    # split K, ragged rows
    (257, 1024, 100),   # ragged columns (a 4-column x-tile) and a 1-row tail
    (64, 11008, 48),    # one row tile, long K
    (1024, 512, 33),    # the smallest wide N
    (128, 4096, 80),    # in-launch split (N % 16 == 0): a column tile with one real x-tile
    (512, 2048, 160),   # in-launch split, three column tiles
]


@pytest.mark.parametrize("qt", Q_TYPES, ids=lambda t: QNAME[t])
@pytest.mark.parametrize("shape", WIDE, ids=lambda s: "x".join(map(str, s)))
def test_wide_gemm_vs_oracle(gpu, oracle, qt, shape):
    M, K, N = shape
    q, x = make_inputs(oracle, qt, M, K, N, seed=M + 3 * N)
    ref = oracle.mat_mul_q(qt, q, M, K, x, tight=True)
    noise = noise_for(oracle, qt, q, M, K, x)
    got = gpu_matmul(qt, q, M, K, N, x)
    ok, msg = parity_ok(got, ref, noise=noise)
    assert ok, msg
    again = gpu_matmul(qt, q, M, K, N, x)
    assert np.array_equal(got.view(np.uint32), again.view(np.uint32)), "wide GEMM is not deterministic"
    got = gpu_matmul(qt, q, M, K, N, x, d_off=16, dst_row_pad=5)
    ok, msg = parity_ok(got, ref, noise=noise)
    assert ok, ("strided dst", msg)


def test_w32_route_and_nonfinite_scales(gpu, oracle):
    """Q4_0 at N > 32 runs gemm_w32_kernel (round 6, lk_wide32.hpp), which applies each block's f16
    scale d to the block's MFMA sum in f32 (acc += d·p). Kotlin multiplies d into every term
    ((d·(q − 8))·x, GGMLComputeOps.kt:120-145), so a non-finite scale makes the row's outputs
    non-finite in both; they may differ only in which non-finite value (NaN vs ±Inf). Checked: the
    route; finite-ness equal to the oracle element by element; every finite element on the oracle."""
    import ggml_hip as G
    M, K, N = 256, 1024, 64
    q, x = make_inputs(oracle, 2, M, K, N, seed=99)
    q = q.copy()
    rb = K // 32 * 18
    for row, blk, bits in ((3, 5, 0x7C00), (100, 0, 0x7E00), (200, 31, 0xFC00)):  # +Inf, NaN, -Inf
        q[row * rb + blk * 18:row * rb + blk * 18 + 2] = np.frombuffer(np.uint16(bits).tobytes(), np.uint8)
    ref = oracle.mat_mul_q(2, q, M, K, x, tight=True)
    G.debugRoute()
    got = gpu_matmul(2, q, M, K, N, x)
    assert "w32" in G.debugRoute()
    assert np.array_equal(np.isfinite(got), np.isfinite(ref))
    fin = np.isfinite(ref).all(axis=1)
    assert fin.sum() == M - 3
    ok, msg = parity_ok(got[fin], ref[fin], noise=noise_for(oracle, 2, q, M, K, x)[fin])
    assert ok, msg


@pytest.mark.parametrize("shape", [(100, 1024, 36), (33, 128, 4), (257, 384, 60), (64, 4096, 32)],
                         ids=lambda s: "x".join(map(str, s)))
def test_f32_lds_kernel_edges(gpu, oracle, shape):
    """The LDS-staged F32 MFMA kernel (dense operands, K % 128 == 0, N % 4 == 0): ragged rows and
    columns (re-read, never stored), one chunk for one of four waves, several chunks per wave;
    against the oracle (F32 path, GGMLComputeOps.kt:1530-1543) and bit-equal on a rerun."""
    import ggml_hip as G
    M, K, N = shape
    a = pattern_f32(M * K, 3)
    x = pattern_f32(K * N, 4)
    ref = oracle.mat_mul_q(oracle.F32, a.view(np.uint8), M, K, x.reshape(K, N))
    outs = []
    for _ in range(2):
        ga = G.GGMLGraphAllocator(defaultBufferSize=4 * (M * K + K * N + M * N) + 1024)
        ta = ga.allocateTensor(G.GGMLType.F32, [K, M]); ga.setTensorBytes(ta, a)
        tb = ga.allocateTensor(G.GGMLType.F32, [N, K]); ga.setTensorBytes(tb, x)
        td = ga.allocateTensor(G.GGMLType.F32, [N, M])
        G.computeMatMul(ga, ga.context, ta, tb, td)
        outs.append(ga.tensorBytes(td).cpu().numpy().view(np.float32).reshape(M, N).copy())
    ok, msg = parity_ok(outs[0], ref, noise=acc_noise(np.abs(a.reshape(M, K)), np.abs(x.reshape(K, N))))
    assert ok, msg
    assert np.array_equal(outs[0].view(np.uint32), outs[1].view(np.uint32))


def test_c1_f32_512_cubed(gpu, oracle):
    """BASELINE config C1 at its size: F32 512x512x512 through computeMatMul's general path
    (GGMLComputeOps.kt:1530-1543), the benchmark test's F32 values
    (T/core/GGMLMatMulBenchmarkTest.kt:51-56, seeds 42 / 84), against the structural oracle."""
    import ggml_hip as G
    n = 512
    a = pattern_f32(n * n, 42)
    x = pattern_f32(n * n, 84)
    ref = oracle.mat_mul_q(oracle.F32, a.view(np.uint8), n, n, x.reshape(n, n))
    ga = G.GGMLGraphAllocator(defaultBufferSize=3 * 4 * n * n + 256)
    ta = ga.allocateTensor(G.GGMLType.F32, [n, n]); ga.setTensorBytes(ta, a)
    tb = ga.allocateTensor(G.GGMLType.F32, [n, n]); ga.setTensorBytes(tb, x)
    td = ga.allocateTensor(G.GGMLType.F32, [n, n])
    G.computeMatMul(ga, ga.context, ta, tb, td)
    got = ga.tensorBytes(td).cpu().numpy().view(np.float32).reshape(n, n)
    ok, msg = parity_ok(got, ref, noise=acc_noise(np.abs(a.reshape(n, n)), np.abs(x.reshape(n, n))))
    assert ok, msg


# More skinny (2 <= N <= 32) shapes on the product kernels (gemm_skinny_pair_kernel for N > 16):
# ragged rows, one slice (K <= 512, no split-K reduction), a half slice at the end of K, many tiles
# per row range.
SKINNY_EXTRA = [
    (257, 4096, 20),    # ragged rows (a 1-row tile), 8 slices
    (64, 256, 24),      # one half slice
    (100, 512, 28),     # one full slice
    (33, 768, 32),      # a full and a half slice
    (1000, 11008, 32),  # 43 blocks x 8: the last slice half, many tiles per range
]


@pytest.mark.parametrize("qt", [2, 3], ids=lambda t: QNAME[t])
@pytest.mark.parametrize("shape", SKINNY_EXTRA, ids=lambda s: "x".join(map(str, s)))
def test_skinny_extra_shapes_vs_oracle(gpu, oracle, qt, shape):
    M, K, N = shape
    for kind in ("random", "pattern"):
        q, x = make_inputs(oracle, qt, M, K, N, kind, seed=M + 7 * N)
        ref = oracle.mat_mul_q(qt, q, M, K, x, tight=True)
        noise = noise_for(oracle, qt, q, M, K, x)
        got = gpu_matmul(qt, q, M, K, N, x)
        ok, msg = parity_ok(got, ref, noise=noise)
        assert ok, (kind, msg)
        again = gpu_matmul(qt, q, M, K, N, x)
        assert np.array_equal(got.view(np.uint32), again.view(np.uint32)), "not deterministic"


def test_no_sync_timeouts(gpu, oracle):
    """The batched kernels' in-launch split-K reduction (every workgroup co-resident, waits bounded
    at 200 ms): after a C3-shaped skinny call, a 22-slice skinny call and a C5-shaped wide call,
    and every batched test before this one, no wait has given up (lk_sync_timeouts)."""
    import ggml_hip as G
    for (qt, M, K, N) in [(2, 11008, 4096, 32), (2, 4096, 11008, 32), (2, 4096, 4096, 64), (3, 1000, 4096, 8)]:
        q, x = make_inputs(oracle, qt, M, K, N, "random", seed=M + N)
        gpu_matmul(qt, q, M, K, N, x)
    assert G.syncTimeouts() == 0
