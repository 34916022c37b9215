"""Direct dot products computeDotProduct{F32Q41, F32Q80, Q80Q80, Q40Q40, Q41Q41, Q80Q40}
(core/GGMLComputeOps.kt:349-629) through lk_dot_direct*.

The reference never reaches these from computeMatMul and holds no known-answer test for them
(their only caller, T/core/GGMLMatMulBenchmarkTest.kt:412-428, is a timing loop whose operands
do not even pass the functions' own K checks). So the C oracle is cross-checked against an
independent numpy restatement below (bit-exact: both evaluate every Kotlin expression in f32
and sum k left to right) — parity with the reference itself is unpinned. The GPU path keeps the
same order and explicit roundings, so it must match the oracle bit for bit."""
import numpy as np
import pytest

import oracle as O
from _util import random_acts, random_weights

F32_Q41, F32_Q80, Q80_Q80, Q40_Q40, Q41_Q41, Q80_Q40 = 1, 2, 3, 4, 5, 6
KINDS = {F32_Q41: (O.F32, O.Q4_1), F32_Q80: (O.F32, O.Q8_0), Q80_Q80: (O.Q8_0, O.Q8_0),
         Q40_Q40: (O.Q4_0, O.Q4_0), Q41_Q41: (O.Q4_1, O.Q4_1), Q80_Q40: (O.Q8_0, O.Q4_0)}
KNAME = {F32_Q41: "F32Q41", F32_Q80: "F32Q80", Q80_Q80: "Q80Q80", Q40_Q40: "Q40Q40", Q41_Q41: "Q41Q41",
         Q80_Q40: "Q80Q40"}
BB = {O.Q4_0: 18, O.Q4_1: 20, O.Q8_0: 34}
# (M, K, N): M*K and K*N multiples of 32 (whole blocks); blocks straddle rows when K % 32 != 0
SHAPES = [(3, 64, 5), (4, 32, 8), (2, 48, 16), (5, 96, 3), (1, 320, 1)]


def operands(kind, M, K, N, seed):
    """(A bytes, B bytes): A is M x K (flat row*K + k, or F32 [K, M] contiguous), B is K x N
    (flat k*N + col)."""
    ta, tb = KINDS[kind]
    if ta == O.F32:
        a = random_acts(M * K, seed).view(np.uint8).copy()
    else:
        a = O.quantize(ta, random_weights(M * K, seed, std=1.0))
    b = O.quantize(tb, random_weights(K * N, seed + 1, std=1.0))
    return a, b


def tensors(kind, a, b, M, K, N, a_nb1=None):
    ta, tb = KINDS[kind]
    nb = None if a_nb1 is None else [4, a_nb1, a_nb1 * M, a_nb1 * M]
    return O.make_tensor(ta, [K, M], a, nb=nb), O.make_tensor(tb, [N, K], b)


# ---- independent restatement (numpy, f32 scalar semantics) --------------------------------

def _q_elems(qt, raw, n):
    """Element values exactly as the Kotlin expressions form them (f32, one rounding per op)."""
    bb = BB[qt]
    blk = raw.reshape(-1, bb)[: (n + 31) // 32]
    d = blk[:, 0:2].copy().view("<f2").astype(np.float32)[:, 0]
    if qt == O.Q8_0:
        q = blk[:, 2:34].view(np.int8).astype(np.float32)
        v = np.float32(d[:, None]) * q
    else:
        base = 2 if qt == O.Q4_0 else 4
        by = blk[:, base:base + 16]
        q = np.empty((blk.shape[0], 32), np.float32)
        q[:, 0::2] = (by & 0x0F).astype(np.float32)
        q[:, 1::2] = (by >> 4).astype(np.float32)
        if qt == O.Q4_0:
            v = d[:, None] * (q - np.float32(8.0))
        else:
            m = blk[:, 2:4].copy().view("<f2").astype(np.float32)[:, 0]
            v = (d[:, None] * q) + m[:, None]
    return v.astype(np.float32).reshape(-1)[:n]


def dot_matrix_ref(kind, a, b, M, K, N, a_nb1=None):
    ta, tb = KINDS[kind]
    wb = _q_elems(tb, b, K * N).reshape(K, N)
    if ta == O.F32:
        row = (a_nb1 or 4 * K) // 4
        wa = a.view(np.float32)[: (M - 1) * row + K].copy()
        wa = np.stack([wa[i * row: i * row + K] for i in range(M)])  # [M, K]
    else:
        wa = _q_elems(ta, a, M * K).reshape(M, K)
    s = np.zeros((M, N), np.float32)
    for k in range(K):
        if kind == Q80_Q80:  # scaleA * scaleB * (qA * qB)
            fa, fb = np.arange(M) * K + k, k * N + np.arange(N)
            blk_a, blk_b = a.reshape(-1, 34), b.reshape(-1, 34)
            sa = blk_a[fa // 32, 0:2].copy().view("<f2").astype(np.float32)[:, 0]
            sb = blk_b[fb // 32, 0:2].copy().view("<f2").astype(np.float32)[:, 0]
            qa = blk_a[fa // 32, 2 + fa % 32].view(np.int8).astype(np.float32)
            qb = blk_b[fb // 32, 2 + fb % 32].view(np.int8).astype(np.float32)
            p = (sa[:, None] * sb[None, :]) * (qa[:, None] * qb[None, :])
        else:
            p = wa[:, k][:, None] * wb[k][None, :]
        s = (s + p.astype(np.float32)).astype(np.float32)
    return s


@pytest.mark.parametrize("kind", list(KINDS), ids=lambda k: KNAME[k])
@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_oracle_matches_numpy_restatement(kind, shape):
    M, K, N = shape
    a, b = operands(kind, M, K, N, seed=M * 31 + K + N)
    ta, tb = tensors(kind, a, b, M, K, N)
    st, got = O.dot_direct_matrix(kind, ta, tb, K)
    assert st == 0, O.last_error()
    ref = dot_matrix_ref(kind, a, b, M, K, N)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


@pytest.mark.parametrize("kind", [F32_Q41, F32_Q80], ids=lambda k: KNAME[k])
def test_oracle_f32_rows_honour_nb(kind):
    M, K, N = 3, 64, 4
    pad = 40  # bytes between rows of A
    dense = random_acts(M * K, 5)
    a = np.zeros(M * (4 * K + pad), np.uint8)
    for i in range(M):
        a[i * (4 * K + pad): i * (4 * K + pad) + 4 * K] = dense[i * K:(i + 1) * K].view(np.uint8)
    b = O.quantize(KINDS[kind][1], random_weights(K * N, 6, std=1.0))
    ta, tb = tensors(kind, a, b, M, K, N, a_nb1=4 * K + pad)
    st, got = O.dot_direct_matrix(kind, ta, tb, K)
    assert st == 0
    ref = dot_matrix_ref(kind, a, b, M, K, N, a_nb1=4 * K + pad)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


def test_oracle_single_dot_is_the_matrix_entry():
    M, K, N = 3, 64, 5
    a, b = operands(Q80_Q40, M, K, N, 9)
    ta, tb = tensors(Q80_Q40, a, b, M, K, N)
    _, mat = O.dot_direct_matrix(Q80_Q40, ta, tb, K)
    for (i, j) in [(0, 0), (2, 4), (1, 3)]:
        st, v = O.dot_direct(Q80_Q40, ta, tb, i, j, K)
        assert st == 0 and np.float32(v).view(np.uint32) == mat[i, j].view(np.uint32)


def _error_cases():
    """(name, kind, a, b, K, expected status) — each a require() or accessor failure."""
    M, K, N = 2, 64, 3
    a, b = operands(Q40_Q40, M, K, N, 1)
    ta, tb = tensors(Q40_Q40, a, b, M, K, N)
    wrong_type = O.make_tensor(O.Q8_0, [K, M], np.zeros(M * K // 32 * 34, np.uint8))
    cases = [("tensorA type", Q40_Q40, wrong_type, tb, K, 1),
             ("tensorB type", Q40_Q40, ta, O.make_tensor(O.Q8_0, [N, K], np.zeros(K * N // 32 * 34, np.uint8)), K, 1),
             ("A K dim", Q40_Q40, ta, tb, K + 32, 1),
             ("unknown kind", 42, ta, tb, K, 2)]
    short = O.make_tensor(O.Q4_0, [K, M], a[:-5].copy())
    cases.append(("A past its buffer", Q40_Q40, short, tb, K, 3))
    cases.append(("B missing buffer", Q40_Q40, ta, O.make_tensor(O.Q4_0, [N, K], None), K, 4))
    # M*K % 32 != 0: the last elements' block is numBlocks -> IllegalArgumentException
    a_odd = O.quantize(O.Q4_0, random_weights(96, 2))
    t_odd = O.make_tensor(O.Q4_0, [40, 2], np.concatenate([a_odd, np.zeros(18, np.uint8)]))
    b40 = O.make_tensor(O.Q4_0, [4, 40], O.quantize(O.Q4_0, random_weights(160, 3)))
    cases.append(("A block past numBlocks", Q40_Q40, t_odd, b40, 40, 1))
    return cases


@pytest.mark.parametrize("case", _error_cases(), ids=lambda c: c[0])
def test_oracle_errors(case):
    _, kind, ta, tb, K, want = case
    st, _ = O.dot_direct_matrix(kind, ta, tb, K)
    assert st == want, O.last_error()


# ---- GPU: bit-identical to the oracle, host and device buffers -----------------------------

GPU_SHAPES = SHAPES + [(64, 4096, 48), (7, 1056, 33)]


def _gpu_dot(kind, a, b, M, K, N, host):
    import ggml_hip as G
    ta_, tb_ = KINDS[kind]
    ga = G.GGMLGraphAllocator(device="host" if host else "cuda", defaultBufferSize=16)
    ia, ib = ga.addBuffer(a.size + 32), ga.addBuffer(b.size + 32)
    A = G.GGMLTensor(G.GGMLType(ta_), [K, M], bufferId=ia, dataOffset=16)
    B = G.GGMLTensor(G.GGMLType(tb_), [N, K], bufferId=ib, dataOffset=16)
    ga.setTensorBytes(A, a)
    ga.setTensorBytes(B, b)
    out = G.computeDotProductMatrix(kind, ga, A, B, K)
    if not host:
        import torch
        torch.cuda.synchronize()
        out = out.cpu().numpy()
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("kind", list(KINDS), ids=lambda k: KNAME[k])
@pytest.mark.parametrize("shape", GPU_SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_direct_dot_gpu_bit_exact(gpu, kind, shape):
    M, K, N = shape
    a, b = operands(kind, M, K, N, seed=M + K * 3 + N)
    ta, tb = tensors(kind, a, b, M, K, N)
    st, ref = O.dot_direct_matrix(kind, ta, tb, K)
    assert st == 0
    for host in (False, True):
        got = _gpu_dot(kind, a, b, M, K, N, host)
        assert got.shape == (M, N)
        bad = np.flatnonzero(got.view(np.uint32) != ref.view(np.uint32))
        assert bad.size == 0, (host, bad[:5], got.reshape(-1)[bad[:5]], ref.reshape(-1)[bad[:5]])


@pytest.mark.gpu
def test_direct_dot_gpu_named_functions(gpu):
    import ggml_hip as G
    M, K, N = 3, 64, 4
    for kind, fn in [(F32_Q41, G.computeDotProductF32Q41), (F32_Q80, G.computeDotProductF32Q80),
                     (Q80_Q80, G.computeDotProductQ80Q80), (Q40_Q40, G.computeDotProductQ40Q40),
                     (Q41_Q41, G.computeDotProductQ41Q41), (Q80_Q40, G.computeDotProductQ80Q40)]:
        a, b = operands(kind, M, K, N, 17)
        ta_, tb_ = KINDS[kind]
        ga = G.GGMLGraphAllocator(device="cuda", defaultBufferSize=16)
        A = G.GGMLTensor(G.GGMLType(ta_), [K, M], bufferId=ga.addBuffer(a.size))
        B = G.GGMLTensor(G.GGMLType(tb_), [N, K], bufferId=ga.addBuffer(b.size))
        ga.setTensorBytes(A, a)
        ga.setTensorBytes(B, b)
        st, v = O.dot_direct(kind, *tensors(kind, a, b, M, K, N), 2, 3, K)
        assert st == 0
        assert np.float32(fn(ga, A, B, 2, 3, K)).view(np.uint32) == np.float32(v).view(np.uint32)


@pytest.mark.gpu
def test_direct_dot_gpu_errors_like_oracle(gpu):
    import ggml_hip as G
    exc = {1: G.IllegalArgumentException, 2: G.NotOffloadedError, 3: G.IndexOutOfBoundsException,
           4: G.IllegalStateException}
    for name, kind, ta, tb, K, want in _error_cases():
        # the same operands as host-buffer tensors of the mirror
        ga = G.GGMLGraphAllocator(device="host", defaultBufferSize=16)
        ts = []
        for t in (ta, tb):
            if t.data:
                raw = np.ctypeslib.as_array((np.ctypeslib.ctypes.c_uint8 * t.buf_bytes).from_address(t.data)).copy()
                bid = ga.addBuffer(raw.size)
                ga.buffers[bid][:] = raw
            else:
                bid = -1
            ts.append(G.GGMLTensor(G.GGMLType(t.type), [t.ne[0], t.ne[1]], bufferId=bid))
        with pytest.raises(exc[want]):
            G.computeDotProductMatrix(kind, ga, ts[0], ts[1], K)
