"""K-quant dots Q2_K / Q4_K / Q8_K x F32 (core/GGMLComputeOps.kt:152-432,
dispatched at :1483-1514).

Pinning: the reference has no known-answer test for these dots (its K-quant tests cover
quantize/dequantize accuracy only, T/core/GGMLKQuantAccuracyTest.kt), so the C oracle is
cross-checked against an independent Python restatement (tests/_kquant.py) on random
super-blocks: bit-exact, since both accumulate left to right in f32 — parity with the
reference itself is unpinned. The GPU path must match the oracle within the §8c F32 bar."""
import numpy as np
import pytest

import oracle as O
from _kquant import BB, Q2_K, Q4_K, Q8_K, mat_mul_kq_ref, random_kblocks
from _util import acc_noise, parity_ok, random_acts

KQ = [Q2_K, Q4_K, Q8_K]
KNAME = {Q2_K: "Q2_K", Q4_K: "Q4_K", Q8_K: "Q8_K"}
# K % 256 != 0 exercises the full-block quirk (rows after the first read a block that does not
# start at their k) and the flat-index partial path
SMALL = [(4, 256, 1), (3, 512, 2), (8, 320, 1), (2, 768, 3), (16, 64, 1)]


def _x(K, N, seed):
    return random_acts(K * N, seed).reshape(K, N)


@pytest.mark.parametrize("qt", KQ, ids=lambda t: KNAME[t])
@pytest.mark.parametrize("shape", SMALL, ids=lambda s: "x".join(map(str, s)))
def test_oracle_matches_python_restatement(qt, shape):
    M, K, N = shape
    raw = random_kblocks(qt, M * K // 256, seed=M * 7 + K)
    x = _x(K, N, 3 + M)
    got = O.mat_mul_q(qt, raw, M, K, x)
    ref = mat_mul_kq_ref(qt, raw, M, K, x)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


@pytest.mark.parametrize("qt", KQ, ids=lambda t: KNAME[t])
def test_oracle_block_bound_and_dst_type(qt):
    # M*K % 256 != 0: the partial path reaches block numBlocks -> IllegalArgumentException
    raw = random_kblocks(qt, 2, seed=1)
    with pytest.raises(O.OracleError) as e:
        O.mat_mul_q(qt, np.concatenate([raw, np.zeros(BB[qt], np.uint8)]), 3, 200, _x(200, 1, 1))
    assert e.value.status == 1
    a = O.make_tensor(qt, [256, 1], random_kblocks(qt, 1, 2))
    b = O.make_tensor(O.F32, [1, 256], _x(256, 1, 2).view(np.uint8).reshape(-1))
    d = O.make_tensor(O.F16, [1, 1], np.zeros(2, np.uint8))
    assert O.compute_mat_mul(a, b, d) == 1


# K % 256 == 0 runs kquant_gemv_kernel (a wave per row, 1 or 4 columns per wave); N = 5, 9 leave
# a partial column group
GPU_SHAPES = SMALL + [(257, 4096, 1), (64, 11008, 2), (100, 4096, 4), (33, 2048, 5), (7, 1280, 9),
                      (40, 4096, 32), (17, 11008, 7)]


def mfma_path(qt, K, N):
    """Q4_K at 16 <= N <= 32 (K % 256 == 0) runs on the MFMA kernel (lk_skinny.hpp): activations
    split as bf16 hi + lo, weights as the affine q·(scale/15) + min of the Kotlin expression."""
    return qt == Q4_K and 16 <= N <= 32 and K % 256 == 0


def q4k_terms(raw, M, K):
    """|q/15·scale| + |min| per weight of a Q4_K matrix with K % 256 == 0 (numpy, the Kotlin
    expressions of :285-298 op for op in f32): the magnitudes the affine form q·s1 + min adds."""
    b = np.asarray(raw, np.uint8).reshape(-1, 144)
    d = b[:, 0:2].copy().view(np.float16).astype(np.float32)[:, 0]
    dmin = b[:, 2:4].copy().view(np.float16).astype(np.float32)[:, 0]
    sc = b[:, 4:12].astype(np.int32)                                   # scale bytes of sub-blocks 0..7
    mh = np.zeros_like(sc)
    mh[:, :6] = b[:, 5:16:2][:, :6].astype(np.int32) & 0x0F          # byte 4 + 2sb + 1 < 16 for sb <= 5
    scale = (np.float32(1) * (sc & 0x3F).astype(np.float32) / np.float32(63)) * d[:, None]
    qm = ((sc >> 6) & 3) | (mh << 2)
    mn = (qm.astype(np.float32) / np.float32(63)) * d[:, None] + dmin[:, None]
    q = np.stack([b[:, 16:144] & 0x0F, b[:, 16:144] >> 4], axis=-1).reshape(-1, 8, 32).astype(np.float32)
    t = np.abs(q / np.float32(15) * scale[:, :, None]) + np.abs(mn)[:, :, None]
    return t.reshape(M, K)


def kq_noise(qt, raw, M, K, x):
    """The batched-path allowance (tests/_util.py acc_noise with the activation split) taken over
    the affine form's term magnitudes, x4 for the f32 rounding of q·s1 + min against the Kotlin
    expression order (a few ulps of each term)."""
    assert qt == Q4_K
    return 4.0 * acc_noise(q4k_terms(raw, M, K), np.abs(x), split=True)


@pytest.mark.gpu
@pytest.mark.parametrize("qt", KQ, ids=lambda t: KNAME[t])
@pytest.mark.parametrize("shape", GPU_SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_kquant_gpu_vs_oracle(gpu, qt, shape):
    from test_gpu_parity import gpu_matmul
    M, K, N = shape
    raw = random_kblocks(qt, M * K // 256, seed=M + K + N)
    x = _x(K, N, 11 + N)
    ref = O.mat_mul_q(qt, raw, M, K, x)
    noise = kq_noise(qt, raw, M, K, x) if mfma_path(qt, K, N) else None
    got = gpu_matmul(qt, raw, M, K, N, x)
    ok, msg = parity_ok(got, ref, noise=noise)
    assert ok, msg
    got = gpu_matmul(qt, raw, M, K, N, x, host=True, dst_row_pad=2)
    ok, msg = parity_ok(got, ref, noise=noise)
    assert ok, ("host path", msg)


# The Q4_K MFMA path (16 <= N <= 32): ragged rows, K with a half slice at the end (11008 = 43
# blocks: the last slice's second half is empty), one 16-column tile, and bit-equal reruns.
KQ_MFMA = [(257, 4096, 32), (100, 11008, 17), (33, 2048, 16), (1000, 1024, 24), (64, 256, 20)]


@pytest.mark.gpu
@pytest.mark.parametrize("shape", KQ_MFMA, ids=lambda s: "x".join(map(str, s)))
def test_q4_k_mfma_vs_oracle(gpu, shape):
    from test_gpu_parity import gpu_matmul
    M, K, N = shape
    raw = random_kblocks(Q4_K, M * K // 256, seed=7 * M + N)
    x = _x(K, N, 31 + N)
    ref = O.mat_mul_q(Q4_K, raw, M, K, x)
    got = gpu_matmul(Q4_K, raw, M, K, N, x)
    ok, msg = parity_ok(got, ref, noise=kq_noise(Q4_K, raw, M, K, x))
    assert ok, msg
    again = gpu_matmul(Q4_K, raw, M, K, N, x)
    assert np.array_equal(got.view(np.uint32), again.view(np.uint32)), "not deterministic"


@pytest.mark.gpu
@pytest.mark.parametrize("qt", KQ, ids=lambda t: KNAME[t])
@pytest.mark.parametrize("offs", [(2, 0, 0), (0, 4, 0), (1, 8, 4)], ids=lambda o: "a%d-b%d-d%d" % o)
def test_kquant_gpu_unaligned_operands(gpu, qt, offs):
    """Byte-offset weights (the word-load variant needs a 4-aligned block base) and
    activations off 16 B (no float4 loads) take the byte-load / scalar variants."""
    from test_gpu_parity import gpu_matmul
    a_off, b_off, d_off = offs
    for (M, K, N) in ((19, 1024, 1), (6, 768, 3)):
        raw = random_kblocks(qt, M * K // 256, seed=M + a_off)
        x = _x(K, N, 5 + b_off)
        ref = O.mat_mul_q(qt, raw, M, K, x)
        got = gpu_matmul(qt, raw, M, K, N, x, a_off=a_off, b_off=b_off, d_off=d_off)
        ok, msg = parity_ok(got, ref)
        assert ok, (M, K, N, msg)
    # a column-strided activation view at N = 1 (k stride != 4)
    raw = random_kblocks(qt, 4 * 512 // 256, seed=9)
    x = _x(512, 1, 9)
    got = gpu_matmul(qt, raw, 4, 512, 1, x, b_stride=3)
    ok, msg = parity_ok(got, O.mat_mul_q(qt, raw, 4, 512, x))
    assert ok, msg


@pytest.mark.gpu
@pytest.mark.parametrize("qt", KQ, ids=lambda t: KNAME[t])
@pytest.mark.parametrize("K", [1024, 2816])
def test_kquant_gpu_weights_bit_exact(gpu, qt, K):
    """One-hot activations turn every output into one weight (x·1 plus exact zeros, any order),
    so the GPU's decoded weights are compared bit for bit with the oracle's Kotlin-order
    values: a contraction or a different quotient would show here, not only a tolerance."""
    from test_gpu_parity import gpu_matmul
    M = 48
    raw = random_kblocks(qt, M * K // 256, seed=K + qt)
    for k in (0, 37, 255, 256 + 129, K - 1):
        x = np.zeros((K, 1), np.float32)
        x[k, 0] = 1.0
        ref = O.mat_mul_q(qt, raw, M, K, x)
        got = gpu_matmul(qt, raw, M, K, 1, x)
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), k
    # batch > 1 (kquant_nc_kernel): column n one-hot at its own k
    ks = [3, 300, K - 2, 130, 511, 77, K // 2, 1, 1000]
    x = np.zeros((K, len(ks)), np.float32)
    x[ks, np.arange(len(ks))] = 1.0
    ref = O.mat_mul_q(qt, raw, M, K, x)
    got = gpu_matmul(qt, raw, M, K, len(ks), x)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("qt", KQ, ids=lambda t: KNAME[t])
def test_kquant_gpu_errors_like_oracle(gpu, qt):
    import ggml_hip as G
    raw = np.concatenate([random_kblocks(qt, 2, seed=5), np.zeros(BB[qt], np.uint8)])
    ga = G.GGMLGraphAllocator(device="cuda", defaultBufferSize=16)
    ia, ib, idd = ga.addBuffer(raw.size + 64), ga.addBuffer(4 * 200 + 64), ga.addBuffer(64)
    a = G.GGMLTensor(G.GGMLType(qt), [200, 3], bufferId=ia)
    b = G.GGMLTensor(G.GGMLType.F32, [1, 200], bufferId=ib)
    d = G.GGMLTensor(G.GGMLType.F32, [1, 3], bufferId=idd)
    ga.setTensorBytes(a, raw)
    with pytest.raises(G.IllegalArgumentException):  # M*K % 256 != 0: block numBlocks is read
        G.computeMatMul(ga, ga.context, a, b, d)
    a2 = G.GGMLTensor(G.GGMLType(qt), [256, 1], bufferId=ia)
    b2 = G.GGMLTensor(G.GGMLType.F32, [1, 256], bufferId=ga.addBuffer(4 * 256))
    with pytest.raises(G.IllegalArgumentException):  # dst must be F32 (:1484, :1495, :1506)
        G.computeMatMul(ga, ga.context, a2, b2, G.GGMLTensor(G.GGMLType.F16, [1, 1], bufferId=idd))
    short = G.GGMLTensor(G.GGMLType(qt), [256, 1], bufferId=ga.addBuffer(BB[qt] - 4))
    with pytest.raises(G.IndexOutOfBoundsException):  # the block runs past the buffer
        G.computeMatMul(ga, ga.context, short, b2, G.GGMLTensor(G.GGMLType.F32, [1, 1], bufferId=idd))


# Q4_K at batch 1 runs on the LDS-DMA stream kernel (gemv_stream_kernel<Q4_K>, units of 16
# blocks) when A and x are 16-byte aligned and K <= 12288: one, two and three units per row,
# a partial last unit (11008 = 43 blocks), ragged and tiny row counts, fewer rows than waves.
Q4K_STREAM = [(11008, 4096, 1), (4096, 11008, 1), (300, 8192, 1), (3, 12288, 1), (5, 256, 1), (129, 2816, 1),
              (2049, 1024, 1)]


@pytest.mark.gpu
@pytest.mark.parametrize("shape", Q4K_STREAM, ids=lambda s: "x".join(map(str, s)))
def test_q4_k_stream_vs_oracle(gpu, shape):
    from test_gpu_parity import gpu_matmul
    M, K, N = shape
    raw = random_kblocks(Q4_K, M * K // 256, seed=3 * M + K)
    x = _x(K, N, 17 + M)
    ref = O.mat_mul_q(Q4_K, raw, M, K, x)
    got = gpu_matmul(Q4_K, raw, M, K, N, x)
    ok, msg = parity_ok(got, ref)
    assert ok, msg
    again = gpu_matmul(Q4_K, raw, M, K, N, x)
    assert np.array_equal(got.view(np.uint32), again.view(np.uint32)), "not deterministic"


@pytest.mark.gpu
@pytest.mark.parametrize("K", [8192, 11008])
def test_q4_k_stream_weights_bit_exact(gpu, K):
    """One-hot activations through the stream kernel's Q4_K units (2 and 3 units per row, the
    last one partial at 11008): every output is one Kotlin weight, bit for bit."""
    from test_gpu_parity import gpu_matmul
    M = 40
    raw = random_kblocks(Q4_K, M * K // 256, seed=K + 1)
    for k in (0, 63, 64, 4095, 4096 + 200, K - 257, K - 1):
        x = np.zeros((K, 1), np.float32)
        x[k, 0] = 1.0
        ref = O.mat_mul_q(Q4_K, raw, M, K, x)
        got = gpu_matmul(Q4_K, raw, M, K, 1, x)
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), k


@pytest.mark.gpu
def test_q4_k_plan_and_chain_equal_single_launches(gpu):
    """Q4_K nodes in lk_plan (independent nodes, one grouped launch) and lk_plan_create_chain
    (dependent stages, one persistent launch): bit-identical to single launches, which match the
    oracle; the Llama-7B-like stage shapes {q,k,v} -> o -> {gate, up} -> down."""
    import torch
    import ggml_hip as G
    ga = G.GGMLGraphAllocator(device="cuda", defaultBufferSize=16)
    dims, fanout = [4096, 4096, 4096, 11008, 4096], [3, 1, 2, 1]
    xb = ga.addBuffer(4 * dims[0] + 64)
    x = G.GGMLTensor(G.GGMLType.F32, [1, dims[0]], bufferId=xb)
    ga.setTensorBytes(x, random_acts(dims[0], 5).view(np.uint8))
    nodes, stages, host_w, cur = [], [], [], x
    for s in range(len(dims) - 1):
        K, M = dims[s], dims[s + 1]
        first = None
        for f in range(fanout[s]):
            raw = random_kblocks(Q4_K, M * K // 256, seed=100 + 10 * s + f)
            a = G.GGMLTensor(G.GGMLType.Q4_K, [K, M], bufferId=ga.addBuffer(raw.size))
            ga.setTensorBytes(a, raw)
            d = G.GGMLTensor(G.GGMLType.F32, [1, M], bufferId=ga.addBuffer(4 * M + 64))
            nodes.append((a, cur, d))
            stages.append(s)
            host_w.append((raw, M, K))
            if first is None:
                first = d
        cur = first
    for (a, b, d) in nodes:
        G.computeMatMul(ga, ga.context, a, b, d)
    torch.cuda.synchronize()
    ref = [ga.tensorBytes(d).cpu().numpy().view(np.float32).copy() for (_, _, d) in nodes]
    xin = ga.tensorBytes(x).cpu().numpy().view(np.float32).copy()
    for i in range(fanout[0]):  # the first stage against the oracle
        raw, M, K = host_w[i]
        ok, msg = parity_ok(ref[i].reshape(-1, 1), O.mat_mul_q(Q4_K, raw, M, K, xin.reshape(K, 1)))
        assert ok, (i, msg)
    # stage 0's independent nodes as one grouped launch
    plan = G.MulMatPlan(ga, nodes[:fanout[0]])
    assert plan.numLaunches == 1
    for (_, _, d) in nodes[:fanout[0]]:
        ga.tensorBytes(d).fill_(0xFF)
    plan.launch()
    torch.cuda.synchronize()
    for i in range(fanout[0]):
        got = ga.tensorBytes(nodes[i][2]).cpu().numpy().view(np.float32)
        assert np.array_equal(got.view(np.uint32), ref[i].view(np.uint32)), i
    # the whole chain in one launch, twice (the barrier counters re-arm)
    chain = G.MulMatPlan(ga, nodes, stages=stages)
    assert chain.numLaunches == 1
    for rep in range(2):
        for (_, _, d) in nodes:
            ga.tensorBytes(d).fill_(0xFF)
        chain.launch()
        torch.cuda.synchronize()
        assert not chain.timedOut()
        for i, (_, _, d) in enumerate(nodes):
            got = ga.tensorBytes(d).cpu().numpy().view(np.float32)
            assert np.array_equal(got.view(np.uint32), ref[i].view(np.uint32)), (rep, i, stages[i])


# Q2_K at batch 1 on the stream kernel too (its rows are whole 16-byte DMA pieces when
# K % 1024 == 0): 1-3 units per row, ragged rows; 11008 stays on kquant_n1_kernel.
Q2K_STREAM = [(11008, 4096, 1), (300, 8192, 1), (3, 12288, 1), (5, 1024, 1), (2049, 1024, 1), (64, 11008, 1)]


@pytest.mark.gpu
@pytest.mark.parametrize("shape", Q2K_STREAM, ids=lambda s: "x".join(map(str, s)))
def test_q2_k_stream_vs_oracle(gpu, shape):
    from test_gpu_parity import gpu_matmul
    M, K, N = shape
    raw = random_kblocks(Q2_K, M * K // 256, seed=5 * M + K)
    x = _x(K, N, 23 + M)
    ref = O.mat_mul_q(Q2_K, raw, M, K, x)
    got = gpu_matmul(Q2_K, raw, M, K, N, x)
    ok, msg = parity_ok(got, ref)
    assert ok, msg


@pytest.mark.gpu
@pytest.mark.parametrize("K", [4096, 12288])
def test_q2_k_stream_weights_bit_exact(gpu, K):
    """One-hot activations through the stream kernel's Q2_K units: every output is one Kotlin
    weight, bit for bit (the FMA-corrected quotient by 3 included)."""
    from test_gpu_parity import gpu_matmul
    M = 40
    raw = random_kblocks(Q2_K, M * K // 256, seed=K + 2)
    for k in (0, 5, 15, 16, 63, 64, 255, 4095, K - 17, K - 1):
        x = np.zeros((K, 1), np.float32)
        x[k, 0] = 1.0
        ref = O.mat_mul_q(Q2_K, raw, M, K, x)
        got = gpu_matmul(Q2_K, raw, M, K, 1, x)
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), k
