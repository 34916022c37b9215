"""Pin the CPU restatement (oracle/) against the reference's own known-answer tests.

The Kotlin/Native reference cannot be built or run here, so these
KATs and thresholds — copied as DATA from the reference's test files cited per test —
plus IEEE f16 conversion are what pin the oracle. Paths are relative to
src/nativeTest/kotlin/ai/solace/llamakotlin/ (T/) and src/nativeMain/... (K/).
"""
import math

import numpy as np
import pytest

from _util import pattern_f32, pattern_src


def f32mm(O, a, b, M, K, N):
    return O.mat_mul_q(O.F32, np.asarray(a, np.float32).view(np.uint8), M, K, np.asarray(b, np.float32).reshape(K, N))


def test_destination_matmul_kat(oracle):
    """T/core/GGMLComputeOpsDestinationTest.kt:218-265: 2x3 . 3x2 -> [58,64,139,154], tol 1e-3."""
    out = f32mm(oracle, [1, 2, 3, 4, 5, 6], [7, 8, 9, 10, 11, 12], 2, 3, 2)
    np.testing.assert_allclose(out.reshape(-1), [58, 64, 139, 154], atol=1e-3)


def test_test_tensor_ops_4x4(oracle):
    """K/core/TestTensorOps.kt:122-168: a[i,j]=4i+j, b[i,j]=4i+j+1, tol 1e-4."""
    a = np.array([[4 * i + j for j in range(4)] for i in range(4)], np.float32)
    b = np.array([[4 * i + j + 1 for j in range(4)] for i in range(4)], np.float32)
    out = f32mm(oracle, a, b, 4, 4, 4)
    np.testing.assert_allclose(out, a @ b, atol=1e-4)


def test_q80_matmul_kat_block_aligned(oracle):
    """T/core/GGMLComputeOpsTest.kt:373-433 (Q8_0 x F32 -> [[58,64],[733,802]], delta 2.0),
    re-shaped to K=32 (the original K=3 is not block-aligned, so the stale test cannot run):
    the 3 original columns plus zero padding."""
    K = 32
    a = np.zeros((2, K), np.float32)
    a[0, :3] = [1, 2, 3]
    a[1, :3] = [4, 5, 60]
    b = np.zeros((K, 2), np.float32)
    b[:3] = [[7, 8], [9, 10], [11, 12]]
    q = oracle.quantize(oracle.Q8_0, a.reshape(-1))
    out = oracle.mat_mul_q(oracle.Q8_0, q, 2, K, b)
    np.testing.assert_allclose(out, [[58, 64], [733, 802]], atol=2.0)


def test_q_vs_dequantized_fallback(oracle):
    """T/core/GGMLMatMulOptimizationTest.kt:232-357: quantized path vs dequantize-then-F32 path
    agree within 1e-3 (shapes M<=8, K=32..128)."""
    for qt in (oracle.Q4_0, oracle.Q4_1, oracle.Q8_0):
        for (M, K, N) in [(4, 64, 3), (3, 64, 4), (2, 32, 2), (8, 128, 5)]:
            src = pattern_f32(M * K, 42)
            q = oracle.quantize(qt, src)
            deq = oracle.dequantize(qt, q, M * K)
            x = pattern_f32(K * N, 84).reshape(K, N)
            opt = oracle.mat_mul_q(qt, q, M, K, x)
            fb = f32mm(oracle, deq, x, M, K, N)
            assert np.max(np.abs(opt - fb)) < 1e-3


def test_dot_product_accuracy(oracle):
    """T/core/GGMLStandardizedQuantizationTest.kt:363-395: Q8_0 x F32 dot of 0.1+2cos(i+off),
    size 128, rel err < MAX_DOT_PRODUCT_ERROR = 0.02 (:31)."""
    n = 128
    i = np.arange(n, dtype=np.float32)
    v1 = (np.float32(0.1) + np.float32(2.0) * np.cos(i)).astype(np.float32)
    v2 = (np.float32(0.1) + np.float32(2.0) * np.cos(i + np.float32(1.0))).astype(np.float32)
    ref = float(np.sum(v1.astype(np.float64) * v2.astype(np.float64)))
    q = oracle.quantize(oracle.Q8_0, v1)
    got = float(oracle.mat_mul_q(oracle.Q8_0, q, 1, n, v2.reshape(n, 1))[0, 0])
    assert abs(ref - got) / abs(ref) < 0.02


def _metrics(orig, deq):
    e = orig.astype(np.float64) - deq.astype(np.float64)
    mse = float(np.mean(e * e))
    mad = float(np.mean(np.abs(e)))
    so = float(np.sum(orig.astype(np.float64) ** 2))
    snr = math.inf if np.sum(e * e) == 0 else 10 * math.log10(so / float(np.sum(e * e)))
    return mse, mad, snr


def _accuracy_data(qt):
    """Data of T/core/GGMLQuantizationAccuracyTest.kt:202-392 (4 blocks each)."""
    out = np.zeros(128, np.float32)
    for i in range(128):
        if qt == 6:  # :203-215
            if i % 32 == 0: v = 0.0
            elif i % 32 == 1: v = 127.0
            elif i % 32 == 2: v = -128.0
            elif i < 32: v = (i / 31.0) * 10.0
            elif i < 64: v = ((i - 32) / 31.0) * -10.0
            elif i < 96: v = 50.5 if i % 2 == 0 else -50.5
            else: v = (i - 96) * 0.1 - 1.0
        elif qt == 2:  # :264-276
            if i % 32 == 0: v = 0.0
            elif i % 32 == 1: v = 7.0
            elif i % 32 == 2: v = -8.0
            elif i < 32: v = (i / 31.0) * 1.0
            elif i < 64: v = ((i - 32) / 31.0) * -1.0
            elif i < 96: v = 0.75 if i % 2 == 0 else -0.75
            else: v = ((i - 96) / 31.0 * 16.0) - 8.0
        else:  # :336-347
            b, w = divmod(i, 32)
            if b == 0: v = (w / 31.0) * 2.0 - 1.0
            elif b == 1: v = (w / 31.0) * 0.5 + 0.25
            elif b == 2: v = 5.0 if w % 2 == 0 else 4.0
            else: v = (w - 16) * 0.1
        out[i] = np.float32(v)
    return out


def _numpy_q8_0_roundtrip(x):
    """Independent numpy restatement of quantizeTensor/dequantizeTensor Q8_0
    (K/core/GGMLComputeOps.kt:1063-1071, :929-935) for cross-checking the C oracle."""
    out = []
    for b in range(x.size // 32):
        blk = x[b * 32:(b + 1) * 32]
        amax = np.float32(np.max(np.abs(blk)))
        scale = np.float32(1.0) if amax == 0 else np.float32(amax / np.float32(127.0))
        inv = np.float32(np.float32(1.0) / scale)
        q = np.clip(np.rint((blk * inv).astype(np.float32)), -128, 127).astype(np.float32)
        out.append((np.float32(np.float16(scale)) * q).astype(np.float32))
    return np.concatenate(out)


def _numpy_q4_0_roundtrip(x):
    """Independent numpy restatement of Q4_0 quantize/dequantize (K/core/GGMLComputeOps.kt:1073-1087,
    :936-943): d = amax/8, q = round(x*(1/d) + 8) clamped to [0,15], w = d*(q-8)."""
    out = []
    for b in range(x.size // 32):
        blk = x[b * 32:(b + 1) * 32]
        amax = np.float32(np.max(np.abs(blk)))
        s = np.float32(1.0) if amax == 0 else np.float32(amax / np.float32(8.0))
        inv = np.float32(np.float32(1.0) / s)
        q = np.clip(np.rint(((blk * inv).astype(np.float32) + np.float32(8)).astype(np.float32)), 0, 15)
        out.append((np.float32(np.float16(s)) * (q.astype(np.float32) - np.float32(8))).astype(np.float32))
    return np.concatenate(out)


# (type, reference MSE bound, reference MAD bound, restated MSE, restated MAD)
_ACC = [(6, 0.05, 0.2, 0.0595055, 0.1940099), (2, 0.02, 0.25, 0.0805380, 0.2403604), (3, 0.015, 0.1, None, None)]


@pytest.mark.parametrize("qt,mse_t,mad_t,mse_r,mad_r", _ACC)
def test_quantization_accuracy_thresholds(oracle, qt, mse_t, mad_t, mse_r, mad_r):
    """T/core/GGMLQuantizationAccuracyTest.kt:248-256 / :308-317 / :385-390.

    Finding: the reference's own MSE bounds for Q8_0 (0.05, :248) and Q4_0 (0.02, :308) are
    NOT met by the reference's quantizer on the tests' own data — 0.0595 and 0.0805, from this
    restatement AND from independent numpy restatements (Q4_0's amax/8 scale clamps +amax to
    q=15, i.e. 7/8 amax). The Kotlin native tests are disabled (build.gradle.kts:84-104), so
    this never surfaced. The MAD bounds hold; Q4_1 meets both bounds."""
    x = _accuracy_data(qt)
    deq = oracle.dequantize(qt, oracle.quantize(qt, x), x.size)
    mse, mad, _ = _metrics(x, deq)
    if qt == 6:
        assert np.array_equal(deq, _numpy_q8_0_roundtrip(x))
    if qt == 2:
        assert np.array_equal(deq, _numpy_q4_0_roundtrip(x))
    assert mad < mad_t, mad
    if mse_r is None:
        assert mse < mse_t, mse
    else:
        assert abs(mse - mse_r) < 1e-6 and abs(mad - mad_r) < 1e-6, (mse, mad)


@pytest.mark.parametrize("qt,n,mse_t,mad_t,snr_t", [(6, 512, 1e-4, 0.01, 40.0), (2, 512, 0.01, 0.2, 20.0),
                                                    (3, 384, 0.015, 0.1, 18.0)])
def test_standardized_synthetic(oracle, qt, n, mse_t, mad_t, snr_t):
    """T/core/GGMLStandardizedQuantizationTest.kt:188-301 on 0.1+2cos(i) (:64-68).
    Finding: Q4_0's MSE is 0.01083 against the test's 0.01 bound (MAD and SNR hold); the
    independent numpy restatement gives the same bytes."""
    i = np.arange(n, dtype=np.float32)
    x = (np.float32(0.1) + np.float32(2.0) * np.cos(i)).astype(np.float32)
    deq = oracle.dequantize(qt, oracle.quantize(qt, x), n)
    mse, mad, snr = _metrics(x, deq)
    assert mad < mad_t and snr >= snr_t, (mse, mad, snr)
    if qt == 2:
        assert np.array_equal(deq, _numpy_q4_0_roundtrip(x))
        assert abs(mse - 0.0108303) < 1e-6
    else:
        assert mse < mse_t, mse


def test_half_to_float_exhaustive(oracle):
    """K/core/NumericConversions.kt:9-54 equals IEEE f16->f32 for all 65536 inputs (NaN: NaN)."""
    h = np.arange(65536, dtype=np.uint16)
    got = oracle.half_to_float(h)
    ref = h.view(np.float16).astype(np.float32)
    nan = np.isnan(ref)
    assert np.array_equal(got[~nan].view(np.uint32), ref[~nan].view(np.uint32))
    assert np.all(np.isnan(got[nan]))


def test_float_to_half_normal_range_is_ieee_rne(oracle):
    """K/core/NumericConversions.kt:61-124 rounds to nearest-even exactly like IEEE for
    |x| in [2^-14, 65504] (all normal f16 outputs), checked on 2M random values + boundaries."""
    rng = np.random.default_rng(1)
    x = (rng.uniform(-1, 1, 2_000_000) * np.exp2(rng.uniform(-14, 16, 2_000_000))).astype(np.float32)
    x = x[(np.abs(x) >= 2.0 ** -14) & (np.abs(x) <= 65504)]
    assert np.array_equal(oracle.float_to_half(x), x.astype(np.float16).view(np.uint16))


def test_float_to_half_reference_quirks(oracle):
    """Behaviours of the Kotlin code that differ from IEEE, restated on purpose:
    the denormal branch shifts one bit too far (result = rint(|x|*2^23) instead of |x|*2^24),
    shift counts are masked to 5 bits (2^-31.5 -> min denormal), and |x| in [65536, ~131008]
    takes the normal branch with exponent 31 (NaN/Inf bit patterns)."""
    f = lambda v: int(oracle.float_to_half(np.array([v], np.float32))[0])
    assert f(2.0 ** -20) == 0x0008          # IEEE: 0x0010
    assert f(2.0 ** -31.5) == 0x0001        # IEEE: 0x0000 (shift 32 masked to 0)
    assert f(2.0 ** -33) == 0x0000
    assert f(65519.0) == 0x7BFF and f(65520.0) == 0x7C00
    assert f(70000.0) == 0x7C46             # exponent-31 pattern with mantissa (a NaN)
    assert f(1e6) == 0x7E00 and f(float("inf")) == 0x7C00 and f(float("nan")) == 0x7E00
    assert f(-0.0) == 0x8000 and f(0.0) == 0


def test_tight_equals_structural(oracle):
    """The 'tight' CPU baseline keeps the structural path's arithmetic order: bit-identical."""
    for qt in (oracle.Q4_0, oracle.Q4_1, oracle.Q8_0):
        M, K, N = 6, 96, 3
        q = oracle.quantize(qt, pattern_src(qt, M * K, 42) * np.float32(0.37))
        x = pattern_f32(K * N, 84).reshape(K, N)
        a = oracle.mat_mul_q(qt, q, M, K, x)
        b = oracle.mat_mul_q(qt, q, M, K, x, tight=True)
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


def test_error_behaviour(oracle):
    """computeMatMul's exceptions (K/core/GGMLComputeOps.kt:1440, :1444, :1449, :1530, :1563;
    accessors K/core/GGMLTypes.kt:361-367, :598-617) as lk_status codes."""
    O = oracle
    M, K, N = 2, 32, 1
    qa = O.quantize(O.Q4_0, pattern_src(O.Q4_0, M * K, 42))
    xb = pattern_f32(K * N, 84).view(np.uint8).copy()
    d = np.zeros(64, np.uint8)
    A = lambda **kw: O.make_tensor(kw.get("t", O.Q4_0), kw.get("ne", [K, M]), kw.get("buf", qa))
    B = lambda **kw: O.make_tensor(O.F32, kw.get("ne", [N, K]), kw.get("buf", xb))
    D = lambda **kw: O.make_tensor(kw.get("t", O.F32), kw.get("ne", [N, M]), kw.get("buf", d))
    assert O.compute_mat_mul(A(), B(), D()) == 0
    assert O.compute_mat_mul(A(), B(ne=[N, K + 32]), D()) == 1           # K mismatch
    assert O.compute_mat_mul(A(), B(), D(ne=[N + 1, M])) == 1           # dst shape
    assert O.compute_mat_mul(A(), B(), D(t=O.F16)) == 1                 # dst type
    assert O.compute_mat_mul(A(t=O.I32, buf=np.zeros(256, np.uint8)), B(), D(t=O.I32)) == 2  # NotImplementedError
    assert O.compute_mat_mul(A(buf=qa[:20].copy()), B(), D()) == 3      # A too short -> IOOBE
    assert O.compute_mat_mul(A(buf=None), B(), D()) == 4                # missing buffer -> ISE
    assert O.compute_mat_mul(A(), B(), D(buf=np.zeros(4, np.uint8))) == 3
