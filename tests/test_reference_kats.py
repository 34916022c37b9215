"""Known-answer tests the reference holds for this path, restated as data and run twice: on the
oracle (CPU, pins the restatement) and through the HIP C-ABI (-m gpu, the product).

Sources (T/ = src/nativeTest/kotlin/ai/solace/llamakotlin/):
  * T/core/GGMLIntegrationTest.kt:158-196  testMatrixMultiplicationChain — (I·I) + 0.1 on 4x4 F32:
    diagonal 1.1, elsewhere 0.1, tolerance 1e-3.
  * T/core/GGMLIntegrationTest.kt:200-240  testQuantizedOperationChain — sin(0.1i) through Q8_0 and
    cos(0.1i) through Q4_0 (64 elements), dequantized, added, multiplied by the first, re-quantized
    to Q8_0 and dequantized: within 0.1 of (sin + cos)·sin for i < 10.
  * T/core/GGMLReferenceValidationTest.kt:160-175 (checked by :303-316) — Q8_0 quantize/dequantize of
    0.1 + 2cos(i), 32 elements: an element fails only if |err| > 0.01 AND |err|/|x| > 0.01.

The ADD / MUL steps of the chains are the reference tests' own glue (computeAdd / computeMul, not
on the MUL_MAT path): they are plain f32 numpy here. Quantize / dequantize / computeMatMul are the
oracle's restatement on CPU and the library's kernels on the GPU.
"""
import numpy as np
import pytest


def _identity_chain(matmul):
    n = 4
    ident = np.array([1.0 if i % (n + 1) == 0 else 0.0 for i in range(n * n)], np.float32)  # :165-167
    ones = np.full(n * n, 0.1, np.float32)                                                  # :168
    prod = matmul(ident, ident, n, n, n).reshape(-1)
    out = (prod + ones).astype(np.float32)                                                  # computeAdd
    want = np.array([1.1 if i == j else 0.1 for i in range(n) for j in range(n)], np.float32)
    assert np.all(np.abs(out - want) <= 1e-3), out                                          # :183-190


def _quantized_chain(quant, dequant):
    i = np.arange(64, dtype=np.float32)
    d1 = np.sin(i * np.float32(0.1)).astype(np.float32)                                     # :204
    d2 = np.cos(i * np.float32(0.1)).astype(np.float32)                                     # :205
    deq1 = dequant(6, quant(6, d1), 64)                                                     # Q8_0 :212, :216
    deq2 = dequant(2, quant(2, d2), 64)                                                     # Q4_0 :213, :217
    add = (deq1 + deq2).astype(np.float32)                                                  # computeAdd :220
    mul = (add * deq1).astype(np.float32)                                                   # computeMul :221
    fin = dequant(6, quant(6, mul), 64)                                                     # :224-225
    for k in range(10):                                                                     # :230-234
        expected = (np.sin(np.float32(k * 0.1)) + np.cos(np.float32(k * 0.1))) * np.sin(np.float32(k * 0.1))
        assert abs(expected - fin[k]) < 0.1, (k, expected, fin[k])
    return fin


def _q8_0_roundtrip(quant, dequant):
    x = (np.float32(0.1) + np.float32(2.0) * np.cos(np.arange(32, dtype=np.float32))).astype(np.float32)  # :162
    got = dequant(6, quant(6, x), 32)
    err = np.abs(x.astype(np.float64) - got.astype(np.float64))
    rel = np.where(np.abs(x) > 1e-10, err / np.abs(x.astype(np.float64)), err)
    failed = np.nonzero((err > 0.01) & (rel > 0.01))[0]                                      # :313-315
    assert failed.size == 0, (failed, err.max())
    return got


# ---- the oracle (CPU) ------------------------------------------------------------------------

def _oracle_f32mm(O):
    def mm(a, b, M, K, N):
        return O.mat_mul_q(O.F32, np.asarray(a, np.float32).view(np.uint8), M, K, np.asarray(b, np.float32).reshape(K, N))
    return mm


def test_matrix_multiplication_chain_oracle(oracle):
    _identity_chain(_oracle_f32mm(oracle))


def test_quantized_operation_chain_oracle(oracle):
    _quantized_chain(oracle.quantize, oracle.dequantize)


def test_q8_0_reference_roundtrip_oracle(oracle):
    _q8_0_roundtrip(oracle.quantize, oracle.dequantize)


# ---- the HIP path (C-ABI) --------------------------------------------------------------------

def _gpu_f32mm(a, b, M, K, N):
    import ggml_hip as G
    ga = G.GGMLGraphAllocator(defaultBufferSize=4 * (M * K + K * N + M * N) + 256)
    ta = ga.allocateTensor(G.GGMLType.F32, [K, M]); ga.setTensorBytes(ta, np.asarray(a, np.float32))
    tb = ga.allocateTensor(G.GGMLType.F32, [N, K]); ga.setTensorBytes(tb, np.asarray(b, np.float32))
    td = ga.allocateTensor(G.GGMLType.F32, [N, M])
    G.computeMatMul(ga, ga.context, ta, tb, td)
    return ga.tensorBytes(td).cpu().numpy().view(np.float32).reshape(M, N).copy()


def _gpu_quant(qt, x):
    import torch
    import ggml_hip as G
    return G.quantizeTensor(torch.from_numpy(np.ascontiguousarray(x, np.float32)).cuda(), G.GGMLType(qt)).cpu().numpy()


def _gpu_dequant(qt, q, n):
    import ggml_hip as G
    ga = G.GGMLGraphAllocator(defaultBufferSize=q.size + 64)
    t = ga.allocateTensor(G.GGMLType(qt), [n])
    ga.setTensorBytes(t, q)
    return G.dequantizeTensor(ga, t).cpu().numpy().astype(np.float32)


@pytest.mark.gpu
def test_matrix_multiplication_chain_gpu(gpu, oracle):
    _identity_chain(_gpu_f32mm)


@pytest.mark.gpu
def test_quantized_operation_chain_gpu(gpu, oracle):
    got = _quantized_chain(_gpu_quant, _gpu_dequant)
    # and the same bytes as the restatement at every step (quantize / dequantize are bit-exact)
    assert np.array_equal(got.view(np.uint32), _quantized_chain(oracle.quantize, oracle.dequantize).view(np.uint32))


@pytest.mark.gpu
def test_q8_0_reference_roundtrip_gpu(gpu, oracle):
    got = _q8_0_roundtrip(_gpu_quant, _gpu_dequant)
    assert np.array_equal(got.view(np.uint32), _q8_0_roundtrip(oracle.quantize, oracle.dequantize).view(np.uint32))
