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
