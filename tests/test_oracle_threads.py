"""The CPU baseline's all-cores line: the tight restatement with rows split over
OpenMP threads is bit-identical to the single-thread tight and structural restatements."""
import numpy as np
import pytest

import oracle as O
from _util import random_acts, random_weights


@pytest.mark.parametrize("qt", [O.Q4_0, O.Q4_1, O.Q8_0], ids=["Q4_0", "Q4_1", "Q8_0"])
@pytest.mark.parametrize("shape", [(100, 256, 1), (37, 1024, 3)], ids=["100x256x1", "37x1024x3"])
def test_tight_threads_bit_identical(qt, shape):
    M, K, N = shape
    q = O.quantize(qt, random_weights(M * K, M + K))
    x = random_acts(K * N, N).reshape(K, N)
    ref = O.mat_mul_q(qt, q, M, K, x)
    for threads in (1, 4, 7):
        got = O.mat_mul_q(qt, q, M, K, x, tight=True, threads=threads)
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), threads
