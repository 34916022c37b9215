"""Committed fixtures (tests/golden/*.npz, made by tests/golden/make_golden.py)."""
import glob
import os

import numpy as np
import pytest

from _util import parity_ok

HERE = os.path.dirname(os.path.abspath(__file__))
FILES = sorted(glob.glob(os.path.join(HERE, "golden", "*.npz")))


def load(path):
    with np.load(path, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def test_fixtures_present():
    assert len(FILES) >= 10


@pytest.mark.parametrize("path", FILES, ids=lambda p: os.path.basename(p)[:-4])
def test_oracle_reproduces_fixture(oracle, path):
    """The restatement still produces the committed bytes and outputs bit for bit."""
    d = load(path)
    qt, M, K = int(d["type"]), int(d["M"]), int(d["K"])
    if qt != oracle.F32:
        assert np.array_equal(oracle.quantize(qt, d["src"]), d["a"])
    out = oracle.mat_mul_q(qt, d["a"], M, K, d["b"])
    assert np.array_equal(out.view(np.uint32), d["dst"].view(np.uint32))


def test_kat_fixtures_hold_reference_values():
    f = load(os.path.join(HERE, "golden", "f32_kat_2x3x2.npz"))
    np.testing.assert_allclose(f["dst"].reshape(-1), [58, 64, 139, 154], atol=1e-3)
    q = load(os.path.join(HERE, "golden", "q8_0_kat_2x32x2.npz"))
    np.testing.assert_allclose(q["dst"], [[58, 64], [733, 802]], atol=2.0)


@pytest.mark.gpu
@pytest.mark.parametrize("path", FILES, ids=lambda p: os.path.basename(p)[:-4])
def test_gpu_matches_fixture(gpu, path):
    from test_gpu_parity import gpu_matmul
    d = load(path)
    qt, M, K, N = int(d["type"]), int(d["M"]), int(d["K"]), int(d["N"])
    if qt == 0:
        import ggml_hip as G
        ga = G.GGMLGraphAllocator(defaultBufferSize=1 << 16)
        ta = ga.allocateTensor(G.GGMLType.F32, [K, M]); ga.setTensorBytes(ta, d["a"])
        tb = ga.allocateTensor(G.GGMLType.F32, [N, K]); ga.setTensorBytes(tb, d["b"])
        td = ga.allocateTensor(G.GGMLType.F32, [N, M])
        G.computeMatMul(ga, ga.context, ta, tb, td)
        got = ga.tensorBytes(td).cpu().numpy().view(np.float32).reshape(M, N)
        noise = None
    else:
        import oracle as O
        from test_gpu_parity import noise_for
        got = gpu_matmul(qt, d["a"], M, K, N, d["b"])
        noise = noise_for(O, qt, d["a"], M, K, d["b"]) if K % 32 == 0 else None
    ok, msg = parity_ok(got, d["dst"], noise=noise)
    assert ok, msg
