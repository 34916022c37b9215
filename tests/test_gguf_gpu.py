"""GGUF quantized-tensor loading on the GPU: the nibble repack kernel,
device/host/resident loads of upstream-layout Q4_0/Q4_1/Q8_0 tensors, and computeMatMul
over loaded weights — all bit-exact against oracle/gguf_oracle (repack, upstream
dequantization) and oracle/ (computeMatMul restatement)."""
import ctypes

import numpy as np
import pytest

import gguf_oracle as GO
from _util import parity_ok, random_acts, random_weights

pytestmark = pytest.mark.gpu

UP2LK = {GO.GGML_Q4_0: 2, GO.GGML_Q4_1: 3, GO.GGML_Q8_0: 6}
BB = {GO.GGML_Q4_0: 18, GO.GGML_Q4_1: 20, GO.GGML_Q8_0: 34}


def _model_file(shapes, seed=1):
    """shapes: [(name, upstream type, K, M)] -> (gguf bytes, {name: raw upstream bytes, x})."""
    tensors, raws, off = [], {}, 0
    for i, (name, ft, K, M) in enumerate(shapes):
        x = random_weights(K * M, seed + i)
        raw = GO.upstream_quantize(ft, x) if ft in BB else x.astype(np.float32).tobytes()
        tensors.append((name, [K, M], ft, off, raw))
        raws[name] = raw
        off = (off + len(raw) + 31) // 32 * 32
    data = GO.write_gguf([("general.architecture", GO.STRING, "llama"), ("general.alignment", GO.UINT32, 32)],
                         tensors)
    return data, raws


@pytest.mark.parametrize("ft", [GO.GGML_Q4_0, GO.GGML_Q4_1])
@pytest.mark.parametrize("nblk", [1, 63, 255, 256, 257, 100003])
def test_repack_kernel_bit_exact_and_inverse(gpu, ft, nblk):
    import torch
    from ggml_hip import _lib
    rng = np.random.default_rng(nblk)
    raw = rng.integers(0, 256, nblk * BB[ft], dtype=np.uint8)
    dev = torch.from_numpy(raw.copy()).to(gpu)
    L = _lib.load()
    _lib.check(L.lk_repack_q4_device(ctypes.c_void_p(dev.data_ptr()), nblk, UP2LK[ft], 0, None))
    torch.cuda.synchronize()
    want = np.frombuffer(GO.repack_to_kotlin(ft, raw.tobytes()), np.uint8)
    assert np.array_equal(dev.cpu().numpy(), want)
    _lib.check(L.lk_repack_q4_device(ctypes.c_void_p(dev.data_ptr()), nblk, UP2LK[ft], 1, None))
    torch.cuda.synchronize()
    assert np.array_equal(dev.cpu().numpy(), raw)


def test_repack_rejects(gpu):
    from ggml_hip import _lib
    L = _lib.load()
    assert L.lk_repack_q4_device(None, 4, 6, 0, None) == _lib.LK_ERR_NOT_IMPLEMENTED  # Q8_0: same layout
    assert L.lk_repack_q4_device(None, 4, 2, 7, None) == _lib.LK_ERR_INVALID_ARG
    assert L.lk_repack_q4_device(None, 4, 2, 0, None) == _lib.LK_ERR_NO_BUFFER
    assert L.lk_repack_q4_device(None, 0, 2, 0, None) == _lib.LK_OK


SHAPES = [("blk.0.attn_q.weight", GO.GGML_Q4_0, 256, 70), ("blk.0.ffn_up.weight", GO.GGML_Q4_1, 4352, 9),
          ("blk.0.ffn_down.weight", GO.GGML_Q8_0, 320, 33), ("output_norm.weight", 0, 64, 1),
          ("blk.0.ragged", GO.GGML_Q4_0, 96, 5)]


@pytest.mark.parametrize("mode", ["device", "host", "resident", "file"])
def test_loaded_tensors_match_oracle(gpu, tmp_path, mode):
    """Bytes of every loaded tensor == oracle repack of the stored bytes, and the device
    dequantization of the loaded Q tensors == upstream dequantization of the stored bytes."""
    import ggml_hip as G
    from ggml_hip.gguf import ModelLoader
    data, raws = _model_file(SHAPES)
    if mode == "file":
        p = tmp_path / "m.gguf"
        p.write_bytes(data)
        m = ModelLoader().loadFromFile(str(p))
    else:
        m = ModelLoader().loadFromBytes(data)
    ga = G.GGMLGraphAllocator(device="host" if mode == "host" else "cuda", defaultBufferSize=1 << 16)
    if mode == "resident":
        m.loadResident(ga)
    for name, ft, K, M in SHAPES:
        t = m.getTensor(name, ga)
        assert t.ne[:2] == [K, M]
        raw = raws[name]
        got = np.frombuffer(bytes(ga.readBytes(t.bufferId, t.dataOffset, len(raw))), np.uint8)
        assert np.array_equal(got, np.frombuffer(GO.repack_to_kotlin(ft, raw), np.uint8)), (mode, name)
        if ft in BB and mode != "host":
            deq = G.dequantizeTensor(ga, t).cpu().numpy()
            want = GO.upstream_dequant(ft, raw, K * M)
            assert np.array_equal(deq.view(np.uint32), want.view(np.uint32)), (mode, name)


@pytest.mark.parametrize("name", [s[0] for s in SHAPES if s[1] in BB])
def test_mul_mat_on_loaded_weights(gpu, oracle, name):
    """GGUF -> resident HBM -> computeMatMul: parity with the oracle's computeMatMul on the
    repacked bytes (the weights llama.kotlin would hold after loading)."""
    import torch
    import ggml_hip as G
    from ggml_hip.gguf import ModelLoader
    from test_gpu_parity import noise_for
    data, raws = _model_file(SHAPES)
    m = ModelLoader().loadFromBytes(data)
    ga = G.GGMLGraphAllocator(device="cuda", defaultBufferSize=1 << 16)
    m.loadResident(ga)
    _, ft, K, M = next(s for s in SHAPES if s[0] == name)
    a = m.getTensor(name, ga)
    for N in (1, 3):
        x = random_acts(K * N, 77 + N).reshape(K, N)
        b = ga.allocateTensor(G.GGMLType.F32, [N, K])
        ga.setTensorBytes(b, np.ascontiguousarray(x))
        d = ga.allocateTensor(G.GGMLType.F32, [N, M])
        G.computeMatMul(ga, ga.context, a, b, d)
        torch.cuda.synchronize()
        got = np.frombuffer(bytes(ga.readBytes(d.bufferId, d.dataOffset, M * N * 4)), np.float32).reshape(M, N)
        kot = np.frombuffer(GO.repack_to_kotlin(ft, raws[name]), np.uint8)
        ref = oracle.mat_mul_q(UP2LK[ft], kot, M, K, x)
        ok, msg = parity_ok(got.astype(np.float64), ref, noise=noise_for(oracle, UP2LK[ft], kot, M, K, x))
        assert ok, (name, N, msg)


def test_large_file_staging(gpu, tmp_path):
    """A 4096x4096 Q4_0 weight (9.4 MB > the 4 MB single-copy threshold) through the pinned
    staging path, per tensor and resident."""
    import torch
    import ggml_hip as G
    from ggml_hip.gguf import ModelLoader
    K = M = 4096
    rng = np.random.default_rng(9)
    raw = rng.integers(0, 256, K * M // 32 * 18, dtype=np.uint8)
    raw.reshape(-1, 18)[:, 1] &= 0x3B  # finite f16 scales
    data = GO.write_gguf([], [("w", [K, M], GO.GGML_Q4_0, 0, raw.tobytes())])
    p = tmp_path / "big.gguf"
    p.write_bytes(data)
    m = ModelLoader().loadFromFile(str(p))
    want = torch.from_numpy(np.frombuffer(GO.repack_to_kotlin(GO.GGML_Q4_0, raw.tobytes()), np.uint8).copy())
    for resident in (False, True):
        ga = G.GGMLGraphAllocator(device="cuda", defaultBufferSize=1 << 16)
        if resident:
            m.loadResident(ga)
        t = m.getTensor("w", ga)
        got = ga.buffers[t.bufferId][t.dataOffset:t.dataOffset + raw.size].cpu()
        assert torch.equal(got, want), resident
