"""The C-ABI library (no GPU needed): it loads, exports every symbol include/lk_hip.h
declares, and its validation path (no device work) raises what the Kotlin operator
raises, agreeing with the oracle's statuses for the offloaded node types."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from _util import pattern_f32, pattern_src

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = [os.path.join(ROOT, "include", h) for h in ("lk_hip.h", "lk_gguf.h")]


def header_functions():
    names = set()
    for h in HEADERS:
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        names |= set(re.findall(r"\b(lk_[a-z0-9_]+)\s*\(", src))
    return sorted(names)


@pytest.fixture(scope="module")
def lib():
    import ggml_hip._lib as L
    if not os.path.exists(L.LIB_PATH):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "llama.kotlin_amd")], check=True)
    return L.load()


def test_exports_every_declared_symbol(lib):
    names = header_functions()
    assert len(names) >= 15
    for n in names:
        assert hasattr(lib, n), f"{n} declared in include/ but not exported"
    import ggml_hip._lib as L
    assert set(L.EXPORTED_SYMBOLS) == set(names)


def test_is_gfx950_code_object(lib):
    import ggml_hip._lib as L
    blob = open(L.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob  # the embedded offload bundle's target id


# Every kernel family the library carries, each reachable by the default dispatch for some shape
# (DESIGN.md §3); lab variants are built from patched copies of csrc/, never into this library.
PRODUCT_KERNELS = {
    "gemv_stream_kernel", "gemv_q_n1_kernel", "gemm_skinny_kernel", "gemm_skinny_pair_kernel",
    "gemm_sk_kernel", "gemm_kpart_kernel", "xsplit_kernel", "gemm_wide_kernel", "splitk_reduce_kernel", "f32_mfma_kernel", "f32_lds_kernel",
    "gemm_q_lds_kernel", "gemm_q_mfma_kernel", "kquant_n1_kernel", "kquant_nc_kernel",
    "kquant_gemv_kernel", "kquant_mul_mat_kernel", "mul_mat_generic_kernel", "dequantize_coop_kernel",
    "quantize_coop_kernel", "dequantize_kernel", "quantize_kernel", "dot_direct_kernel",
    "repack_q4_kernel", "gemv_stream_peer_kernel", "gemm_w32_kernel", "xsplit32_kernel",
    "gemm_skinny_pair_group_kernel", "splitk_reduce_group_kernel",
}


def test_kernel_list_is_the_product(lib):
    """The device code object holds only the product's kernel families: kernel
    descriptors are the `<mangled name>.kd` symbols of namespace lk."""
    import ggml_hip._lib as L
    blob = open(L.LIB_PATH, "rb").read()
    names = re.findall(rb"_ZN2lk\d+([A-Za-z_0-9]+?_kernel)", blob)  # device symbols and host stubs
    found = {m.decode().removeprefix("__device_stub__") for m in names}
    assert found, "no lk:: kernels found in the library"
    assert found <= PRODUCT_KERNELS, f"kernels outside the product set: {sorted(found - PRODUCT_KERNELS)}"
    for k in ("gemv_stream_kernel", "gemm_skinny_pair_kernel", "gemm_wide_kernel", "xsplit_kernel"):
        assert k in found


def test_version_and_no_device(lib):
    assert b"gfx950" in lib.lk_version()
    import torch
    if not torch.cuda.is_available():
        assert lib.lk_device_count() == 0


def test_struct_layout_matches_header():
    import ggml_hip._lib as L
    import oracle as O
    assert ctypes.sizeof(L.LkTensor) == 4 + 4 + 32 + 32 + 8 + 8 + 8
    assert ctypes.sizeof(L.LkTensor) == ctypes.sizeof(O.LkTensor)
    for (n1, _), (n2, _) in zip(L.LkTensor._fields_, O.LkTensor._fields_):
        assert n1 == n2


def _lk(t):
    import ggml_hip._lib as L
    lt = L.LkTensor()
    ctypes.memmove(ctypes.byref(lt), ctypes.byref(t), ctypes.sizeof(lt))
    return lt


def test_validation_statuses_match_oracle(lib, oracle):
    """lk_mul_mat_validate vs the oracle's computeMatMul status on the same descriptors."""
    O = oracle
    cases = []
    M, K, N = 3, 64, 2
    for qt in (O.Q4_0, O.Q4_1, O.Q8_0):
        qa = O.quantize(qt, pattern_src(qt, M * K, 42))
        xb = pattern_f32(K * N, 84).view(np.uint8).copy()
        d = np.zeros(M * N * 4, np.uint8)
        cases += [
            (O.make_tensor(qt, [K, M], qa), O.make_tensor(O.F32, [N, K], xb), O.make_tensor(O.F32, [N, M], d), 0),
            (O.make_tensor(qt, [K, M], qa), O.make_tensor(O.F32, [N, K + 32], xb), O.make_tensor(O.F32, [N, M], d), 1),
            (O.make_tensor(qt, [K, M], qa), O.make_tensor(O.F32, [N, K], xb), O.make_tensor(O.F32, [N, M + 1], d), 1),
            (O.make_tensor(qt, [K, M], qa), O.make_tensor(O.F32, [N, K], xb), O.make_tensor(O.F16, [N, M], d), 1),
            (O.make_tensor(qt, [K, M], qa[:10].copy()), O.make_tensor(O.F32, [N, K], xb), O.make_tensor(O.F32, [N, M], d), 3),
            (O.make_tensor(qt, [K, M], qa), O.make_tensor(O.F32, [N, K], xb[:8].copy()), O.make_tensor(O.F32, [N, M], d), 3),
            (O.make_tensor(qt, [K, M], None), O.make_tensor(O.F32, [N, K], xb), O.make_tensor(O.F32, [N, M], d), 4),
            (O.make_tensor(qt, [K, M], qa), O.make_tensor(O.F32, [N, K], xb), O.make_tensor(O.F32, [N, M], None), 4),
            # K % 32 != 0 and M*K % 32 != 0: the last block index exceeds getNumBlocks -> IAE
            (O.make_tensor(qt, [33, 1], qa), O.make_tensor(O.F32, [1, 33], xb), O.make_tensor(O.F32, [1, 1], d), 1),
        ]
    fa = pattern_f32(M * K, 1).view(np.uint8).copy()
    fb = pattern_f32(K * N, 2).view(np.uint8).copy()
    d = np.zeros(M * N * 4, np.uint8)
    cases += [
        (O.make_tensor(O.F32, [K, M], fa), O.make_tensor(O.F32, [N, K], fb), O.make_tensor(O.F32, [N, M], d), 0),
        (O.make_tensor(O.F32, [K, M], fa), O.make_tensor(O.F32, [N, K], fb), O.make_tensor(O.F16, [N, M], d), 1),
        (O.make_tensor(O.I32, [K, M], fa), O.make_tensor(O.I32, [N, K], fb), O.make_tensor(O.I32, [N, M], d), 2),
        # empty output: nothing is read, nothing fails
        (O.make_tensor(O.Q4_0, [K, 0], None), O.make_tensor(O.F32, [N, K], None), O.make_tensor(O.F32, [N, 0], None), 0),
    ]
    for a, b, dd, want in cases:
        got = lib.lk_mul_mat_validate(ctypes.byref(_lk(a)), ctypes.byref(_lk(b)), ctypes.byref(_lk(dd)))
        ref = O.compute_mat_mul(a, b, dd)
        assert got == want, (got, want)
        assert ref == want, (ref, want, O.last_error())
