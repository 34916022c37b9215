"""TEST INFRASTRUCTURE ONLY — ctypes front end of the C restatement (lk_oracle.c).

Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg may
import this module, and only as the checker. The product (llama.kotlin_amd/) never
imports it and has no CPU fallback.

The restatement follows llama.kotlin's CPU computeMatMul
(src/nativeMain/kotlin/ai/solace/llamakotlin/core/GGMLComputeOps.kt:1435-1565) and
the accessors/conversions it calls; see oracle/lk_oracle.c for file:line citations.
It is pinned by the reference's own known-answer tests (tests/test_oracle_kats.py),
because the Kotlin/Native reference cannot be built offline.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liblk_oracle.so")

# lk_type ids (include/lk_hip.h; GGMLType.fromValue, core/GGMLTypes.kt:145-168)
F32, F16, Q4_0, Q4_1, Q5_0, Q5_1, Q8_0 = 0, 1, 2, 3, 4, 5, 6
Q2_K, Q4_K, Q8_K, I8, I16, I32, I64 = 8, 10, 13, 15, 16, 17, 18
BLOCK_BYTES = {Q4_0: 18, Q4_1: 20, Q8_0: 34, Q2_K: 84, Q4_K: 144, Q8_K: 292}
QK_K = 256
TYPE_NAMES = {F32: "F32", F16: "F16", Q4_0: "Q4_0", Q4_1: "Q4_1", Q8_0: "Q8_0", Q2_K: "Q2_K", Q4_K: "Q4_K", Q8_K: "Q8_K"}


class LkTensor(ctypes.Structure):
    """Layout of ``lk_tensor`` (include/lk_hip.h)."""

    _fields_ = [
        ("type", ctypes.c_int32),
        ("reserved", ctypes.c_int32),
        ("ne", ctypes.c_int64 * 4),
        ("nb", ctypes.c_uint64 * 4),
        ("data", ctypes.c_void_p),
        ("buf_bytes", ctypes.c_uint64),
        ("data_offset", ctypes.c_uint64),
    ]


def build() -> str:
    """Compile the restatement (gcc, -ffp-contract=off) into oracle/build/."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.POINTER(LkTensor)
        L.lko_half_to_float.restype = ctypes.c_float
        L.lko_half_to_float.argtypes = [ctypes.c_uint16]
        L.lko_float_to_half.restype = ctypes.c_uint16
        L.lko_float_to_half.argtypes = [ctypes.c_float]
        L.lko_half_to_float_n.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]
        L.lko_float_to_half_n.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]
        L.lko_kotlin_round.restype = ctypes.c_float
        L.lko_kotlin_round.argtypes = [ctypes.c_float]
        L.lko_quantize.argtypes = [ctypes.c_int32, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
        L.lko_dequantize.argtypes = [ctypes.c_int32, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
        L.lko_compute_mat_mul.argtypes = [P, P, P]
        L.lko_compute_mat_mul_tight.argtypes = [P, P, P]
        L.lko_compute_mat_mul_tight_mt.argtypes = [P, P, P, ctypes.c_int]
        L.lko_dot_direct.argtypes = [ctypes.c_int32, P, P, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                     ctypes.POINTER(ctypes.c_float)]
        L.lko_dot_direct_matrix.argtypes = [ctypes.c_int32, P, P, ctypes.c_int64, ctypes.c_void_p]
        L.lko_last_error.restype = ctypes.c_char_p
        _lib = L
    return _lib


class OracleError(Exception):
    def __init__(self, status: int, msg: str):
        super().__init__(f"status {status}: {msg}")
        self.status = status


def _check(st: int):
    if st != 0:
        raise OracleError(st, lib().lko_last_error().decode())


# ---- numeric helpers --------------------------------------------------------

def half_to_float(h: np.ndarray) -> np.ndarray:
    h = np.ascontiguousarray(h, dtype=np.uint16)
    out = np.empty(h.shape, np.float32)
    lib().lko_half_to_float_n(h.ctypes.data, out.ctypes.data, h.size)
    return out


def float_to_half(f: np.ndarray) -> np.ndarray:
    f = np.ascontiguousarray(f, dtype=np.float32)
    out = np.empty(f.shape, np.uint16)
    lib().lko_float_to_half_n(f.ctypes.data, out.ctypes.data, f.size)
    return out


def quantize(qtype: int, x: np.ndarray) -> np.ndarray:
    """quantizeTensor (GGMLComputeOps.kt:1040-1204) of a flat F32 array -> block bytes."""
    x = np.ascontiguousarray(x, dtype=np.float32).reshape(-1)
    out = np.zeros(x.size // 32 * BLOCK_BYTES[qtype], np.uint8)
    _check(lib().lko_quantize(qtype, x.ctypes.data, x.size, out.ctypes.data))
    return out


def dequantize(qtype: int, blocks: np.ndarray, n: int) -> np.ndarray:
    """dequantizeTensor (GGMLComputeOps.kt:918-964) -> flat F32."""
    blocks = np.ascontiguousarray(blocks, dtype=np.uint8)
    out = np.empty(n, np.float32)
    _check(lib().lko_dequantize(qtype, blocks.ctypes.data, n, out.ctypes.data))
    return out


# ---- tensors over host buffers ---------------------------------------------

def contiguous_nb(qtype: int, ne):
    """calculateContiguousStrides (core/GGMLOps.kt:3-28) for element types."""
    es = {F32: 4, F16: 2}.get(qtype, BLOCK_BYTES.get(qtype, 0))
    nb = [es, 0, 0, 0]
    for d in range(1, 4):
        nb[d] = nb[d - 1] * (ne[d - 1] if ne[d - 1] > 0 else 1)
    return nb


def make_tensor(qtype: int, ne, buf: np.ndarray | None, data_offset: int = 0, nb=None) -> LkTensor:
    ne = list(ne) + [1] * (4 - len(ne))
    t = LkTensor()
    t.type = qtype
    for i in range(4):
        t.ne[i] = int(ne[i])
    nbv = nb if nb is not None else contiguous_nb(qtype, ne)
    nbv = list(nbv) + [0] * (4 - len(nbv))
    for i in range(4):
        t.nb[i] = int(nbv[i])
    if buf is None:
        t.data = None
        t.buf_bytes = 0
    else:
        assert buf.dtype == np.uint8 and buf.flags["C_CONTIGUOUS"]
        t.data = buf.ctypes.data
        t.buf_bytes = buf.size
    t.data_offset = int(data_offset)
    return t


def compute_mat_mul(a: LkTensor, b: LkTensor, dst: LkTensor) -> int:
    """computeMatMul restatement; returns lk_status (0 = OK). dst written in place."""
    return lib().lko_compute_mat_mul(ctypes.byref(a), ctypes.byref(b), ctypes.byref(dst))


def compute_mat_mul_tight(a: LkTensor, b: LkTensor, dst: LkTensor) -> int:
    return lib().lko_compute_mat_mul_tight(ctypes.byref(a), ctypes.byref(b), ctypes.byref(dst))


def last_error() -> str:
    return lib().lko_last_error().decode()


def mat_mul_q(qtype: int, a_blocks: np.ndarray, M: int, K: int, x: np.ndarray, tight: bool = False,
              threads: int = 1) -> np.ndarray:
    """Convenience: dst[M,N] = computeMatMul(A (qtype, ne=[K,M]), B (F32, ne=[N,K])).

    ``x`` is the B operand as a [K, N] float32 array (N fastest, as B.ne=[N,K] stores it).
    Returns dst as an [M, N] float32 array (dst.ne=[N,M]).
    """
    x = np.ascontiguousarray(x, dtype=np.float32)
    N = x.shape[1]
    abuf = np.ascontiguousarray(a_blocks, dtype=np.uint8)
    bbuf = x.view(np.uint8).reshape(-1)
    dbuf = np.zeros(M * N * 4, np.uint8)
    if qtype == F32:
        a = make_tensor(F32, [K, M], abuf)
    else:
        a = make_tensor(qtype, [K, M], abuf)
    b = make_tensor(F32, [N, K], bbuf)
    d = make_tensor(F32, [N, M], dbuf)
    if tight and threads > 1:
        st = lib().lko_compute_mat_mul_tight_mt(ctypes.byref(a), ctypes.byref(b), ctypes.byref(d), int(threads))
    else:
        st = (compute_mat_mul_tight if tight else compute_mat_mul)(a, b, d)
    _check(st)
    return dbuf.view(np.float32).reshape(M, N)


def dot_direct_matrix(kind: int, a: LkTensor, b: LkTensor, K: int) -> tuple[int, np.ndarray]:
    """lko_dot_direct_matrix: (status, [a.ne[1], b.ne[0]] float32) — the direct dot products of
    core/GGMLComputeOps.kt:349-629 for every (row, col), Kotlin arithmetic order."""
    M, N = max(int(a.ne[1]), 0), max(int(b.ne[0]), 0)
    out = np.zeros((M, N), dtype=np.float32)
    st = lib().lko_dot_direct_matrix(int(kind), ctypes.byref(a), ctypes.byref(b), int(K),
                                     out.ctypes.data if out.size else None)
    return st, out


def dot_direct(kind: int, a: LkTensor, b: LkTensor, row: int, col: int, K: int) -> tuple[int, float]:
    """lko_dot_direct: one computeDotProduct<kind>(ga, a, b, row, col, K)."""
    v = ctypes.c_float(0.0)
    st = lib().lko_dot_direct(int(kind), ctypes.byref(a), ctypes.byref(b), int(row), int(col), int(K), ctypes.byref(v))
    return st, float(v.value)
