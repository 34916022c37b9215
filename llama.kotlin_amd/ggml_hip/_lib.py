"""ctypes binding of the C-ABI in include/lk_hip.h (liblk_hip.so, built in-tree).

There is no CPU fallback anywhere in this package: if the HIP library is missing
or cannot be loaded, every operator raises. torch is imported first so the
process has exactly one HIP runtime (torch's libamdhip64.so.7 satisfies the
library's NEEDED entry by SONAME) and torch streams can be handed to the C-ABI.
"""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liblk_hip.so")

# status codes (include/lk_hip.h)
LK_OK = 0
LK_ERR_INVALID_ARG = 1
LK_ERR_NOT_IMPLEMENTED = 2
LK_ERR_OUT_OF_BOUNDS = 3
LK_ERR_NO_BUFFER = 4
LK_ERR_DEVICE = 5


class LkTensor(ctypes.Structure):
    """``lk_tensor`` (include/lk_hip.h)."""

    _fields_ = [
        ("type", ctypes.c_int32),
        ("reserved", ctypes.c_int32),
        ("ne", ctypes.c_int64 * 4),
        ("nb", ctypes.c_uint64 * 4),
        ("data", ctypes.c_void_p),
        ("buf_bytes", ctypes.c_uint64),
        ("data_offset", ctypes.c_uint64),
    ]


# Exceptions mirroring what the Kotlin operator throws.
class IllegalArgumentException(ValueError):
    pass


class IndexOutOfBoundsException(IndexError):
    pass


class IllegalStateException(RuntimeError):
    pass


class HipDeviceError(RuntimeError):
    pass


class NotOffloadedError(NotImplementedError):
    """The node is not one this backend computes (GGMLHipBackend.supportsOp is false)."""


def raise_for_status(status: int, msg: str):
    if status == LK_OK:
        return
    if status == LK_ERR_INVALID_ARG:
        raise IllegalArgumentException(msg)
    if status == LK_ERR_NOT_IMPLEMENTED:
        raise NotOffloadedError(msg)
    if status == LK_ERR_OUT_OF_BOUNDS:
        raise IndexOutOfBoundsException(msg)
    if status == LK_ERR_NO_BUFFER:
        raise IllegalStateException(msg)
    raise HipDeviceError(msg)


EXPORTED_SYMBOLS = (
    "lk_init", "lk_device_count", "lk_last_error", "lk_shutdown", "lk_version",
    "lk_mul_mat_validate", "lk_mul_mat", "lk_mul_mat_device",
    "lk_plan_create", "lk_plan_launch", "lk_plan_num_launches", "lk_plan_destroy",
    "lk_weights_pin", "lk_weights_evict_all", "lk_weights_cached_bytes",
    "lk_dequantize_device", "lk_quantize_device",
)

_lib = None


def load():
    """Load liblk_hip.so (raises if it is absent: there is no fallback path)."""
    global _lib
    if _lib is not None:
        return _lib
    try:
        import torch  # noqa: F401  (one HIP runtime per process; see module docstring)
    except Exception:  # pragma: no cover - torch is part of the image
        pass
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"HIP backend library not built: {LIB_PATH} is missing "
            "(run `make -C llama.kotlin_amd` or __graft_entry__.build())")
    L = ctypes.CDLL(LIB_PATH)
    P = ctypes.POINTER(LkTensor)
    vp = ctypes.c_void_p
    L.lk_init.argtypes = [ctypes.c_int]
    L.lk_device_count.argtypes = []
    L.lk_last_error.restype = ctypes.c_char_p
    L.lk_version.restype = ctypes.c_char_p
    L.lk_shutdown.restype = None
    L.lk_mul_mat_validate.argtypes = [P, P, P]
    L.lk_mul_mat.argtypes = [P, P, P]
    L.lk_mul_mat_device.argtypes = [P, P, P, vp]
    L.lk_plan_create.argtypes = [P, P, P, ctypes.c_int, ctypes.POINTER(vp)]
    L.lk_plan_launch.argtypes = [vp, vp]
    L.lk_plan_num_launches.argtypes = [vp]
    L.lk_plan_destroy.argtypes = [vp]
    L.lk_plan_destroy.restype = None
    L.lk_weights_pin.argtypes = [P, ctypes.c_uint64]
    L.lk_weights_evict_all.restype = None
    L.lk_weights_cached_bytes.restype = ctypes.c_uint64
    L.lk_dequantize_device.argtypes = [P, vp, vp]
    L.lk_quantize_device.argtypes = [vp, ctypes.c_int64, ctypes.c_int32, vp, vp]
    _lib = L
    return L


def last_error() -> str:
    return load().lk_last_error().decode(errors="replace")


def check(status: int):
    if status != LK_OK:
        raise_for_status(status, last_error())
