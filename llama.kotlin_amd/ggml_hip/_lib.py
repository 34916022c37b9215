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
LIB_PATH = os.environ.get("LK_HIP_LIB") or os.path.join(HERE, "liblk_hip.so")  # env: lab A/B builds only

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
    "lk_mul_mat_validate", "lk_mul_mat", "lk_mul_mat_device", "lk_mul_mat_sharded", "lk_weights_pin_sharded",
    "lk_mul_mat_sharded_at", "lk_weights_pin_sharded_at",
    "lk_plan_create", "lk_plan_launch", "lk_plan_num_launches", "lk_plan_destroy", "lk_plan_create_chain",
    "lk_plan_chain_timed_out", "lk_sync_timeouts", "lk_set_sync_wait_bound", "lk_sync_counters_sum",
    "lk_debug_route", "lk_debug_route_clear", "lk_debug_scratch_epoch", "lk_debug_poke_gemm_counter",
    "lk_scratch_release", "lk_scratch_bytes",
    "lk_graph_create", "lk_graph_create_sharded", "lk_graph_num_sharded", "lk_graph_compute",
    "lk_graph_num_levels", "lk_graph_num_launches",
    "lk_graph_transfer_bytes", "lk_graph_destroy", "lk_graph_num_rebinds",
    "lk_weights_pin", "lk_weights_evict", "lk_weights_evict_buffer", "lk_weights_evict_all",
    "lk_weights_cached_bytes", "lk_weights_cached_count",
    "lk_comm_unique_id", "lk_comm_init_rank", "lk_comm_init_all", "lk_comm_nranks", "lk_comm_rank",
    "lk_comm_device", "lk_comm_num_collectives",
    "lk_comm_destroy", "lk_comm_abort", "lk_comm_group_start", "lk_comm_group_end",
    "lk_sharded_plan_create", "lk_sharded_plan_launch", "lk_sharded_plan_launch_split", "lk_sharded_plan_num_gathers", "lk_sharded_plan_destroy",
    "lk_p2p_group_create", "lk_p2p_group_nranks", "lk_p2p_group_destroy", "lk_p2p_plan_create", "lk_p2p_plan_launch",
    "lk_p2p_plan_num_launches", "lk_p2p_plan_signal", "lk_p2p_plan_destroy",
    "lk_p2p_chain_create", "lk_p2p_chain_launch", "lk_p2p_chain_timed_out", "lk_p2p_chain_num_launches",
    "lk_p2p_chain_destroy", "lk_p2p_chain_rank_stream",
    "lk_dequantize_device", "lk_quantize_device", "lk_dot_direct", "lk_dot_direct_device",
    # include/lk_gguf.h
    "lk_gguf_open_memory", "lk_gguf_open_file", "lk_gguf_close", "lk_gguf_version", "lk_gguf_alignment",
    "lk_gguf_data_offset", "lk_gguf_data_bytes", "lk_gguf_kv_count", "lk_gguf_find_key", "lk_gguf_kv_key",
    "lk_gguf_kv_type", "lk_gguf_kv_array_info", "lk_gguf_kv_get", "lk_gguf_kv_array_data",
    "lk_gguf_kv_get_string", "lk_gguf_tensor_count", "lk_gguf_find_tensor", "lk_gguf_get_tensor_info",
    "lk_gguf_tensor_data", "lk_gguf_load_tensor", "lk_gguf_load_all_device", "lk_repack_q4_device",
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
    L.lk_mul_mat_sharded.argtypes = [P, P, P, ctypes.c_int]
    L.lk_weights_pin_sharded.argtypes = [P, ctypes.c_uint64, ctypes.c_int]
    if hasattr(L, "lk_mul_mat_sharded_at"):  # (absent from round-4 lab builds loaded for A/B)
        L.lk_mul_mat_sharded_at.argtypes = [P, P, P, ctypes.c_int, ctypes.c_int]
        L.lk_weights_pin_sharded_at.argtypes = [P, ctypes.c_uint64, ctypes.c_int, ctypes.c_int]
    L.lk_plan_create.argtypes = [P, P, P, ctypes.c_int, ctypes.POINTER(vp)]
    L.lk_plan_launch.argtypes = [vp, vp]
    L.lk_plan_create_chain.argtypes = [P, P, P, ctypes.POINTER(ctypes.c_int32), ctypes.c_int, ctypes.POINTER(vp)]
    L.lk_plan_chain_timed_out.argtypes = [vp]
    L.lk_sync_timeouts.argtypes = [ctypes.POINTER(ctypes.c_uint32)]
    L.lk_set_sync_wait_bound.argtypes = [ctypes.c_uint64]
    L.lk_sync_counters_sum.argtypes = [ctypes.POINTER(ctypes.c_uint64)]
    if hasattr(L, "lk_debug_route"):  # (absent from round-4 lab builds loaded for A/B)
        L.lk_debug_route.restype = ctypes.c_char_p
        L.lk_debug_route_clear.restype = None
        L.lk_debug_scratch_epoch.restype = ctypes.c_uint64
    if hasattr(L, "lk_scratch_release"):  # (absent from round-5 lab builds loaded for A/B)
        L.lk_debug_poke_gemm_counter.argtypes = [vp, ctypes.c_int64, ctypes.c_int32]
        L.lk_scratch_release.argtypes = [vp]
        L.lk_scratch_bytes.restype = ctypes.c_uint64
    L.lk_plan_num_launches.argtypes = [vp]
    L.lk_plan_destroy.argtypes = [vp]
    L.lk_plan_destroy.restype = None
    L.lk_graph_create.argtypes = [P, P, P, ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(vp)]
    L.lk_graph_create_sharded.argtypes = [ctypes.POINTER(vp), ctypes.c_int, P, P, P, ctypes.c_int, ctypes.c_void_p,
                                          ctypes.c_uint64, ctypes.POINTER(vp)]
    L.lk_graph_num_sharded.argtypes = [vp]
    L.lk_graph_compute.argtypes = [vp]
    L.lk_graph_num_levels.argtypes = [vp]
    L.lk_graph_num_launches.argtypes = [vp]
    L.lk_graph_transfer_bytes.argtypes = [vp, ctypes.c_int]
    L.lk_graph_transfer_bytes.restype = ctypes.c_uint64
    L.lk_graph_destroy.argtypes = [vp]
    L.lk_graph_destroy.restype = None
    L.lk_weights_pin.argtypes = [P, ctypes.c_uint64]
    L.lk_weights_evict.argtypes = [P]
    L.lk_weights_evict_buffer.argtypes = [vp, ctypes.c_uint64]
    L.lk_weights_evict_all.restype = None
    L.lk_weights_cached_bytes.restype = ctypes.c_uint64
    L.lk_weights_cached_count.restype = ctypes.c_uint64
    L.lk_graph_num_rebinds.argtypes = [vp]
    L.lk_comm_unique_id.argtypes = [vp]
    L.lk_comm_init_rank.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.POINTER(vp)]
    L.lk_comm_init_all.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(vp)]
    L.lk_comm_nranks.argtypes = [vp]
    L.lk_comm_rank.argtypes = [vp]
    L.lk_comm_device.argtypes = [vp]
    L.lk_comm_num_collectives.argtypes = [vp]
    L.lk_comm_num_collectives.restype = ctypes.c_uint64
    L.lk_comm_destroy.argtypes = [vp]
    L.lk_comm_destroy.restype = None
    if hasattr(L, "lk_comm_abort"):  # (absent from round-3 lab builds loaded for A/B)
        L.lk_comm_abort.argtypes = [vp]
    L.lk_sharded_plan_create.argtypes = [vp, P, P, P, ctypes.c_int, ctypes.POINTER(vp)]
    L.lk_sharded_plan_launch.argtypes = [vp, vp]
    if hasattr(L, "lk_sharded_plan_launch_split"):  # (absent from round-5 lab builds loaded for A/B)
        L.lk_sharded_plan_launch_split.argtypes = [vp, vp, vp]
    L.lk_sharded_plan_num_gathers.argtypes = [vp]
    L.lk_sharded_plan_destroy.argtypes = [vp]
    L.lk_sharded_plan_destroy.restype = None
    if hasattr(L, "lk_p2p_plan_create"):  # (absent from round-3 lab builds loaded for A/B)
        L.lk_p2p_group_create.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(vp)]
        L.lk_p2p_group_nranks.argtypes = [vp]
        L.lk_p2p_group_destroy.argtypes = [vp]
        L.lk_p2p_group_destroy.restype = None
        L.lk_p2p_plan_create.argtypes = [vp, P, P, P, ctypes.c_int, ctypes.POINTER(vp)]
        L.lk_p2p_plan_launch.argtypes = [vp, ctypes.POINTER(vp)]
        L.lk_p2p_plan_num_launches.argtypes = [vp]
        L.lk_p2p_plan_num_launches.restype = ctypes.c_uint64
        L.lk_p2p_plan_signal.argtypes = [vp, ctypes.c_int, ctypes.POINTER(ctypes.c_uint64)]
        L.lk_p2p_plan_destroy.argtypes = [vp]
        L.lk_p2p_plan_destroy.restype = None
    if hasattr(L, "lk_p2p_chain_create"):  # (absent from round-4 lab builds loaded for A/B)
        L.lk_p2p_chain_create.argtypes = [vp, P, P, P, ctypes.POINTER(ctypes.c_int32), ctypes.c_int, ctypes.POINTER(vp)]
        L.lk_p2p_chain_launch.argtypes = [vp, ctypes.c_void_p]
        L.lk_p2p_chain_timed_out.argtypes = [vp]
        L.lk_p2p_chain_num_launches.argtypes = [vp]
        L.lk_p2p_chain_num_launches.restype = ctypes.c_uint64
        L.lk_p2p_chain_destroy.argtypes = [vp]
        if hasattr(L, "lk_p2p_chain_rank_stream"):
            L.lk_p2p_chain_rank_stream.argtypes = [vp, ctypes.c_int]
            L.lk_p2p_chain_rank_stream.restype = vp
        L.lk_p2p_chain_destroy.restype = None
    L.lk_dequantize_device.argtypes = [P, vp, vp]
    L.lk_quantize_device.argtypes = [vp, ctypes.c_int64, ctypes.c_int32, vp, vp]
    L.lk_dot_direct.argtypes = [ctypes.c_int32, P, P, ctypes.c_int64, vp]
    L.lk_dot_direct_device.argtypes = [ctypes.c_int32, P, P, ctypes.c_int64, vp, vp]
    # GGUF (include/lk_gguf.h); handles are opaque void*
    u64, i64, i32, pvp, pu64 = ctypes.c_uint64, ctypes.c_int64, ctypes.c_int32, ctypes.POINTER(vp), ctypes.POINTER(ctypes.c_uint64)
    L.lk_gguf_open_memory.argtypes = [vp, u64, i32, pvp]
    L.lk_gguf_open_file.argtypes = [ctypes.c_char_p, i32, pvp]
    L.lk_gguf_close.argtypes = [vp]
    L.lk_gguf_close.restype = None
    L.lk_gguf_version.argtypes = [vp]
    L.lk_gguf_version.restype = ctypes.c_uint32
    for f in (L.lk_gguf_alignment, L.lk_gguf_data_offset, L.lk_gguf_data_bytes):
        f.argtypes = [vp]
        f.restype = u64
    for f in (L.lk_gguf_kv_count, L.lk_gguf_tensor_count):
        f.argtypes = [vp]
        f.restype = i64
    for f in (L.lk_gguf_find_key, L.lk_gguf_find_tensor):
        f.argtypes = [vp, ctypes.c_char_p]
        f.restype = i64
    L.lk_gguf_kv_key.argtypes = [vp, i64]
    L.lk_gguf_kv_key.restype = ctypes.c_char_p
    L.lk_gguf_kv_type.argtypes = [vp, i64]
    L.lk_gguf_kv_type.restype = i32
    L.lk_gguf_kv_array_info.argtypes = [vp, i64, ctypes.POINTER(i32), pu64]
    L.lk_gguf_kv_get.argtypes = [vp, i64, i64, vp, u64]
    L.lk_gguf_kv_array_data.argtypes = [vp, i64, pvp, pu64]
    L.lk_gguf_kv_get_string.argtypes = [vp, i64, i64, pvp, pu64]
    L.lk_gguf_get_tensor_info.argtypes = [vp, i64, vp]
    L.lk_gguf_tensor_data.argtypes = [vp, i64, pvp, pu64]
    L.lk_gguf_load_tensor.argtypes = [vp, i64, vp, u64, i32, vp]
    L.lk_gguf_load_all_device.argtypes = [vp, vp, u64, vp]
    L.lk_repack_q4_device.argtypes = [vp, i64, i32, i32, vp]
    _lib = L
    return L


def last_error() -> str:
    return load().lk_last_error().decode(errors="replace")


def check(status: int):
    if status != LK_OK:
        raise_for_status(status, last_error())
