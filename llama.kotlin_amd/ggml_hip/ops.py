"""The MUL_MAT operator over the HIP C-ABI, mirroring the reference's signatures.

  computeMatMul(graphAllocator, context, a, b, dst)
      core/GGMLComputeOps.kt:1435 — destination-tensor semantics: dst is pre-allocated,
      results land in graphAllocator.buffers[dst.bufferId] at dst.dataOffset, nothing is
      returned, inputs are never mutated. Exceptions as the Kotlin operator throws them
      (IllegalArgumentException / IndexOutOfBoundsException / IllegalStateException /
      NotImplementedError); see _lib.raise_for_status.
  dequantizeTensor / quantizeTensor
      core/GGMLComputeOps.kt:918 / :1040, on device (the format steps either side of the
      path).
  computeDotProductMatrix(kind, graphAllocator, a, b, K) and computeDotProduct{F32Q41, F32Q80,
      Q80Q80, Q40Q40, Q41Q41, Q80Q40}
      core/GGMLComputeOps.kt:349-629, the direct dot products (not reachable from
      computeMatMul in the reference), every (row, col) in one launch.

Device buffers go through lk_mul_mat_device on the current torch stream (asynchronous,
no host sync); host buffers through lk_mul_mat (the Kotlin ByteArray drop-in).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from .tensor import GGMLCGraph, GGMLContext, GGMLGraphAllocator, GGMLTensor, GGMLType, calculateTensorByteSize


def _is_host(ga: GGMLGraphAllocator, t: GGMLTensor) -> bool:
    if t.bufferId < 0 or t.bufferId >= len(ga.buffers):
        return ga.device == "host"
    return isinstance(ga.buffers[t.bufferId], np.ndarray)


def to_lk(ga: GGMLGraphAllocator, t: GGMLTensor) -> _lib.LkTensor:
    """GGMLTensor -> lk_tensor (buffer base, size and dataOffset; NULL for a missing buffer)."""
    lt = _lib.LkTensor()
    lt.type = int(t.type)
    for i in range(4):
        lt.ne[i] = int(t.ne[i])
        lt.nb[i] = int(t.nb[i])
    if 0 <= t.bufferId < len(ga.buffers) and ga.buffers[t.bufferId] is not None:
        lt.data = ga.dataPtr(t.bufferId)
        lt.buf_bytes = ga.bufferSize(t.bufferId)
    else:
        lt.data = None
        lt.buf_bytes = 0
    lt.data_offset = int(t.dataOffset)
    return lt


_side_streams: dict = {}


class _OnStream:
    """Pick the HIP stream a launch goes to, ordered with torch's work.

    An explicit (non-default) stream is used as is. When the caller is on torch's default
    stream (handle 0), the launch goes to a library-owned side stream fenced both ways with
    events (side waits for the caller's queue, the caller's queue waits for the launch):
    on the GPU box, launches from this library onto the null stream were observed to be
    unordered with torch's own null-stream copies (stale dst reads in round 1)."""

    def __init__(self, stream=None):
        import torch
        self.caller = stream if stream is not None else torch.cuda.current_stream()
        if int(self.caller.cuda_stream) != 0:
            self.stream, self.fence = self.caller, False
        else:
            dev = self.caller.device
            key = dev.index if dev.index is not None else torch.cuda.current_device()
            if key not in _side_streams:
                _side_streams[key] = torch.cuda.Stream(device=dev)
            self.stream, self.fence = _side_streams[key], True

    def __enter__(self):
        if self.fence:
            self.stream.wait_stream(self.caller)
        return int(self.stream.cuda_stream)

    def __exit__(self, *exc):
        if self.fence:
            self.caller.wait_stream(self.stream)
        return False


def computeMatMul(graphAllocator: GGMLGraphAllocator, context: GGMLContext | None, a: GGMLTensor, b: GGMLTensor,
                  dst: GGMLTensor, stream=None) -> None:
    """core/GGMLComputeOps.kt:1435 on the MI355X. ``context`` is unused, as in the reference."""
    L = _lib.load()
    la, lb, ld = to_lk(graphAllocator, a), to_lk(graphAllocator, b), to_lk(graphAllocator, dst)
    host = [_is_host(graphAllocator, t) for t in (a, b, dst)]
    if all(host):
        st = L.lk_mul_mat(ctypes.byref(la), ctypes.byref(lb), ctypes.byref(ld))
    elif not any(host):
        with _OnStream(stream) as sh:
            st = L.lk_mul_mat_device(ctypes.byref(la), ctypes.byref(lb), ctypes.byref(ld), sh)
    else:
        raise _lib.IllegalArgumentException("operands must all be host or all be device buffers")
    _lib.check(st)


def computeMatMulSharded(graphAllocator: GGMLGraphAllocator, context: GGMLContext | None, a: GGMLTensor,
                         b: GGMLTensor, dst: GGMLTensor, nShards: int, firstDevice: int = 0) -> None:
    """computeMatMul over host buffers with A's rows split over nShards GPUs of this process
    (lk_mul_mat_sharded_at; shard r on device (firstDevice + r) mod device count). Same results as
    computeMatMul."""
    if not all(_is_host(graphAllocator, t) for t in (a, b, dst)):
        raise _lib.IllegalArgumentException("computeMatMulSharded takes host (ByteArray) buffers")
    L = _lib.load()
    la, lb, ld = to_lk(graphAllocator, a), to_lk(graphAllocator, b), to_lk(graphAllocator, dst)
    _lib.check(L.lk_mul_mat_sharded_at(ctypes.byref(la), ctypes.byref(lb), ctypes.byref(ld), int(nShards), int(firstDevice)))


def validateMatMul(graphAllocator: GGMLGraphAllocator, a: GGMLTensor, b: GGMLTensor, dst: GGMLTensor) -> int:
    """computeMatMul's checks only; returns the lk_status code (0 = would run)."""
    L = _lib.load()
    return L.lk_mul_mat_validate(ctypes.byref(to_lk(graphAllocator, a)), ctypes.byref(to_lk(graphAllocator, b)),
                                 ctypes.byref(to_lk(graphAllocator, dst)))


class MulMatPlan:
    """Independent MUL_MAT nodes prepared once and launched together
    (GGMLBackend.graphCompute over such a graph, core/GGMLBackend.kt:146): nodes of
    one quant type share a single grouped kernel launch."""

    def __init__(self, ga: GGMLGraphAllocator, nodes, stages=None):
        """stages: None — the nodes are mutually independent (lk_plan_create); or one stage id
        per node (0, non-decreasing) — a chain of dependent stages in one persistent launch with
        a device-side grid barrier between stages (lk_plan_create_chain): stage s+1 may read
        what stage s wrote."""
        L = _lib.load()
        n = len(nodes)
        A = (_lib.LkTensor * max(n, 1))()
        B = (_lib.LkTensor * max(n, 1))()
        D = (_lib.LkTensor * max(n, 1))()
        for i, (a, b, d) in enumerate(nodes):
            A[i], B[i], D[i] = to_lk(ga, a), to_lk(ga, b), to_lk(ga, d)
        self._handle = ctypes.c_void_p()
        if stages is None:
            _lib.check(L.lk_plan_create(A, B, D, n, ctypes.byref(self._handle)))
            S = None
        else:
            if len(stages) != n:
                raise _lib.IllegalArgumentException("one stage id per node")
            S = (ctypes.c_int32 * max(n, 1))(*[int(v) for v in stages])
            _lib.check(L.lk_plan_create_chain(A, B, D, S, n, ctypes.byref(self._handle)))
        self._keep = (A, B, D, S)

    def timedOut(self) -> bool:
        """Chain plans: True if a launch gave up waiting at a barrier (grid not co-resident)."""
        st = _lib.load().lk_plan_chain_timed_out(self._handle)
        if st < 0 or st > 1:
            _lib.check(st)
        return st == 1

    @property
    def numLaunches(self) -> int:
        return _lib.load().lk_plan_num_launches(self._handle)

    def launch(self, stream=None):
        with _OnStream(stream) as sh:
            _lib.check(_lib.load().lk_plan_launch(self._handle, sh))

    def close(self):
        if self._handle:
            _lib.load().lk_plan_destroy(self._handle)
            self._handle = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class ResidentGraph:
    """GGMLComputeOps.computeGraph over MUL_MAT nodes on HOST buffers (core/GGMLComputeOps.kt:
    2515-2652) with the activations kept in HBM between nodes (lk_graph_*).

    ``nodes``: [(a, b, dst)] in graph order; a node reading bytes an earlier node writes runs
    after it. ``outputs``: per-node flags for which dst bytes are written back (None: all).
    Quantized A operands no node writes are pinned once (``weightGeneration``).

    ``comms``: row-shard the graph over RCCL communicators (lk_graph_create_sharded): a list
    holding this process's ``sharded.Comm`` (one process per GPU), or every rank's Comm of one
    ``sharded.Comm.init_all`` (one process driving several GPUs). Weight nodes then run their
    rank's rows on each device and an in-place all-gather per level completes every result."""

    def __init__(self, ga: GGMLGraphAllocator, nodes, outputs=None, weightGeneration: int = 0, comms=None):
        L = _lib.load()
        n = len(nodes)
        A = (_lib.LkTensor * max(n, 1))()
        B = (_lib.LkTensor * max(n, 1))()
        D = (_lib.LkTensor * max(n, 1))()
        for i, (a, b, d) in enumerate(nodes):
            A[i], B[i], D[i] = to_lk(ga, a), to_lk(ga, b), to_lk(ga, d)
        outs = None
        if outputs is not None:
            outs = (ctypes.c_uint8 * max(n, 1))(*[1 if o else 0 for o in outputs])
        self._handle = ctypes.c_void_p()
        if comms:
            H = (ctypes.c_void_p * len(comms))(*[c._handle for c in comms])
            _lib.check(L.lk_graph_create_sharded(H, len(comms), A, B, D, n, outs, weightGeneration, ctypes.byref(self._handle)))
        else:
            _lib.check(L.lk_graph_create(A, B, D, n, outs, weightGeneration, ctypes.byref(self._handle)))
        self._keep = (ga, A, B, D, outs, comms)

    def compute(self):
        _lib.check(_lib.load().lk_graph_compute(self._handle))

    @property
    def numLevels(self) -> int:
        return _lib.load().lk_graph_num_levels(self._handle)

    @property
    def numLaunches(self) -> int:
        return _lib.load().lk_graph_num_launches(self._handle)

    @property
    def numSharded(self) -> int:
        return _lib.load().lk_graph_num_sharded(self._handle)

    @property
    def numRebinds(self) -> int:
        return _lib.load().lk_graph_num_rebinds(self._handle)

    def transferBytes(self, toDevice: bool) -> int:
        return int(_lib.load().lk_graph_transfer_bytes(self._handle, 1 if toDevice else 0))

    def close(self):
        if self._handle:
            _lib.load().lk_graph_destroy(self._handle)
            self._handle = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def dequantizeTensor(graphAllocator: GGMLGraphAllocator, tensor: GGMLTensor, stream=None):
    """core/GGMLComputeOps.kt:918 for Q8_0/Q4_0/Q4_1 on device: returns a float32 torch tensor
    of numElements values (bit-exact with the reference)."""
    import torch
    L = _lib.load()
    n = tensor.getNumBlocks() * 32
    out = torch.empty(n, dtype=torch.float32, device=graphAllocator.buffers[tensor.bufferId].device)
    with _OnStream(stream) as sh:
        _lib.check(L.lk_dequantize_device(ctypes.byref(to_lk(graphAllocator, tensor)), ctypes.c_void_p(out.data_ptr()), sh))
    return out


def quantizeTensor(src, targetType: GGMLType, stream=None):
    """core/GGMLComputeOps.kt:1040 for a contiguous device F32 torch tensor -> uint8 block bytes
    (bit-exact: round-half-even, Kotlin floatToHalf)."""
    import torch
    L = _lib.load()
    src = src.contiguous().view(-1)
    if src.dtype != torch.float32:
        raise _lib.IllegalArgumentException(f"quantizeTensor expects F32 input, got {src.dtype}")
    n = src.numel()
    bs = GGMLType(targetType).byteSize
    out = torch.empty((n // 32) * bs if n % 32 == 0 else 0, dtype=torch.uint8, device=src.device)
    with _OnStream(stream) as sh:
        _lib.check(L.lk_quantize_device(ctypes.c_void_p(src.data_ptr()), n, int(targetType),
                                        ctypes.c_void_p(out.data_ptr() if out.numel() else 0), sh))
    return out


class DotKind:
    """lk_dot_kind (include/lk_hip.h): the direct dot products of core/GGMLComputeOps.kt:349-629."""
    F32_Q4_1 = 1   # computeDotProductF32Q41 :349
    F32_Q8_0 = 2   # computeDotProductF32Q80 :442
    Q8_0_Q8_0 = 3  # computeDotProductQ80Q80 :474
    Q4_0_Q4_0 = 4  # computeDotProductQ40Q40 :512
    Q4_1_Q4_1 = 5  # computeDotProductQ41Q41 :552
    Q8_0_Q4_0 = 6  # computeDotProductQ80Q40 :594


def computeDotProductMatrix(kind: int, graphAllocator: GGMLGraphAllocator, tensorA: GGMLTensor, tensorB: GGMLTensor,
                            commonDimK: int, stream=None):
    """Every computeDotProduct<kind>(graphAllocator, tensorA, tensorB, row, col, commonDimK) for
    row < tensorA.ne[1], col < tensorB.ne[0], as an [M, N] float32 array (numpy for host buffers,
    a torch tensor on the buffers' device otherwise). Bit-identical to the Kotlin arithmetic."""
    L = _lib.load()
    la, lb = to_lk(graphAllocator, tensorA), to_lk(graphAllocator, tensorB)
    M, N = max(int(tensorA.ne[1]), 0), max(int(tensorB.ne[0]), 0)
    host = [_is_host(graphAllocator, t) for t in (tensorA, tensorB)]
    if all(host):
        out = np.zeros((M, N), dtype=np.float32)
        _lib.check(L.lk_dot_direct(int(kind), ctypes.byref(la), ctypes.byref(lb), int(commonDimK),
                                   ctypes.c_void_p(out.ctypes.data if out.size else 0)))
        return out
    if any(host):
        raise _lib.IllegalArgumentException("operands must all be host or all be device buffers")
    import torch
    out = torch.zeros((M, N), dtype=torch.float32, device=graphAllocator.buffers[tensorA.bufferId].device)
    with _OnStream(stream) as sh:
        _lib.check(L.lk_dot_direct_device(int(kind), ctypes.byref(la), ctypes.byref(lb), int(commonDimK),
                                          ctypes.c_void_p(out.data_ptr() if out.numel() else 0), sh))
    return out


def _dot_one(kind):
    def f(graphAllocator: GGMLGraphAllocator, tensorA: GGMLTensor, tensorB: GGMLTensor, rowIndex: int, colIndex: int,
          commonDimK: int) -> float:
        return float(computeDotProductMatrix(kind, graphAllocator, tensorA, tensorB, commonDimK)[rowIndex, colIndex])
    return f


# the reference's per-(row, col) functions, by name (each evaluates the whole matrix: a test convenience)
computeDotProductF32Q41 = _dot_one(DotKind.F32_Q4_1)
computeDotProductF32Q80 = _dot_one(DotKind.F32_Q8_0)
computeDotProductQ80Q80 = _dot_one(DotKind.Q8_0_Q8_0)
computeDotProductQ40Q40 = _dot_one(DotKind.Q4_0_Q4_0)
computeDotProductQ41Q41 = _dot_one(DotKind.Q4_1_Q4_1)
computeDotProductQ80Q40 = _dot_one(DotKind.Q8_0_Q4_0)


def weightsPin(graphAllocator: GGMLGraphAllocator, a: GGMLTensor, generation: int = 0):
    """Host path: make a device mirror of a's bytes current as of ``generation``
    (GGMLBackendBuffer.setTensor residency). Pinning the same bytes with another generation
    supersedes the old mirror (the caller rewrote them); see include/lk_hip.h."""
    _lib.check(_lib.load().lk_weights_pin(ctypes.byref(to_lk(graphAllocator, a)), generation))


def weightsEvict(graphAllocator: GGMLGraphAllocator, a: GGMLTensor):
    """Drop every device mirror overlapping a's bytes."""
    _lib.check(_lib.load().lk_weights_evict(ctypes.byref(to_lk(graphAllocator, a))))


def weightsEvictBuffer(graphAllocator: GGMLGraphAllocator, bufferId: int):
    """Drop every device mirror of graphAllocator.buffers[bufferId] (the allocator replaced or
    reset it: core/GGMLAlloc.kt:392, :404-480, :638)."""
    _lib.check(_lib.load().lk_weights_evict_buffer(ctypes.c_void_p(graphAllocator.dataPtr(bufferId)),
                                                    graphAllocator.bufferSize(bufferId)))


def weightsCachedBytes() -> int:
    return int(_lib.load().lk_weights_cached_bytes())


def weightsCachedCount() -> int:
    return int(_lib.load().lk_weights_cached_count())


def weightsPinSharded(graphAllocator: GGMLGraphAllocator, a: GGMLTensor, nShards: int, generation: int = 0,
                      firstDevice: int = 0):
    """Pin each row shard of a on the device computeMatMulSharded runs it on."""
    _lib.check(_lib.load().lk_weights_pin_sharded_at(ctypes.byref(to_lk(graphAllocator, a)), generation, int(nShards),
                                                     int(firstDevice)))


def syncTimeouts() -> int:
    """In-kernel waits of the batched kernels' fused split-K reduction that gave up at their bound
    since the last call (lk_sync_timeouts; synchronizes the device, resets the count)."""
    n = ctypes.c_uint32(0)
    _lib.check(_lib.load().lk_sync_timeouts(ctypes.byref(n)))
    return int(n.value)


def setSyncWaitBound(ticks: int):
    """Bound of every device-side wait in 100 MHz ticks (lk_set_sync_wait_bound; default 20000000 =
    200 ms). Test hook of the failure path: 0 makes the batched kernels' split-K waits give up."""
    _lib.check(_lib.load().lk_set_sync_wait_bound(int(ticks)))


def syncCountersSum() -> int:
    """Sum of every split-K arrival/departure counter word on the current device (0 between launches)."""
    v = ctypes.c_uint64(0)
    _lib.check(_lib.load().lk_sync_counters_sum(ctypes.byref(v)))
    return int(v.value)


def weightsEvictAll():
    _lib.load().lk_weights_evict_all()


def debugRoute(clear: bool = True) -> str:
    """The kernels this thread's calls launched since the last clear (lk_debug_route), e.g.
    "A=mirror[0,+55296)g0 gemm_q_mfma<2>:t2s12"; '' from a library built without it."""
    L = _lib.load()
    if not hasattr(L, "lk_debug_route"):
        return ""
    r = L.lk_debug_route().decode(errors="replace")
    if clear:
        L.lk_debug_route_clear()
    return r


def debugScratchEpoch() -> int:
    """Reallocations of the current device's batched-kernel scratch so far (lk_debug_scratch_epoch)."""
    return int(_lib.load().lk_debug_scratch_epoch())


def _stream_ptr(stream=None) -> int:
    """The HIP stream handle launches requested with `stream` go to (_OnStream's choice)."""
    return int(_OnStream(stream).stream.cuda_stream)


def debugPokeGemmCounter(index: int, value: int, stream=None) -> None:
    """Store `value` into the gemm_q_* split-K tile counter `index` of the (current device, stream)
    scratch (lk_debug_poke_gemm_counter): a test of the re-arm every split-K launch does first."""
    _lib.check(_lib.load().lk_debug_poke_gemm_counter(_stream_ptr(stream), int(index), int(value)))


def scratchRelease(stream=None) -> None:
    """Free the batched kernels' scratch of (current device, stream) (lk_scratch_release); no HIP graph
    that will still be replayed may have captured a launch on that stream."""
    _lib.check(_lib.load().lk_scratch_release(_stream_ptr(stream)))


def scratchBytes() -> int:
    """Device bytes of batched-kernel scratch on the current device, all streams (lk_scratch_bytes)."""
    return int(_lib.load().lk_scratch_bytes())


__all__ = ["syncTimeouts", "setSyncWaitBound", "syncCountersSum", "debugRoute", "debugScratchEpoch",
           "debugPokeGemmCounter", "scratchRelease", "scratchBytes", "computeMatMul", "computeMatMulSharded", "ResidentGraph", "weightsPinSharded", "validateMatMul", "MulMatPlan", "dequantizeTensor", "quantizeTensor", "weightsPin",
           "weightsEvictAll", "weightsEvict", "weightsEvictBuffer", "weightsCachedBytes", "weightsCachedCount", "to_lk", "GGMLCGraph", "calculateTensorByteSize"]
