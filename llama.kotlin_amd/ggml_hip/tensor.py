"""Host mirror of llama.kotlin's tensor model for the MUL_MAT path.

Mirrors (paths relative to src/nativeMain/kotlin/ai/solace/llamakotlin/):
  GGMLType              core/GGMLTypes.kt:99-170   (ids = GGMLType.fromValue)
  GGMLTensor            core/GGMLTypes.kt:251-357  (type, ne, nb, bufferId, dataOffset)
  GGMLGraphAllocator    core/GGMLAlloc.kt:266-640  (buffers[bufferId], allocateTensor, reserve)
  GGMLContext/GGMLCGraph core/GGMLTypes.kt:1092-1130
  calculateContiguousStrides core/GGMLOps.kt:3-28
  calculateTensorByteSize    core/GGMLTypes.kt:1136-1190

Buffers are either device allocations (torch.uint8 CUDA tensors: the MI355X-resident
case the HIP kernels read) or host numpy uint8 arrays (the Kotlin ByteArray case,
served by lk_mul_mat's host path). Operand bytes are never converted on the way in:
the kernels consume llama.kotlin's block layout as stored.
"""
from __future__ import annotations

import enum
import struct
import weakref

import numpy as np

GGML_MAX_DIMS = 4
QK4_0 = QK4_1 = QK8_0 = 32


class GGMLType(enum.IntEnum):
    """Ids follow GGMLType.fromValue (core/GGMLTypes.kt:145-168), not upstream GGUF ids."""

    F32 = 0
    F16 = 1
    Q4_0 = 2
    Q4_1 = 3
    Q5_0 = 4
    Q5_1 = 5
    Q8_0 = 6
    Q8_1 = 7
    Q2_K = 8
    Q3_K = 9
    Q4_K = 10
    Q5_K = 11
    Q6_K = 12
    Q8_K = 13
    Q1_5_K = 14
    I8 = 15
    I16 = 16
    I32 = 17
    I64 = 18
    BITNET_1_58 = 19

    @property
    def byteSize(self) -> int:
        """Bytes per element, or per 32-weight block for block types (core/GGMLTypes.kt:99-133)."""
        return _BYTE_SIZE.get(self, 0)

    @property
    def isBlockQuantized(self) -> bool:
        return self in (GGMLType.Q4_0, GGMLType.Q4_1, GGMLType.Q8_0)

    @staticmethod
    def fromValue(v: int) -> "GGMLType | None":
        try:
            t = GGMLType(v)
        except ValueError:
            return None
        return None if t == GGMLType.BITNET_1_58 else t


_BYTE_SIZE = {
    GGMLType.F32: 4, GGMLType.F16: 2, GGMLType.Q4_0: 18, GGMLType.Q4_1: 20, GGMLType.Q8_0: 34,
    GGMLType.Q2_K: 84, GGMLType.Q3_K: 110, GGMLType.Q4_K: 144, GGMLType.Q5_K: 176, GGMLType.Q6_K: 210,
    GGMLType.Q8_K: 292, GGMLType.BITNET_1_58: 10, GGMLType.I8: 1, GGMLType.I16: 2, GGMLType.I32: 4,
    GGMLType.I64: 8,
}


class GGMLOp(enum.Enum):
    NONE = 0
    MUL_MAT = 1
    ADD = 2  # present so supportsOp has something to refuse


def calculateContiguousStrides(ne, type_: GGMLType, rank: int | None = None):
    """core/GGMLOps.kt:3-28: nb[0] = byteSize, nb[d] = nb[d-1]*ne[d-1]."""
    nb = [0] * GGML_MAX_DIMS
    bs = GGMLType(type_).byteSize
    if bs == 0:
        return nb
    nb[0] = bs
    for d in range(1, GGML_MAX_DIMS):
        dim = ne[d - 1] if d - 1 < len(ne) else 1
        nb[d] = nb[d - 1] * (dim if dim > 0 else 1)
    return nb


GGML_TENSOR_FLAG_OUTPUT = 1 << 0  # core/GGMLTypes.kt:83

# Descriptor epoch: bumped whenever any GGMLTensor's type / ne / nb / bufferId / dataOffset / op /
# src / flags is assigned or mutated in place, or a tensor is created. A backend that cached work
# for a set of descriptors at epoch e knows nothing it baked in changed while the epoch is still e
# (GGMLHipBackend.graphCompute's fast path); any change sends it back to the full comparison.
_desc_epoch = [0]
_DESC_FIELDS = frozenset(("type", "ne", "nb", "bufferId", "dataOffset", "op", "src", "flags"))


def descriptorEpoch() -> int:
    return _desc_epoch[0]


class _Tracked(list):
    """A list whose in-place mutations bump the descriptor epoch (GGMLTensor.ne / nb / src)."""

    __slots__ = ()

    def _bump(self):
        _desc_epoch[0] += 1

    def __setitem__(self, i, v):
        self._bump()
        super().__setitem__(i, v)

    def __delitem__(self, i):
        self._bump()
        super().__delitem__(i)

    def __iadd__(self, other):
        self._bump()
        return super().__iadd__(other)

    def __imul__(self, n):
        self._bump()
        return super().__imul__(n)

    def append(self, v):
        self._bump()
        super().append(v)

    def extend(self, v):
        self._bump()
        super().extend(v)

    def insert(self, i, v):
        self._bump()
        super().insert(i, v)

    def pop(self, *a):
        self._bump()
        return super().pop(*a)

    def remove(self, v):
        self._bump()
        super().remove(v)

    def clear(self):
        self._bump()
        super().clear()

    def sort(self, *a, **k):
        self._bump()
        super().sort(*a, **k)

    def reverse(self):
        self._bump()
        super().reverse()


class GGMLTensor:
    """core/GGMLTypes.kt:251-270 — a descriptor; bytes live in graphAllocator.buffers[bufferId]."""

    def __setattr__(self, name, value):
        if name in _DESC_FIELDS:
            _desc_epoch[0] += 1
            if name in ("ne", "nb", "src") and value is not None and not isinstance(value, _Tracked):
                value = _Tracked(value)
        object.__setattr__(self, name, value)

    def __init__(self, type=GGMLType.F32, ne=None, nb=None, name: str = "", bufferId: int = -1,
                 dataOffset: int = 0, op: GGMLOp = GGMLOp.NONE, src=None, flags: int = 0):
        self.type = GGMLType(type)
        self.ne = list(ne) if ne is not None else [0] * GGML_MAX_DIMS
        self.ne += [1] * (GGML_MAX_DIMS - len(self.ne)) if len(self.ne) < GGML_MAX_DIMS else []
        self.nb = list(nb) if nb is not None else calculateContiguousStrides(self.ne, self.type)
        self.name = name
        self.bufferId = bufferId
        self.dataOffset = int(dataOffset)
        self.op = op
        self.src = list(src) if src is not None else [None, None]
        self.flags = int(flags)

    def isOutput(self) -> bool:
        """core/GGMLTypes.kt:268 (GGML_TENSOR_FLAG_OUTPUT = 1, :83)."""
        return (self.flags & GGML_TENSOR_FLAG_OUTPUT) != 0

    # core/GGMLTypes.kt:275-280
    def rank(self) -> int:
        if all(v <= 1 for v in self.ne):
            return 1 if any(v > 0 for v in self.ne) else 0
        return max(i for i, v in enumerate(self.ne) if v > 1) + 1

    # core/GGMLTypes.kt:286-300
    def numElements(self) -> int:
        r = self.rank()
        if r == 0 and all(v <= 1 for v in self.ne):
            return 1
        if r == 0 and any(v == 0 for v in self.ne):
            return 0
        count = 1
        for i in range(max(r, 1)):
            if self.ne[i] == 0 and r > 1:
                return 0
            if self.ne[i] > 0:
                count *= self.ne[i]
        return count

    # core/GGMLTypes.kt:507-535
    def getNumBlocks(self) -> int:
        if not self.type.isBlockQuantized:
            return 0
        return self.numElements() // 32

    def __repr__(self):
        return f"GGMLTensor({self.name!r}, {self.type.name}, ne={self.ne}, buf={self.bufferId}, off={self.dataOffset})"

    # -- element accessors (test convenience; core/GGMLTypes.kt:360-452) ------
    def _byte_offset(self, idx):
        off = 0
        for d, i in enumerate(idx):
            if i < 0 or i >= self.ne[d]:
                from ._lib import IllegalArgumentException
                raise IllegalArgumentException(f"Index {i} for dimension {d} is out of bounds")
            off += i * self.nb[d]
        return self.dataOffset + off

    def getFloat(self, ga: "GGMLGraphAllocator", *idx) -> float:
        raw = ga.readBytes(self.bufferId, self._byte_offset(idx), 4)
        return struct.unpack("<f", raw)[0]

    def setFloat(self, ga: "GGMLGraphAllocator", value: float, *idx):
        ga.writeBytes(self.bufferId, self._byte_offset(idx), struct.pack("<f", value))

    def getHalf(self, ga: "GGMLGraphAllocator", *idx) -> float:
        raw = ga.readBytes(self.bufferId, self._byte_offset(idx), 2)
        return float(np.frombuffer(raw, np.float16)[0])


def calculateTensorByteSize(t: GGMLTensor) -> int:
    """core/GGMLTypes.kt:1136-1190."""
    n = t.numElements()
    if n == 0:
        return 0
    if t.type.isBlockQuantized or t.type in (GGMLType.Q2_K, GGMLType.Q4_K, GGMLType.Q8_K):
        per = 256 if t.type in (GGMLType.Q2_K, GGMLType.Q4_K, GGMLType.Q8_K) else 32
        return (n // per) * t.type.byteSize
    return n * t.type.byteSize


class GGMLContext:
    """core/GGMLTypes.kt:1092 (unused by computeMatMul; kept for signature parity)."""

    def __init__(self, computeImmediately: bool = True):
        self.computeImmediately = computeImmediately


class GGMLCGraph:
    """core/GGMLTypes.kt:1118."""

    def __init__(self, nodes=None, allocator: "GGMLGraphAllocator | None" = None):
        self.nodes = list(nodes or [])
        self.nNodes = len(self.nodes)
        self.allocator = allocator


def _evict_host_buffer(ptr: int, size: int):
    from . import _lib
    if _lib._lib is not None:  # nothing can be pinned before the library is loaded
        _lib._lib.lk_weights_evict_buffer(ptr, size)


class GGMLGraphAllocator:
    """core/GGMLAlloc.kt:266-640 — owns the byte buffers tensors point into.

    ``device="cuda"`` buffers are device-resident (torch uint8 tensors on the current
    HIP device); ``device="host"`` buffers are numpy uint8 arrays (the ByteArray case).
    allocateTensor uses GGMLDynTensorAllocator's 16-byte alignment (core/GGMLAlloc.kt:122).
    """

    ALIGNMENT = 16

    def __init__(self, device: str = "cuda", defaultBufferSize: int = 1024 * 1024):
        self.device = device
        self.buffers: list = []
        self._tops: list[int] = []
        self.context = GGMLContext()
        self.addBuffer(defaultBufferSize)

    def _new_buffer(self, nbytes: int):
        if self.device == "host":
            buf = np.zeros(max(nbytes, 0), np.uint8)
            # The device weight mirrors are keyed by host address (include/lk_hip.h residency
            # contract): when this ByteArray goes away its address can come back with other
            # bytes, so its mirrors are evicted with it.
            if buf.size:
                weakref.finalize(buf, _evict_host_buffer, int(buf.ctypes.data), int(buf.size))
                # ... and a new ByteArray supersedes whatever mirrors still cover its address (an
                # earlier buffer's eviction can run late, e.g. when a graph object held it in a cycle)
                _evict_host_buffer(int(buf.ctypes.data), int(buf.size))
            return buf
        import torch
        return torch.zeros(max(nbytes, 0), dtype=torch.uint8, device=self.device)

    def addBuffer(self, nbytes: int) -> int:
        self.buffers.append(self._new_buffer(nbytes))
        self._tops.append(0)
        return len(self.buffers) - 1

    def bufferSize(self, bufferId: int) -> int:
        b = self.buffers[bufferId]
        return int(b.size if isinstance(b, np.ndarray) else b.numel())

    def reserve(self, nbytes: int, bufferId: int = 0):
        """core/GGMLAlloc.kt:638 — grow buffer 0 (contents preserved, unlike the reference's replace)."""
        if self.bufferSize(bufferId) >= nbytes:
            return
        old = self.buffers[bufferId]
        new = self._new_buffer(nbytes)
        new[: self.bufferSize(bufferId)] = old
        self.buffers[bufferId] = new

    def allocateTensor(self, type_: GGMLType, ne, bufferId: int = 0, name: str = "",
                       nbytes: int | None = None) -> GGMLTensor:
        """core/GGMLAlloc.kt:486-499: a leaf tensor with contiguous strides in buffer bufferId.

        ``nbytes`` overrides calculateTensorByteSize for storage it does not size (the
        K-quant and Q5/Q8_1 blocks a GGUF file can hold)."""
        ne = list(ne) + [1] * (GGML_MAX_DIMS - len(ne))
        t = GGMLTensor(type_, ne, name=name)
        size = calculateTensorByteSize(t) if nbytes is None else int(nbytes)
        off = (self._tops[bufferId] + self.ALIGNMENT - 1) // self.ALIGNMENT * self.ALIGNMENT
        if off + size > self.bufferSize(bufferId):
            self.reserve(max(off + size, 2 * self.bufferSize(bufferId)), bufferId)
        self._tops[bufferId] = off + size
        t.bufferId = bufferId
        t.dataOffset = off
        return t

    # -- byte access ------------------------------------------------------
    def readBytes(self, bufferId: int, offset: int, n: int) -> bytes:
        buf = self.buffers[bufferId]
        if buf is None:
            from ._lib import IllegalStateException
            raise IllegalStateException(f"Tensor buffer not found for bufferId {bufferId}")
        if offset + n > self.bufferSize(bufferId):
            from ._lib import IndexOutOfBoundsException
            raise IndexOutOfBoundsException(f"offset {offset}+{n} out of bounds")
        if isinstance(buf, np.ndarray):
            return buf[offset:offset + n].tobytes()
        return buf[offset:offset + n].cpu().numpy().tobytes()

    def writeBytes(self, bufferId: int, offset: int, data: bytes):
        buf = self.buffers[bufferId]
        arr = np.frombuffer(bytes(data), np.uint8)
        if isinstance(buf, np.ndarray):
            buf[offset:offset + arr.size] = arr
        else:
            import torch
            buf[offset:offset + arr.size] = torch.from_numpy(arr.copy()).to(buf.device)

    def setTensorBytes(self, t: GGMLTensor, data):
        """GGMLBackendBuffer.setTensor (core/GGMLBackend.kt:63): copy raw bytes to t's storage."""
        buf = self.buffers[t.bufferId]
        if isinstance(data, np.ndarray):
            data = np.ascontiguousarray(data).view(np.uint8).reshape(-1)
        if isinstance(buf, np.ndarray):
            buf[t.dataOffset:t.dataOffset + data.size] = data
        else:
            import torch
            src = data if isinstance(data, torch.Tensor) else torch.from_numpy(np.array(data, copy=True))
            src = src.reshape(-1).view(torch.uint8) if src.dtype != torch.uint8 else src.reshape(-1)
            buf[t.dataOffset:t.dataOffset + src.numel()].copy_(src, non_blocking=False)

    def tensorBytes(self, t: GGMLTensor, nbytes: int | None = None):
        """A view (device) or copy (host) of t's bytes."""
        n = calculateTensorByteSize(t) if nbytes is None else nbytes
        return self.buffers[t.bufferId][t.dataOffset:t.dataOffset + n]

    def dataPtr(self, bufferId: int) -> int:
        buf = self.buffers[bufferId]
        if buf is None:
            return 0
        return int(buf.ctypes.data) if isinstance(buf, np.ndarray) else int(buf.data_ptr())
