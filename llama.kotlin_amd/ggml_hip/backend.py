"""GGMLHipBackend — the MI355X backend behind the reference's plugin API.

Mirrors the interfaces in core/GGMLBackend.kt (paths relative to
src/nativeMain/kotlin/ai/solace/llamakotlin/):
  GGMLBackendBufferType   :24-39    getName/allocBuffer/getAlignment/getMaxSize/isHost
  GGMLBackendBuffer       :45-75    getType/getName/getBase/getSize/free/setTensor/getTensor/copyTensor/clear
  GGMLStatus              :80-84
  GGMLBackend             :90-157   getGuid/getName/free/getDefaultBufferType/graphCompute/
                                    supportsOp/supportsBufferType/offloadOp/synchronize
  GGMLBackendRegistry     :172-251  register / find by name
The CPU backend (core/GGMLCpuBackend.kt:150-225) is what this replaces for MUL_MAT;
graphCompute catches operator exceptions and returns FAILED exactly as it does there
(:167-176).
"""
from __future__ import annotations

import enum

from . import _lib
from .ops import MulMatPlan, ResidentGraph, _is_host, computeMatMul
from .tensor import GGMLCGraph, GGMLOp, GGMLTensor, GGMLType


class GGMLStatus(enum.Enum):
    SUCCESS = 0
    FAILED = 1
    ABORTED = 2


class GGMLHipBuffer:
    """A device allocation (torch uint8 tensor on the backend's device)."""

    def __init__(self, btype: "GGMLHipBufferType", size: int):
        import torch
        self._type = btype
        self._data = torch.zeros(size, dtype=torch.uint8, device=btype.device)

    def getType(self):
        return self._type

    def getName(self) -> str:
        return "HIP"

    def getBase(self):
        return self._data

    def getSize(self) -> int:
        return int(self._data.numel())

    def free(self):
        self._data = None

    def setTensor(self, tensor: GGMLTensor, data, offset: int, size: int):
        import torch
        import numpy as np
        src = torch.from_numpy(np.frombuffer(bytes(data), np.uint8)[offset:offset + size].copy())
        start = tensor.dataOffset + offset
        self._data[start:start + size].copy_(src)

    def getTensor(self, tensor: GGMLTensor, data: bytearray, offset: int, size: int):
        start = tensor.dataOffset + offset
        data[offset:offset + size] = self._data[start:start + size].cpu().numpy().tobytes()

    def copyTensor(self, src: GGMLTensor, dst: GGMLTensor) -> bool:
        return False

    def clear(self, value: int):
        self._data.fill_(value)


class GGMLHipBufferType:
    def __init__(self, device="cuda"):
        self.device = device

    def getName(self) -> str:
        return "HIP"

    def allocBuffer(self, size: int):
        return GGMLHipBuffer(self, size)

    def getAlignment(self) -> int:
        return 256

    def getMaxSize(self) -> int:
        import torch
        return int(torch.cuda.get_device_properties(self.device).total_memory)

    def isHost(self) -> bool:
        return False


class GGMLHipBackend:
    """core/GGMLBackend.kt:90-157 implemented on the MI355X.

    supportsOp is true exactly for the node types lk_hip computes:
    MUL_MAT with src0 in {Q4_0, Q4_1, Q8_0} x src1 F32 -> F32, plus the general
    F32 x F32 -> F32 and F16 x F16 -> F16 fallbacks. Everything else stays on the CPU
    backend (GGMLBackendManager's AUTO selection, core/GGMLBackendUtils.kt:152-173).
    """

    GUID = "HIP-GFX950-LLAMAKOTLIN"

    def __init__(self, graphAllocator=None, device="cuda"):
        _lib.load()  # fail loudly when the HIP library is absent
        self._bufferType = GGMLHipBufferType(device)
        self.graphAllocator = graphAllocator
        self._plans: dict = {}

    def getGuid(self) -> str:
        return self.GUID

    def getName(self) -> str:
        return "HIP"

    def free(self):
        for p in self._plans.values():
            p.close()
        self._plans.clear()

    def getDefaultBufferType(self):
        return self._bufferType

    def allocBuffer(self, size: int):
        return self._bufferType.allocBuffer(size)

    def getAlignment(self) -> int:
        return self._bufferType.getAlignment()

    def getMaxSize(self) -> int:
        return self._bufferType.getMaxSize()

    def synchronize(self):
        import torch
        torch.cuda.synchronize()

    def supportsBufferType(self, bufferType) -> bool:
        return isinstance(bufferType, GGMLHipBufferType)

    def supportsOp(self, tensor: GGMLTensor) -> bool:
        if tensor.op != GGMLOp.MUL_MAT:
            return False
        a, b = tensor.src[0], tensor.src[1]
        if a is None or b is None:
            return False
        if a.type in (GGMLType.Q4_0, GGMLType.Q4_1, GGMLType.Q8_0, GGMLType.Q2_K, GGMLType.Q4_K, GGMLType.Q8_K):
            return b.type == GGMLType.F32 and tensor.type == GGMLType.F32
        if a.type == GGMLType.F32:
            return b.type == GGMLType.F32 and tensor.type == GGMLType.F32
        if a.type == GGMLType.F16:
            return b.type == GGMLType.F16 and tensor.type == GGMLType.F16
        return False

    def offloadOp(self, tensor: GGMLTensor) -> bool:
        return self.supportsOp(tensor)

    def graphCompute(self, graph: GGMLCGraph) -> GGMLStatus:
        """Compute every MUL_MAT node of the graph (core/GGMLCpuBackend.kt:167-176 contract:
        any operator exception -> FAILED).

        Host (ByteArray) allocators: one ResidentGraph per node set, cached — weights pinned,
        activations kept in HBM between dependent nodes, levels of independent nodes grouped.
        Device allocators: mutually independent nodes run as one plan, otherwise in order."""
        ga = graph.allocator or self.graphAllocator
        try:
            nodes = [n for n in graph.nodes[: graph.nNodes] if n is not None and n.op != GGMLOp.NONE]
            for n in nodes:
                if not self.supportsOp(n):
                    raise _lib.NotOffloadedError(f"node {n.name!r} ({n.op}) is not supported by the HIP backend")
            if nodes and _is_host(ga, nodes[0]):
                key = ("host",) + tuple((id(n), n.dataOffset, n.src[0].dataOffset, n.src[1].dataOffset,
                                         ga.dataPtr(n.bufferId), ga.dataPtr(n.src[0].bufferId),
                                         ga.dataPtr(n.src[1].bufferId)) for n in nodes)
                g = self._plans.get(key)
                if g is None:
                    g = ResidentGraph(ga, [(n.src[0], n.src[1], n) for n in nodes])
                    self._plans[key] = g
                g.compute()
                return GGMLStatus.SUCCESS
            ids = {id(n) for n in nodes}
            independent = all(id(s) not in ids for n in nodes for s in n.src[:2] if s is not None)
            if independent and len(nodes) > 1:
                key = tuple((id(n), n.dataOffset, n.src[0].dataOffset, n.src[1].dataOffset) for n in nodes)
                plan = self._plans.get(key)
                if plan is None:
                    plan = MulMatPlan(ga, [(n.src[0], n.src[1], n) for n in nodes])
                    self._plans[key] = plan
                plan.launch()
            else:
                for n in nodes:
                    computeMatMul(ga, ga.context, n.src[0], n.src[1], n)
            return GGMLStatus.SUCCESS
        except Exception as e:  # mirror of the CPU backend's catch-all
            print(f"GGMLHipBackend: Error computing graph: {e}")
            return GGMLStatus.FAILED


class GGMLBackendRegistration:
    def __init__(self, name: str, initFn, defaultBufferType=None):
        self.name = name
        self.initFn = initFn
        self.defaultBufferType = defaultBufferType


class GGMLBackendRegistry:
    """core/GGMLBackend.kt:172-251 (register the HIP backend next to CPU)."""

    _backends: list = []

    @classmethod
    def register(cls, reg: GGMLBackendRegistration):
        cls._backends = [r for r in cls._backends if r.name != reg.name] + [reg]

    @classmethod
    def findBackend(cls, name: str):
        for r in cls._backends:
            if r.name.lower() == name.lower():
                return r
        return None

    @classmethod
    def getBackendCount(cls) -> int:
        return len(cls._backends)

    @classmethod
    def initBackend(cls, name: str, *args, **kw):
        r = cls.findBackend(name)
        return r.initFn(*args, **kw) if r else None


GGMLBackendRegistry.register(GGMLBackendRegistration("HIP", GGMLHipBackend))
