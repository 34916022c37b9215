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
from collections import OrderedDict

from . import _lib
from .ops import MulMatPlan, ResidentGraph, _is_host, computeMatMul
from .tensor import GGMLCGraph, GGMLOp, GGMLTensor, GGMLType, descriptorEpoch


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


def _buffer_table(ga) -> tuple:
    """(base address, size) of every buffer of the allocator, looked up once per graphCompute."""
    return tuple((ga.dataPtr(i), ga.bufferSize(i)) if b is not None else (0, 0) for i, b in enumerate(ga.buffers))


def _graph_key(ga, nodes, extra) -> tuple:
    """Everything a plan bakes in about the nodes' tensors — type, shape, strides, offset, buffer
    (base and size, via the buffer table) — plus `extra` per node, as one flat tuple."""
    key = [_buffer_table(ga)]
    for n, e in zip(nodes, extra):
        for t in (n.src[0], n.src[1], n):
            key.append(t.type._value_)
            key.extend(t.ne)
            key.extend(t.nb)
            key.append(t.dataOffset)
            key.append(t.bufferId)
        key.append(e)
    return tuple(key)


def writeBackMask(nodes, wholeGraph: bool = False) -> list:
    """Which MUL_MAT results must reach the host ByteArrays.

    By default every one: the graph handed to graphCompute may be one split of a larger graph
    (GGMLScheduler.executeGraphSplit, core/GGMLScheduler.kt:245-258, passes split subgraphs and
    sets no output flags), so a node of a later split — a CPU op — may read any result.
    wholeGraph=True (the caller passes whole graphs): only a node flagged as a graph output
    (GGMLTensor.isOutput, core/GGMLTypes.kt:268) or one no other node of the graph consumes goes
    back; results only consumed by later offloaded nodes of the same graph stay in HBM."""
    if not wholeGraph:
        return [True] * len(nodes)
    consumed = {id(s) for n in nodes for s in n.src[:2] if s is not None}
    return [n.isOutput() or id(n) not in consumed for n in nodes]


class GGMLHipBackend:
    """core/GGMLBackend.kt:90-157 implemented on the MI355X.

    supportsOp is true exactly for the node types lk_hip computes:
    MUL_MAT with src0 in {Q4_0, Q4_1, Q8_0, Q2_K, Q4_K, Q8_K} x src1 F32 -> F32, plus the general
    F32 x F32 -> F32 and F16 x F16 -> F16 fallbacks. Everything else stays on the CPU
    backend (GGMLBackendManager's AUTO selection, core/GGMLBackendUtils.kt:152-173).

    Host (ByteArray) allocators: the weights of a graph are mirrored in HBM once per weight
    generation (include/lk_hip.h residency contract). The caller calls bumpWeightGeneration()
    whenever the allocator re-places or rewrites tensors (GGMLGraphAllocator.allocateGraph,
    core/GGMLAlloc.kt:404-480; reserve, :392, :638)."""

    GUID = "HIP-GFX950-LLAMAKOTLIN"
    MAX_CACHED_GRAPHS = 32

    def __init__(self, graphAllocator=None, device="cuda", wholeGraphs: bool = False, shardDevices=None):
        """wholeGraphs: graphCompute receives whole graphs (see writeBackMask), so results consumed
        only inside the graph need not be written back. shardDevices: HIP devices to row-shard
        every host-allocator graph over (lk_graph_create_sharded with one RCCL communicator per
        device from lk_comm_init_all; a list of one device runs the same path at world size 1)."""
        _lib.load()  # fail loudly when the HIP library is absent
        self._bufferType = GGMLHipBufferType(device)
        self.graphAllocator = graphAllocator
        self.weightGeneration = 0
        self.wholeGraphs = wholeGraphs
        self._plans: "OrderedDict[tuple, object]" = OrderedDict()
        # fast path: (graph, allocator, node identities, descriptor epoch, ...) -> full plan key
        self._fast: dict = {}
        self.comms = None
        if shardDevices:
            from .sharded import Comm
            self.comms = Comm.init_all(list(shardDevices))

    def getGuid(self) -> str:
        return self.GUID

    def getName(self) -> str:
        return "HIP"

    def free(self):
        for p in self._plans.values():
            p.close()
        self._plans.clear()
        self._fast.clear()

    def close(self):
        """free() plus the communicators (after every graph that uses them)."""
        self.free()
        for c in self.comms or []:
            c.close()
        self.comms = None

    def bumpWeightGeneration(self) -> int:
        """The host bytes of weights changed: every cached graph re-binds (or is rebuilt) against
        freshly copied mirrors. Returns the new generation."""
        self.weightGeneration += 1
        self.free()
        return self.weightGeneration

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

    def _cached(self, key, make):
        p = self._plans.get(key)
        if p is None:
            p = make()
            self._plans[key] = p
            while len(self._plans) > self.MAX_CACHED_GRAPHS:
                self._plans.popitem(last=False)[1].close()
        else:
            self._plans.move_to_end(key)
        return p

    def graphCompute(self, graph: GGMLCGraph) -> GGMLStatus:
        """Compute every MUL_MAT node of the graph (core/GGMLCpuBackend.kt:167-176 contract:
        any operator exception -> FAILED).

        Host (ByteArray) allocators: the whole node set is one ResidentGraph (lk_graph), cached
        by the full tensor descriptors and the weight generation — weights pinned, results
        written back per writeBackMask, levels of independent nodes grouped into one launch
        each, the device part replayed as a HIP graph; with shardDevices, the graph is
        row-sharded over those GPUs with an RCCL all-gather per level (lk_graph_create_sharded).
        Device allocators: mutually independent nodes run as one plan, otherwise in order."""
        ga = graph.allocator or self.graphAllocator
        try:
            nodes = [n for n in graph.nodes[: graph.nNodes] if n is not None and n.op != GGMLOp.NONE]
            # fast path: the same node objects, no descriptor changed since (tensor.descriptorEpoch),
            # the same buffers and weight generation: the cached graph's key without rebuilding it
            fast = (id(graph), id(ga), descriptorEpoch(), self.weightGeneration, _buffer_table(ga), tuple(map(id, nodes)))
            key = self._fast.get(fast)
            if key is not None and key in self._plans:
                self._plans.move_to_end(key)
                self._plans[key].compute()
                return GGMLStatus.SUCCESS
            for n in nodes:
                if not self.supportsOp(n):
                    raise _lib.NotOffloadedError(f"node {n.name!r} ({n.op}) is not supported by the HIP backend")
            if not nodes:
                return GGMLStatus.SUCCESS
            if _is_host(ga, nodes[0]):
                mask = writeBackMask(nodes, self.wholeGraphs)
                key = ("host", self.weightGeneration, id(ga), _graph_key(ga, nodes, mask))
                g = self._cached(key, lambda: ResidentGraph(ga, [(n.src[0], n.src[1], n) for n in nodes], outputs=mask,
                                                            weightGeneration=self.weightGeneration, comms=self.comms))
                if len(self._fast) > 4 * self.MAX_CACHED_GRAPHS:
                    self._fast.clear()
                self._fast[fast] = key
                g.compute()
                return GGMLStatus.SUCCESS
            ids = {id(n) for n in nodes}
            independent = all(id(s) not in ids for n in nodes for s in n.src[:2] if s is not None)
            if independent and len(nodes) > 1:
                key = ("device", id(ga), _graph_key(ga, nodes, [0] * len(nodes)))
                plan = self._cached(key, lambda: MulMatPlan(ga, [(n.src[0], n.src[1], n) for n in nodes]))
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
