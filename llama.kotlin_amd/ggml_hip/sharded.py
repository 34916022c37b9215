"""Row-sharded MUL_MAT across the GPUs of one node (one process per GPU, RCCL over xGMI).

The reference has no multi-device code; this is the north star's design:
the dot products dst(j,i) are independent per output row i, so rank r owns rows
[r0, r1) of the weight matrix A — one contiguous byte range, because a row is
K/32 blocks — computes the matching contiguous [N x (r1-r0)] slice of dst, and one
all-gather (torch.distributed over the "nccl" backend = RCCL) reassembles the full
dst on every rank (the next layer needs every output row). B is replicated.

Shards are balanced with equal sizes (ceil(M/P) rows; the last rank may own fewer
real rows and the gather buffer is padded) so the collective is a single
all_gather_into_tensor on one contiguous buffer.
"""
from __future__ import annotations

from dataclasses import dataclass

from .tensor import GGMLGraphAllocator, GGMLTensor, GGMLType


def shard_rows(M: int, world: int, rank: int) -> tuple[int, int]:
    """Rows [r0, r1) owned by `rank` under the equal-size split (ceil(M/world) per rank)."""
    per = -(-M // world) if world > 0 else M
    r0 = min(rank * per, M)
    return r0, min(r0 + per, M)


def row_bytes(t: GGMLTensor) -> int:
    """Bytes of one row of A (ne[0] = K elements): K/32 blocks for block types."""
    K = t.ne[0]
    if t.type.isBlockQuantized:
        if K % 32:
            raise ValueError("row sharding needs K % 32 == 0 so rows are whole blocks")
        return K // 32 * t.type.byteSize
    return t.nb[1]


def row_slice(t: GGMLTensor, r0: int, r1: int, name: str = "") -> GGMLTensor:
    """A view of rows [r0, r1) of a 2-D tensor (A: ne=[K,M]; dst: ne=[N,M])."""
    s = GGMLTensor(t.type, [t.ne[0], r1 - r0, 1, 1], nb=list(t.nb), name=name or t.name,
                   bufferId=t.bufferId, dataOffset=t.dataOffset + r0 * row_bytes(t))
    return s


@dataclass
class ShardSpec:
    world: int
    rank: int
    M: int

    @property
    def rows(self) -> tuple[int, int]:
        return shard_rows(self.M, self.world, self.rank)

    @property
    def per_rank(self) -> int:
        return -(-self.M // self.world)


class RowShardedMulMat:
    """dst = A·B with A's rows sharded over the process group.

    Each rank passes its LOCAL shard a_local (ne=[K, rows owned]) and the replicated B.
    ``compute(ga, a, b, dst)`` is the local operator (default: computeMatMul on the HIP
    backend); the gather is ``torch.distributed.all_gather_into_tensor`` on ``group``.
    """

    def __init__(self, ga: GGMLGraphAllocator, M: int, N: int, world: int, rank: int, group=None, compute=None):
        import torch
        self.ga = ga
        self.spec = ShardSpec(world, rank, M)
        self.N = N
        self.group = group
        if compute is None:
            from .ops import computeMatMul
            compute = computeMatMul
        self.compute = compute
        dev = ga.buffers[0].device if hasattr(ga.buffers[0], "device") else "cpu"
        per = self.spec.per_rank
        # one contiguous gather buffer: rank r's slot holds rows [r*per, r*per+per) x N floats
        self.gathered = torch.zeros(world * per * N, dtype=torch.float32, device=dev)
        self.local = torch.zeros(per * N, dtype=torch.float32, device=dev)

    def local_rows(self) -> tuple[int, int]:
        return self.spec.rows

    def forward(self, a_local: GGMLTensor, b: GGMLTensor, local_dst: GGMLTensor):
        """Compute the local rows into local_dst (ne=[N, rows owned]) then all-gather.
        Returns the full [M, N] float32 result (a view of the gather buffer)."""
        import torch
        import torch.distributed as dist
        r0, r1 = self.spec.rows
        if r1 > r0:
            self.compute(self.ga, self.ga.context, a_local, b, local_dst)
        n_local = (r1 - r0) * self.N
        src = self.ga.buffers[local_dst.bufferId]
        if isinstance(src, torch.Tensor):
            flat = src[local_dst.dataOffset:local_dst.dataOffset + 4 * n_local].view(torch.float32)
        else:
            import numpy as np
            flat = torch.from_numpy(np.frombuffer(src[local_dst.dataOffset:local_dst.dataOffset + 4 * n_local].tobytes(),
                                                  np.float32).copy())
        self.local.zero_()
        self.local[:n_local].copy_(flat)
        if self.spec.world > 1:
            dist.all_gather_into_tensor(self.gathered, self.local, group=self.group)
        else:
            self.gathered.copy_(self.local)
        return self.gathered[: self.spec.M * self.N].view(self.spec.M, self.N)


# ---- the C-ABI path: lk_comm (RCCL held by liblk_hip.so) + lk_sharded_plan -----------------

def shard_view(t: GGMLTensor, world: int, rank: int, name: str = "") -> GGMLTensor:
    """Rows [rank·M/world, (rank+1)·M/world) of a 2-D tensor (A: ne=[K,M]; dst: ne=[N,M]) under the
    exact split lk_sharded_plan requires (M % world == 0)."""
    M = t.ne[1]
    if M % world:
        raise ValueError(f"M = {M} is not divisible by {world} ranks")
    per = M // world
    return row_slice(t, rank * per, (rank + 1) * per, name)


class Comm:
    """An RCCL communicator held by the C-ABI (lk_comm, include/lk_hip.h), on the current device."""

    def __init__(self, handle, nranks: int, rank: int):
        self._handle = handle
        self.nranks = nranks
        self.rank = rank

    @classmethod
    def from_unique_id(cls, uid: bytes, nranks: int, rank: int) -> "Comm":
        import ctypes
        from . import _lib
        L = _lib.load()
        h = ctypes.c_void_p()
        buf = ctypes.create_string_buffer(bytes(uid), 128)
        _lib.check(L.lk_comm_init_rank(buf, nranks, rank, ctypes.byref(h)))
        return cls(h, nranks, rank)

    @staticmethod
    def unique_id() -> bytes:
        import ctypes
        from . import _lib
        buf = ctypes.create_string_buffer(128)
        _lib.check(_lib.load().lk_comm_unique_id(buf))
        return buf.raw

    @classmethod
    def init_all(cls, devices) -> list:
        """One process driving several GPUs: rank r on devices[r] (lk_comm_init_all)."""
        import ctypes
        from . import _lib
        n = len(devices)
        devs = (ctypes.c_int * n)(*devices)
        hs = (ctypes.c_void_p * n)()
        _lib.check(_lib.load().lk_comm_init_all(n, devs, hs))
        return [cls(ctypes.c_void_p(hs[r]), n, r) for r in range(n)]

    @property
    def device(self) -> int:
        from . import _lib
        return _lib.load().lk_comm_device(self._handle)

    @property
    def rcclRanks(self) -> int:
        """The rank count the C-ABI communicator holds (lk_comm_nranks: what RCCL was initialised with)."""
        from . import _lib
        return int(_lib.load().lk_comm_nranks(self._handle))

    @property
    def numCollectives(self) -> int:
        """ncclAllGather calls enqueued through this communicator so far."""
        from . import _lib
        return int(_lib.load().lk_comm_num_collectives(self._handle))

    @classmethod
    def single(cls) -> "Comm":
        """A one-rank communicator (the N = 1 case of the sharded path)."""
        return cls.from_unique_id(cls.unique_id(), 1, 0)

    @classmethod
    def from_process_group(cls, group=None) -> "Comm":
        """Rank 0 makes the id, torch.distributed broadcasts its 128 bytes, every rank joins on its
        current device (one process per GPU)."""
        import torch.distributed as dist
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        box = [cls.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(box, src=0, group=group)
        return cls.from_unique_id(box[0], world, rank)

    def close(self):
        if self._handle:
            from . import _lib
            _lib.load().lk_comm_destroy(self._handle)
            self._handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class ShardedMulMatPlan:
    """lk_sharded_plan: independent MUL_MAT nodes row-sharded over `comm`. ``nodes`` =
    [(a_shard, b, dst_full)]: this rank's rows of A (shard_view), the full activations and the
    FULL destination. One launch computes the local rows in place inside dst_full, then one RCCL
    group of in-place all-gathers completes every dst_full on every rank."""

    def __init__(self, comm: Comm, ga: GGMLGraphAllocator, nodes):
        import ctypes
        from . import _lib
        from .ops import to_lk
        L = _lib.load()
        n = len(nodes)
        A = (_lib.LkTensor * max(n, 1))()
        B = (_lib.LkTensor * max(n, 1))()
        D = (_lib.LkTensor * max(n, 1))()
        for i, (a, b, d) in enumerate(nodes):
            A[i], B[i], D[i] = to_lk(ga, a), to_lk(ga, b), to_lk(ga, d)
        self._handle = ctypes.c_void_p()
        _lib.check(L.lk_sharded_plan_create(comm._handle, A, B, D, n, ctypes.byref(self._handle)))
        self.comm = comm

    @property
    def numGathers(self) -> int:
        from . import _lib
        return _lib.load().lk_sharded_plan_num_gathers(self._handle)

    def launch(self, stream=None):
        from . import _lib
        from .ops import _OnStream
        with _OnStream(stream) as sh:
            _lib.check(_lib.load().lk_sharded_plan_launch(self._handle, sh))

    def launchSplit(self, compute, gather):
        """Throughput form (lk_sharded_plan_launch_split): the local rows on torch stream `compute`,
        the all-gathers on `gather` behind them, so the next plan's rows overlap this exchange. The
        caller joins `gather` back (compute.wait_stream(gather)) before it reads the outputs."""
        from . import _lib
        _lib.check(_lib.load().lk_sharded_plan_launch_split(self._handle, int(compute.cuda_stream), int(gather.cuda_stream)))

    def close(self):
        if self._handle:
            from . import _lib
            _lib.load().lk_sharded_plan_destroy(self._handle)
            self._handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class P2PGroup:
    """lk_p2p_group (include/lk_hip.h): ranks 0..P-1 on ``devices`` driven by this process, peer
    access enabled between distinct devices. Devices may repeat (several ranks on one GPU)."""

    def __init__(self, devices):
        import ctypes
        from . import _lib
        n = len(devices)
        devs = (ctypes.c_int * n)(*devices)
        self._handle = ctypes.c_void_p()
        _lib.check(_lib.load().lk_p2p_group_create(n, devs, ctypes.byref(self._handle)))
        self.devices = list(devices)
        self.nranks = n

    def close(self):
        if self._handle:
            from . import _lib
            _lib.load().lk_p2p_group_destroy(self._handle)
            self._handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class P2PMulMatPlan:
    """lk_p2p_plan: the one-shot peer-write alternative to ShardedMulMatPlan. ``ranks[r]`` =
    [(a_shard, b, dst_full)] for rank r (on rank r's device; ``ga`` one allocator or one per rank).
    A launch computes every rank's rows in place, pushes them into every peer's dst and signals;
    the next plan launched in the group waits (hipStreamWaitValue64) until they all arrived.
    Eager only (HipDeviceError/NotImplemented while capturing)."""

    def __init__(self, group: P2PGroup, ga, ranks):
        import ctypes
        from . import _lib
        from .ops import to_lk
        P = group.nranks
        if len(ranks) != P or len({len(nodes) for nodes in ranks}) != 1:
            raise ValueError("one node list of equal length per rank")
        gas = ga if isinstance(ga, (list, tuple)) else [ga] * P
        n = len(ranks[0])
        A = (_lib.LkTensor * max(P * n, 1))()
        B = (_lib.LkTensor * max(P * n, 1))()
        D = (_lib.LkTensor * max(P * n, 1))()
        for r, nodes in enumerate(ranks):
            for i, (a, b, d) in enumerate(nodes):
                A[r * n + i], B[r * n + i], D[r * n + i] = to_lk(gas[r], a), to_lk(gas[r], b), to_lk(gas[r], d)
        self._handle = ctypes.c_void_p()
        _lib.check(_lib.load().lk_p2p_plan_create(group._handle, A, B, D, n, ctypes.byref(self._handle)))
        self.group = group

    def launch(self, streams):
        """``streams``: one torch stream per rank, or one stream for all (ranks on one device)."""
        import ctypes
        from . import _lib
        P = self.group.nranks
        if not isinstance(streams, (list, tuple)):
            streams = [streams] * P
        hs = (ctypes.c_void_p * P)(*[int(s.cuda_stream) for s in streams])
        _lib.check(_lib.load().lk_p2p_plan_launch(self._handle, hs))

    @property
    def numLaunches(self) -> int:
        from . import _lib
        return int(_lib.load().lk_p2p_plan_num_launches(self._handle))

    def signal(self, rank: int) -> int:
        """Rank's arrival signal after synchronizing its device (launches · P when all arrived)."""
        import ctypes
        from . import _lib
        v = ctypes.c_uint64()
        _lib.check(_lib.load().lk_p2p_plan_signal(self._handle, rank, ctypes.byref(v)))
        return int(v.value)

    def close(self):
        if self._handle:
            from . import _lib
            _lib.load().lk_p2p_plan_destroy(self._handle)
            self._handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class P2PChain:
    """lk_p2p_chain: dependent stages of N = 1 MUL_MAT nodes (a model's layers) as ONE persistent
    launch per rank. ``ranks[r]`` = [(a_shard, b, dst_full)] for rank r — its row shard of each node's
    weights, its copy of the activations (for a later stage: its copy of an earlier node's dst), its
    full dst; every rank's dst tensors laid out alike. ``stages``: one stage id per node (0, then
    non-decreasing by at most 1). A launch streams every rank's rows, stores each into every rank's
    dst and waits, between stages, for every rank (no collective, no host gate)."""

    def __init__(self, group: P2PGroup, ga, ranks, stages):
        import ctypes
        from . import _lib
        from .ops import to_lk
        P = group.nranks
        if len(ranks) != P or len({len(nodes) for nodes in ranks}) != 1:
            raise ValueError("one node list of equal length per rank")
        gas = ga if isinstance(ga, (list, tuple)) else [ga] * P
        n = len(ranks[0])
        if len(stages) != n:
            raise _lib.IllegalArgumentException("one stage id per node")
        A = (_lib.LkTensor * max(P * n, 1))()
        B = (_lib.LkTensor * max(P * n, 1))()
        D = (_lib.LkTensor * max(P * n, 1))()
        for r, nodes in enumerate(ranks):
            for i, (a, b, d) in enumerate(nodes):
                A[r * n + i], B[r * n + i], D[r * n + i] = to_lk(gas[r], a), to_lk(gas[r], b), to_lk(gas[r], d)
        S = (ctypes.c_int32 * max(n, 1))(*[int(v) for v in stages])
        self._handle = ctypes.c_void_p()
        _lib.check(_lib.load().lk_p2p_chain_create(group._handle, A, B, D, S, n, ctypes.byref(self._handle)))
        self.group = group
        self._keep = (A, B, D, S)

    def launch(self, streams=None):
        """``streams``: one torch stream per rank (ranks on one device: distinct streams that can run
        at once), or None: the group's own per-rank streams (CU-partitioned where ranks share a GPU)."""
        import ctypes
        from . import _lib
        if streams is None:
            _lib.check(_lib.load().lk_p2p_chain_launch(self._handle, None))
            return
        P = self.group.nranks
        hs = (ctypes.c_void_p * P)(*[int(s.cuda_stream) for s in streams])
        _lib.check(_lib.load().lk_p2p_chain_launch(self._handle, hs))

    def rankStream(self, r: int):
        """The group's own stream of rank r (what launch() uses) as a torch ExternalStream."""
        import torch
        from . import _lib
        h = _lib.load().lk_p2p_chain_rank_stream(self._handle, int(r))
        if not h:
            _lib.check(_lib.LK_ERR_DEVICE)
        return torch.cuda.ExternalStream(h, device=torch.device("cuda", self.group.devices[r]))

    def timedOut(self) -> bool:
        """True if any rank's barrier gave up waiting (synchronizes the ranks' devices; re-arms)."""
        from . import _lib
        st = _lib.load().lk_p2p_chain_timed_out(self._handle)
        if st < 0 or st > 1:
            _lib.check(st)
        return st == 1

    @property
    def numLaunches(self) -> int:
        from . import _lib
        return int(_lib.load().lk_p2p_chain_num_launches(self._handle))

    def close(self):
        if self._handle:
            from . import _lib
            _lib.load().lk_p2p_chain_destroy(self._handle)
            self._handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
