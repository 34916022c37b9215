"""Row-sharded MUL_MAT over a world_size-2 process group on the CPU (gloo).

The N>1 path of RowShardedMulMat (llama.kotlin_amd/ggml_hip/sharded.py): every rank owns a
contiguous row range of A, computes its rows, and one all_gather_into_tensor reassembles
dst. On the GPU box the local operator is computeMatMul (HIP) and the collective runs on
RCCL; here the local operator is the oracle (test-only) and the collective runs on gloo,
so the sharding, padding and gather logic is checked without a GPU.
"""
import ctypes
import os
import socket

import numpy as np
import pytest

from _util import random_acts, random_weights


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _oracle_compute(ga, ctx, a, b, d):
    import oracle as O
    from ggml_hip.ops import to_lk

    def conv(t):
        lt = O.LkTensor()
        src = to_lk(ga, t)
        ctypes.memmove(ctypes.byref(lt), ctypes.byref(src), ctypes.sizeof(lt))
        return lt

    la, lb, ld = conv(a), conv(b), conv(d)
    st = O.compute_mat_mul(la, lb, ld)
    assert st == 0, O.last_error()


def _worker(rank, world, port, qt, M, K, N, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    import oracle as O
    import ggml_hip as G
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q = O.quantize(qt, random_weights(M * K, 0x5EED + 7))
        x = random_acts(K * N, 0x5EED + 8).reshape(K, N)
        ga = G.GGMLGraphAllocator(device="host", defaultBufferSize=1 << 20)
        sh = G.RowShardedMulMat(ga, M, N, world, rank, compute=_oracle_compute)
        r0, r1 = sh.local_rows()
        bs = G.GGMLType(qt).byteSize
        rb = K // 32 * bs
        a_local = ga.allocateTensor(G.GGMLType(qt), [K, max(r1 - r0, 0)])
        if r1 > r0:
            ga.setTensorBytes(a_local, q[r0 * rb:r1 * rb])
        b = ga.allocateTensor(G.GGMLType.F32, [N, K])
        ga.setTensorBytes(b, np.ascontiguousarray(x))  # B(j,k) at k*4N + 4j = x[k, j]
        d_local = ga.allocateTensor(G.GGMLType.F32, [N, max(r1 - r0, 1)])
        full = sh.forward(a_local, b, d_local).numpy()
        np.save(os.path.join(out_dir, f"rank{rank}.npy"), full)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("qt,M,K,N", [(2, 64, 256, 1), (6, 37, 128, 3), (3, 5, 64, 2)])
def test_row_sharded_world2_gloo(oracle, tmp_path, qt, M, K, N):
    import torch.multiprocessing as mp
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), qt, M, K, N, str(tmp_path)), nprocs=world, join=True)
    q = oracle.quantize(qt, random_weights(M * K, 0x5EED + 7))
    x = random_acts(K * N, 0x5EED + 8).reshape(K, N)
    ref = oracle.mat_mul_q(qt, q, M, K, x)  # [M, N]
    for r in range(world):
        got = np.load(tmp_path / f"rank{r}.npy")
        # same oracle arithmetic on both sides: the gather must reproduce it bit for bit
        assert got.shape == ref.shape
        assert np.array_equal(got.view(np.uint32), ref.astype(np.float32).view(np.uint32))


def test_shard_rows_cover_and_balance():
    import ggml_hip as G
    for M in (1, 7, 4096, 11008):
        for world in (1, 2, 3, 4, 8):
            spans = [G.shard_rows(M, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == M
            for (a0, a1), (b0, b1) in zip(spans, spans[1:]):
                assert a1 == b0
            assert max(r1 - r0 for r0, r1 in spans) == -(-M // world)


def test_row_slice_byte_offsets():
    import ggml_hip as G
    ga = G.GGMLGraphAllocator(device="host", defaultBufferSize=1 << 16)
    a = ga.allocateTensor(G.GGMLType.Q4_0, [256, 10])
    s = G.row_slice(a, 3, 7)
    assert s.ne[1] == 4 and s.dataOffset == a.dataOffset + 3 * (256 // 32) * 18


def _inplace_worker(rank, world, port, out_dir):
    """lk_sharded_plan's contract on gloo: rank r computes rows [r·M/P, (r+1)·M/P) of each node
    straight into their place in the FULL dst (shard_view of A and of dst), then an in-place
    all-gather fills in the other ranks' rows; the next node reads the gathered dst as its B.
    Local operator: the oracle (test-only); collective: gloo all_gather of the same chunks."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    import oracle as O
    import ggml_hip as G
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        K, M1, M2 = 256, 64, 96
        ga = G.GGMLGraphAllocator(device="host", defaultBufferSize=1 << 20)
        a1 = ga.allocateTensor(G.GGMLType.Q4_0, [K, M1])
        ga.setTensorBytes(a1, O.quantize(2, random_weights(M1 * K, 11)))
        a2 = ga.allocateTensor(G.GGMLType.Q8_0, [M1, M2])
        ga.setTensorBytes(a2, O.quantize(6, random_weights(M2 * M1, 12)))
        x = ga.allocateTensor(G.GGMLType.F32, [1, K])
        ga.setTensorBytes(x, random_acts(K, 13))
        d1 = ga.allocateTensor(G.GGMLType.F32, [1, M1])
        d2 = ga.allocateTensor(G.GGMLType.F32, [1, M2])
        buf = ga.buffers[0]
        for a, b, d in ((a1, x, d1), (a2, d1, d2)):  # node 2 reads node 1's gathered dst
            _oracle_compute(ga, None, G.shard_view(a, world, rank), b, G.shard_view(d, world, rank))
            M = d.ne[1]
            chunk = 4 * (M // world)
            mine = torch.from_numpy(buf[d.dataOffset + rank * chunk:d.dataOffset + (rank + 1) * chunk].copy())
            parts = [torch.empty_like(mine) for _ in range(world)]
            dist.all_gather(parts, mine)
            buf[d.dataOffset:d.dataOffset + world * chunk] = torch.cat(parts).numpy()
        np.save(os.path.join(out_dir, f"rank{rank}.npy"), buf[d2.dataOffset:d2.dataOffset + 4 * M2].view(np.float32))
    finally:
        dist.destroy_process_group()


def test_sharded_plan_inplace_layout_world2_gloo(oracle, tmp_path):
    import torch.multiprocessing as mp
    world = 2
    mp.spawn(_inplace_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    K, M1, M2 = 256, 64, 96
    q1 = oracle.quantize(2, random_weights(M1 * K, 11))
    q2 = oracle.quantize(6, random_weights(M2 * M1, 12))
    h = oracle.mat_mul_q(2, q1, M1, K, random_acts(K, 13).reshape(K, 1))
    ref = oracle.mat_mul_q(6, q2, M2, M1, h.reshape(M1, 1)).reshape(-1)
    for r in range(world):
        got = np.load(tmp_path / f"rank{r}.npy")
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


def test_shard_view_requires_exact_split():
    import ggml_hip as G
    ga = G.GGMLGraphAllocator(device="host", defaultBufferSize=1 << 16)
    d = ga.allocateTensor(G.GGMLType.F32, [1, 96])
    v = G.shard_view(d, 4, 3)
    assert v.ne[1] == 24 and v.dataOffset == d.dataOffset + 3 * 24 * 4
    with pytest.raises(ValueError):
        G.shard_view(ga.allocateTensor(G.GGMLType.F32, [1, 10]), 4, 0)
