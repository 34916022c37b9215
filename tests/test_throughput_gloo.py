"""The north star's "4096x4096xbatch throughput at 1/2/4/8 GPUs" legs of bench.py,
host logic on the CPU:
  * leg_geometry: every leg splits over 1, 2, 4 and 8 ranks; each rank streams more distinct weight
    bytes per timed pass than the 256 MiB Infinity Cache holds; the per-rank bytes and flops add up
    to the whole call's; the all-gather's incoming bytes per rank;
  * the legs' data path at world size 2 over gloo: each rank quantizes the same full matrix (same
    seed), keeps its row shard, computes its rows in place inside the FULL dst (here with the oracle,
    test-only: on the GPU box the HIP kernels through lk_sharded_plan), and an all-gather of the
    per-rank chunks (the in-place ncclAllGather's layout) completes dst on every rank — equal to the
    oracle's unsharded result on both ranks, bit for bit.
The GPU side of the same legs is tests/test_throughput_gpu.py."""
import os
import socket

import numpy as np
import pytest

from _util import random_acts, random_weights


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_leg_geometry_every_world(world):
    import bench
    for (name, shapes, N) in bench.THROUGHPUT_LEGS:
        g = bench.leg_geometry(shapes, N, world)
        w_full = sum(M * K // 32 * 18 for (M, K) in shapes)
        assert g["copies"] * w_full / world >= 300e6 > 256 * 2 ** 20, name  # beyond the Infinity Cache
        assert g["rank_alg_bytes_per_call"] * world >= w_full, name
        assert g["rank_flop_per_call"] * world == g["useful_flop_per_call"], name
        assert g["gather_bytes_in_per_rank"] == g["output_bytes_per_call"] * (world - 1) // world, name
        assert g["alg_bytes_per_call"] == sum(bench.alg_bytes(M, K, N) for (M, K) in shapes), name
    with pytest.raises(ValueError):
        bench.leg_geometry([(4095, 4096)], 1, 2)


def _worker(rank, world, port, M, K, N, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    import oracle as O
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q = O.quantize(2, random_weights(M * K, 0xC0FFEE))  # every rank: the same full matrix
        x = random_acts(K * N, 0xC0FFEE + 1).reshape(K, N)
        rb, per = K // 32 * 18, M // world
        shard = q[rank * per * rb:(rank + 1) * per * rb]
        full = np.full((M, N), np.nan, np.float32)  # dst(n, m) at m*4N + 4n: row m's N outputs contiguous
        full[rank * per:(rank + 1) * per] = O.mat_mul_q(2, shard, per, K, x)  # the rank's rows, in place
        t = torch.from_numpy(full.reshape(-1))
        chunks = list(t.split(per * N))
        dist.all_gather(chunks, chunks[rank].clone())  # the in-place all-gather's layout
        np.save(os.path.join(out_dir, f"rank{rank}.npy"), torch.cat(chunks).numpy().reshape(M, N))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("M,K,N", [(256, 512, 1), (128, 256, 32), (64, 256, 512)])
def test_throughput_leg_world2_gloo(oracle, tmp_path, M, K, N):
    import torch.multiprocessing as mp
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), M, K, N, str(tmp_path)), nprocs=world, join=True)
    q = oracle.quantize(2, random_weights(M * K, 0xC0FFEE))
    x = random_acts(K * N, 0xC0FFEE + 1).reshape(K, N)
    want = oracle.mat_mul_q(2, q, M, K, x)
    for r in range(world):
        got = np.load(tmp_path / f"rank{r}.npy")
        assert got.tobytes() == want.astype(np.float32).tobytes(), r
