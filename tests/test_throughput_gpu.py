"""bench.py's multi_gpu_throughput legs on the one GPU of the box, through the
same code the driver's N-GPU runs execute: lk_sharded_plan over a one-rank RCCL communicator, the
serial and the split-stream (overlapped gather) schedules, graph-captured. The gathered output of the
first call is checked against the oracle (core/GGMLComputeOps.kt:120-145 restated) at the §8c bar, on
small shapes and on the C5 shape."""
import numpy as np
import pytest

from _util import parity_ok
from test_gpu_parity import noise_for

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shapes,N", [([(512, 1024)], 1), ([(768, 2048)], 32), ([(512, 1024), (256, 2048)], 8),
                                      ([(4096, 4096)], 512)])
def test_throughput_leg_world1_on_the_oracle(gpu, oracle, shapes, N):
    import torch
    import bench
    import ggml_hip as G
    comm = G.Comm.single()
    keep = {}
    out = bench.throughput_leg(torch, G, torch.device("cuda", 0), comm, 1, 0, None, "t", shapes, N, reps=2, keep=keep,
                               min_rank_bytes=2e6)
    comm.close()
    assert out["check"]["ok"], out["check"]
    assert out["ranks_seen_by_rccl"] == 1
    for k in ("local", "serial", "overlap"):
        assert out[k]["us_per_call"] > 0 and out[k]["hip_graph"], (k, out[k])
    M, K = keep["M"], keep["K"]
    ref = oracle.mat_mul_q(2, keep["q"], M, K, np.ascontiguousarray(keep["x"]), tight=True, threads=16)
    x = np.ascontiguousarray(keep["x"])
    ok, msg = parity_ok(keep["got"], ref, noise=noise_for(oracle, 2, keep["q"], M, K, x) if N > 1 else None)
    assert ok, msg
