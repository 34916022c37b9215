"""lk_mul_mat_sharded: computeMatMul over host buffers with A's rows split over
the GPUs of one process. On a one-GPU box every shard maps to device 0 (shard r runs on
device r mod device count), which exercises the row split, the per-shard staging offsets
and the disjoint dst write-back exactly as on eight devices."""
import numpy as np
import pytest

from _util import parity_ok, random_acts, random_weights
from test_gpu_parity import gpu_matmul, noise_for

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("qt,M,K,N,P", [
    (2, 4096, 4096, 1, 8), (3, 70, 256, 1, 3), (6, 33, 320, 2, 2), (2, 5, 64, 1, 8),
    (2, 130, 512, 17, 4), (3, 11008, 4096, 1, 8), (6, 37, 11008, 1, 3),
])
def test_sharded_matches_single_and_oracle(gpu, oracle, qt, M, K, N, P):
    q = oracle.quantize(qt, random_weights(M * K, 0x5EED + M))
    x = random_acts(K * N, 0x5EED + K).reshape(K, N)
    single = gpu_matmul(qt, q, M, K, N, x, host=True)
    for pin in (False, True):
        got = gpu_matmul(qt, q, M, K, N, x, host=True, n_shards=P, pin=pin)
        if N == 1:  # one wave per row, sequential in k: the split cannot change a bit
            assert np.array_equal(got.view(np.uint32), single.view(np.uint32)), pin
        ref = oracle.mat_mul_q(qt, q, M, K, x, tight=True)
        ok, msg = parity_ok(got, ref, noise=noise_for(oracle, qt, q, M, K, x))
        assert ok, (pin, msg)


def test_sharded_strided_dst_and_offsets(gpu, oracle):
    qt, M, K, N = 2, 96, 256, 3
    q = oracle.quantize(qt, random_weights(M * K, 3))
    x = random_acts(K * N, 4).reshape(K, N)
    ref = oracle.mat_mul_q(qt, q, M, K, x)
    got = gpu_matmul(qt, q, M, K, N, x, a_off=36, b_off=20, d_off=8, dst_row_pad=5, host=True, n_shards=4)
    ok, msg = parity_ok(got, ref, noise=noise_for(oracle, qt, q, M, K, x))
    assert ok, msg


def test_sharded_falls_back_when_rows_straddle_blocks(gpu, oracle):
    """K % 32 != 0: rows are not byte ranges of A (flat-index blocks), so one device runs it."""
    qt, M, K, N = 2, 8, 40, 2
    q = oracle.quantize(qt, random_weights(M * K, 5))
    x = random_acts(K * N, 6).reshape(K, N)
    got = gpu_matmul(qt, q, M, K, N, x, host=True, n_shards=4)
    single = gpu_matmul(qt, q, M, K, N, x, host=True)
    assert np.array_equal(got.view(np.uint32), single.view(np.uint32))


def test_sharded_errors_and_pins(gpu, oracle):
    import ggml_hip as G
    ga = G.GGMLGraphAllocator(device="host", defaultBufferSize=1 << 16)
    a = ga.allocateTensor(G.GGMLType.Q4_0, [64, 8])
    b = ga.allocateTensor(G.GGMLType.F32, [1, 64])
    d = ga.allocateTensor(G.GGMLType.F32, [1, 8])
    with pytest.raises(G.IllegalArgumentException):
        G.computeMatMulSharded(ga, ga.context, a, b, d, 0)
    bad = ga.allocateTensor(G.GGMLType.F32, [1, 9])
    with pytest.raises(G.IllegalArgumentException):
        G.computeMatMulSharded(ga, ga.context, a, b, bad, 2)
    G.weightsEvictAll()
    G.weightsPinSharded(ga, a, 3)
    from ggml_hip import _lib
    assert _lib.load().lk_weights_cached_bytes() == 8 * 2 * 18
    G.weightsEvictAll()
    assert _lib.load().lk_weights_cached_bytes() == 0


def test_rccl_sharded_plan_world1_equals_plan(gpu, oracle):
    """The C-ABI RCCL path (lk_comm + lk_sharded_plan) at world size 1 on the one GPU of the box:
    bit-equal to lk_plan over the same nodes, and a second plan reading the first one's dst."""
    import torch
    import ggml_hip as G
    from _util import random_acts, random_weights
    comm = G.Comm.single()
    assert comm.nranks == 1
    K, F = 256, 384
    ga = G.GGMLGraphAllocator(defaultBufferSize=1 << 20)
    specs = [("q", 2, K, K), ("k", 3, K, K), ("v", 6, K, K), ("gate", 2, K, F), ("up", 2, K, F)]
    x = ga.allocateTensor(G.GGMLType.F32, [1, K]); ga.setTensorBytes(x, random_acts(K, 1))
    nodes, ref_nodes = [], []
    for i, (name, qt, k, m) in enumerate(specs):
        a = ga.allocateTensor(G.GGMLType(qt), [k, m]); ga.setTensorBytes(a, oracle.quantize(qt, random_weights(k * m, 10 + i)))
        d = ga.allocateTensor(G.GGMLType.F32, [1, m])
        dr = ga.allocateTensor(G.GGMLType.F32, [1, m])
        nodes.append((G.shard_view(a, 1, 0), x, d))
        ref_nodes.append((a, x, dr))
    plan = G.ShardedMulMatPlan(comm, ga, nodes)
    assert plan.numGathers == len(nodes)
    ref = G.MulMatPlan(ga, ref_nodes)
    # level 2 reads level 1's (gathered) outputs
    wd = ga.allocateTensor(G.GGMLType.Q4_0, [F, K]); ga.setTensorBytes(wd, oracle.quantize(2, random_weights(F * K, 99)))
    d2 = ga.allocateTensor(G.GGMLType.F32, [1, K])
    d2r = ga.allocateTensor(G.GGMLType.F32, [1, K])
    plan2 = G.ShardedMulMatPlan(comm, ga, [(G.shard_view(wd, 1, 0), nodes[4][2], d2)])
    ref2 = G.MulMatPlan(ga, [(wd, ref_nodes[4][2], d2r)])
    s = torch.cuda.Stream()
    for _ in range(2):
        plan.launch(stream=s); plan2.launch(stream=s)
        ref.launch(stream=s); ref2.launch(stream=s)
    torch.cuda.synchronize()
    for (_, _, d), (_, _, dr) in zip(nodes + [(None, None, d2)], ref_nodes + [(None, None, d2r)]):
        assert bytes(ga.tensorBytes(d).cpu().numpy()) == bytes(ga.tensorBytes(dr).cpu().numpy())
    plan.close(); plan2.close(); comm.close()


def test_rccl_sharded_plan_rejects_uneven_rows(gpu):
    import ggml_hip as G
    comm = G.Comm.single()
    ga = G.GGMLGraphAllocator(defaultBufferSize=1 << 16)
    a = ga.allocateTensor(G.GGMLType.Q4_0, [64, 8])
    b = ga.allocateTensor(G.GGMLType.F32, [1, 64])
    d = ga.allocateTensor(G.GGMLType.F32, [1, 16])  # A holds 8 rows of a 16-row dst at P = 1
    with pytest.raises(G.IllegalArgumentException):
        G.ShardedMulMatPlan(comm, ga, [(a, b, d)])
    comm.close()


def _llama_nodes(G, ga, oracle, shapes, seed=0):
    """Weights (ne=[K, M]) + activations on device buffers; returns [(a, x, dst)] per shape."""
    out = []
    for i, (M, K) in enumerate(shapes):
        a = ga.allocateTensor(G.GGMLType.Q4_0, [K, M])
        ga.setTensorBytes(a, oracle.quantize(2, random_weights(M * K, seed + 10 + i)))
        x = ga.allocateTensor(G.GGMLType.F32, [1, K])
        ga.setTensorBytes(x, random_acts(K, seed + 20 + i))
        out.append((a, x, ga.allocateTensor(G.GGMLType.F32, [1, M])))
    return out


def test_rccl_allgather_executes_at_world1_and_replays_in_a_hip_graph(gpu, oracle):
    """lk_sharded_plan_launch issues its RCCL group at world size 1 too (counted per communicator),
    and a HIP-graph capture of the launches replays bit-equal to lk_plan — over the Llama-7B shapes,
    the down projection (4096 x 11008, reading the up projection's gathered output) included."""
    import torch
    import ggml_hip as G
    comm = G.Comm.single()
    ga = G.GGMLGraphAllocator(defaultBufferSize=1 << 27)
    (wq, x, dq), (wu, _, du) = _llama_nodes(G, ga, oracle, [(4096, 4096), (11008, 4096)])
    wd = ga.allocateTensor(G.GGMLType.Q4_0, [11008, 4096])
    ga.setTensorBytes(wd, oracle.quantize(2, random_weights(4096 * 11008, 77)))
    dd = ga.allocateTensor(G.GGMLType.F32, [1, 4096])
    refs = [ga.allocateTensor(G.GGMLType.F32, [1, m]) for m in (4096, 11008, 4096)]
    plan1 = G.ShardedMulMatPlan(comm, ga, [(G.shard_view(wq, 1, 0), x, dq), (G.shard_view(wu, 1, 0), x, du)])
    plan2 = G.ShardedMulMatPlan(comm, ga, [(G.shard_view(wd, 1, 0), du, dd)])
    ref1 = G.MulMatPlan(ga, [(wq, x, refs[0]), (wu, x, refs[1])])
    ref2 = G.MulMatPlan(ga, [(wd, refs[1], refs[2])])
    s = torch.cuda.Stream()
    n0 = comm.numCollectives
    plan1.launch(stream=s); plan2.launch(stream=s)
    ref1.launch(stream=s); ref2.launch(stream=s)
    assert comm.numCollectives == n0 + 3  # one ncclAllGather per node, issued eagerly
    torch.cuda.synchronize()
    want = [bytes(ga.tensorBytes(r).cpu().numpy()) for r in refs]
    assert [bytes(ga.tensorBytes(d).cpu().numpy()) for d in (dq, du, dd)] == want
    for d in (dq, du, dd):
        ga.buffers[d.bufferId][d.dataOffset:d.dataOffset + 4 * d.ne[1]].zero_()
    torch.cuda.synchronize()
    hg = torch.cuda.CUDAGraph()
    with torch.cuda.graph(hg, stream=s):
        plan1.launch(stream=s); plan2.launch(stream=s)
    assert comm.numCollectives == n0 + 6  # captured
    for _ in range(3):
        hg.replay()
    torch.cuda.synchronize()
    assert [bytes(ga.tensorBytes(d).cpu().numpy()) for d in (dq, du, dd)] == want
    ok, msg = parity_ok(ga.tensorBytes(dd).cpu().numpy().view(np.float32).reshape(4096, 1),
                        oracle.mat_mul_q(2, oracle.quantize(2, random_weights(4096 * 11008, 77)), 4096, 11008,
                                         ga.tensorBytes(du).cpu().numpy().view(np.float32).reshape(11008, 1), tight=True))
    assert ok, msg
    del hg
    plan1.close(); plan2.close(); comm.close()


def _host_layer(G, ga, oracle, K=512, F=768, seed=0):
    """A Llama-style block on host buffers: q,k,v,gate,up from x; o from q; down from up."""
    x = ga.allocateTensor(G.GGMLType.F32, [1, K], name="x")
    ga.setTensorBytes(x, random_acts(K, seed + 1))
    nodes = []

    def node(name, qt, src, k, m, s):
        w = ga.allocateTensor(G.GGMLType(qt), [k, m], name="w" + name)
        ga.setTensorBytes(w, oracle.quantize(qt, random_weights(k * m, s)))
        d = ga.allocateTensor(G.GGMLType.F32, [1, m], name=name)
        nodes.append((w, src, d))
        return d

    q = node("q", 2, x, K, K, seed + 2)
    node("k", 3, x, K, K, seed + 3)
    node("v", 6, x, K, K, seed + 4)
    node("o", 2, q, K, K, seed + 5)
    node("g", 2, x, K, F, seed + 6)
    u = node("u", 2, x, K, F, seed + 7)
    node("d", 2, u, F, K, seed + 8)
    return nodes


@pytest.mark.parametrize("mode", ["rank", "init_all", "backend"])
def test_rccl_sharded_graph_equals_graph(gpu, oracle, mode):
    """lk_graph_create_sharded over the one GPU (a one-rank communicator from lk_comm_init_rank, or
    lk_comm_init_all over [0], or GGMLHipBackend(shardDevices=[0])): every weight node runs through a
    sharded plan and its in-place RCCL all-gather, and every result equals lk_graph's bit for bit,
    over repeated computes (eager, then HIP-graph replay)."""
    import ggml_hip as G
    ga = G.GGMLGraphAllocator(device="host", defaultBufferSize=1 << 22)
    nodes = _host_layer(G, ga, oracle)
    plain = G.ResidentGraph(ga, nodes)
    plain.compute()
    want = [bytes(ga.tensorBytes(d)) for _, _, d in nodes]
    for _, _, d in nodes:
        ga.setTensorBytes(d, np.zeros(4 * d.ne[1], np.uint8))
    if mode == "backend":
        dsts = []
        for a, b, d in nodes:
            d.op, d.src = G.GGMLOp.MUL_MAT, [a, b]
            dsts.append(d)
        be = G.GGMLHipBackend(ga, shardDevices=[0])
        for _ in range(3):
            assert be.graphCompute(G.GGMLCGraph(dsts, ga)) == G.GGMLStatus.SUCCESS
            assert [bytes(ga.tensorBytes(d)) for _, _, d in nodes] == want
        assert be.comms[0].numCollectives >= len(nodes)
        be.close()
        return
    comms = [G.Comm.single()] if mode == "rank" else G.Comm.init_all([0])
    g = G.ResidentGraph(ga, nodes, comms=comms)
    assert g.numSharded == len(nodes) and g.numLevels == plain.numLevels
    n0 = comms[0].numCollectives
    for i in range(3):
        g.compute()
        assert [bytes(ga.tensorBytes(d)) for _, _, d in nodes] == want, i
        for _, _, d in nodes:
            ga.setTensorBytes(d, np.zeros(4 * d.ne[1], np.uint8))
    assert comms[0].numCollectives >= n0 + len(nodes)
    g.close(); plain.close()
    for c in comms:
        c.close()


def test_comm_from_world1_nccl_process_group(gpu, oracle):
    """The bench's N > 1 set-up at world size 1: a torch.distributed NCCL (= RCCL) process group,
    Comm.from_process_group (rank 0's unique id broadcast through the group, lk_comm_init_rank on
    the current device), then a Llama-shape sharded plan captured in a HIP graph — bit-equal to
    lk_plan over the same nodes."""
    import socket
    import torch
    import torch.distributed as dist
    import ggml_hip as G
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    dev = torch.device("cuda", torch.cuda.current_device())
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
    try:
        comm = G.Comm.from_process_group()
        assert comm.nranks == 1 and comm.rank == 0 and comm.device == dev.index
        ga = G.GGMLGraphAllocator(defaultBufferSize=1 << 26)
        nodes = _llama_nodes(G, ga, oracle, [(4096, 4096), (11008, 4096)], seed=5)
        refs = [ga.allocateTensor(G.GGMLType.F32, [1, d.ne[1]]) for (_, _, d) in nodes]
        plan = G.ShardedMulMatPlan(comm, ga, [(G.shard_view(a, 1, 0), x, d) for (a, x, d) in nodes])
        ref = G.MulMatPlan(ga, [(a, x, r) for (a, x, _), r in zip(nodes, refs)])
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            ref.launch(stream=s)
        torch.cuda.synchronize()
        hg = torch.cuda.CUDAGraph()
        with torch.cuda.graph(hg, stream=s):
            plan.launch(stream=s)
        for _ in range(2):
            hg.replay()
        torch.cuda.synchronize()
        for (_, _, d), r in zip(nodes, refs):
            assert bytes(ga.tensorBytes(d).cpu().numpy()) == bytes(ga.tensorBytes(r).cpu().numpy())
        del hg
        plan.close(); comm.close()
    finally:
        dist.destroy_process_group()
