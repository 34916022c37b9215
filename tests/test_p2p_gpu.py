"""The one-shot peer-write multi-GPU path (lk_p2p_*) on the one GPU of the
box: at world size 1 (peer = self: no copies, the signal and the gate) bit-equal to lk_sharded_plan
and lk_plan, and with P = 2 / 4 ranks on device 0 — each rank its own activation and dst buffers,
so the push kernel really copies every rank's rows into every other rank's dst and the next plan
really waits on signals the other ranks' pushes raise — bit-equal on every rank to lk_plan over the
unsharded weights. Shapes are Llama-7B's (4096 x 4096, 11008 x 4096, the down projection reading
the gathered up projection)."""
import numpy as np
import pytest

from _util import random_acts, random_weights

pytestmark = pytest.mark.gpu


def _weights(G, ga, oracle, seed=0):
    shapes = {"q": (4096, 4096), "up": (11008, 4096), "down": (4096, 11008)}
    w = {}
    for i, (name, (M, K)) in enumerate(shapes.items()):
        t = ga.allocateTensor(G.GGMLType.Q4_0, [K, M])
        ga.setTensorBytes(t, oracle.quantize(2, random_weights(M * K, seed + 10 + i)))
        w[name] = t
    return w


def _reference(G, ga, w, x, s):
    refs = {k: ga.allocateTensor(G.GGMLType.F32, [1, m]) for k, m in (("q", 4096), ("up", 11008), ("down", 4096))}
    p1 = G.MulMatPlan(ga, [(w["q"], x, refs["q"]), (w["up"], x, refs["up"])])
    p2 = G.MulMatPlan(ga, [(w["down"], refs["up"], refs["down"])])
    p1.launch(stream=s); p2.launch(stream=s)
    return refs


def _bytes(ga, t):
    return bytes(ga.tensorBytes(t).cpu().numpy())


def test_p2p_world1_equals_sharded_plan(gpu, oracle):
    import torch
    import ggml_hip as G
    ga = G.GGMLGraphAllocator(defaultBufferSize=1 << 27)
    w = _weights(G, ga, oracle)
    x = ga.allocateTensor(G.GGMLType.F32, [1, 4096]); ga.setTensorBytes(x, random_acts(4096, 3))
    s = torch.cuda.Stream()
    refs = _reference(G, ga, w, x, s)
    comm = G.Comm.single()
    sd = {k: ga.allocateTensor(G.GGMLType.F32, [1, m]) for k, m in (("q", 4096), ("up", 11008), ("down", 4096))}
    sp1 = G.ShardedMulMatPlan(comm, ga, [(G.shard_view(w["q"], 1, 0), x, sd["q"]), (G.shard_view(w["up"], 1, 0), x, sd["up"])])
    sp2 = G.ShardedMulMatPlan(comm, ga, [(G.shard_view(w["down"], 1, 0), sd["up"], sd["down"])])
    sp1.launch(stream=s); sp2.launch(stream=s)
    group = G.P2PGroup([0])
    pd = {k: ga.allocateTensor(G.GGMLType.F32, [1, m]) for k, m in (("q", 4096), ("up", 11008), ("down", 4096))}
    pp1 = G.P2PMulMatPlan(group, ga, [[(G.shard_view(w["q"], 1, 0), x, pd["q"]), (G.shard_view(w["up"], 1, 0), x, pd["up"])]])
    pp2 = G.P2PMulMatPlan(group, ga, [[(G.shard_view(w["down"], 1, 0), pd["up"], pd["down"])]])
    pp1.launch(s)
    # the push kernel's signal must have arrived before anything is gated on it
    assert pp1.signal(0) == 1
    pp2.launch(s)  # gated on pp1's signal >= 1
    for _ in range(2):
        pp1.launch(s); pp2.launch(s)
    torch.cuda.synchronize()
    assert pp1.signal(0) == 3 and pp2.signal(0) == 3 and pp1.numLaunches == 3
    for k in ("q", "up", "down"):
        assert _bytes(ga, pd[k]) == _bytes(ga, sd[k]) == _bytes(ga, refs[k]), k
    for p in (pp1, pp2, sp1, sp2):
        p.close()
    group.close(); comm.close()


@pytest.mark.parametrize("P", [2, 4])
def test_p2p_ranks_on_one_gpu_push_and_gate(gpu, oracle, P):
    import torch
    import ggml_hip as G
    ga = G.GGMLGraphAllocator(defaultBufferSize=1 << 27)
    w = _weights(G, ga, oracle, seed=P)
    xs = random_acts(4096, 7 + P)
    x0 = ga.allocateTensor(G.GGMLType.F32, [1, 4096]); ga.setTensorBytes(x0, xs)
    s = torch.cuda.Stream()
    refs = _reference(G, ga, w, x0, s)
    ranks1, ranks2, dsts = [], [], []
    for r in range(P):
        x = ga.allocateTensor(G.GGMLType.F32, [1, 4096]); ga.setTensorBytes(x, xs)
        d = {k: ga.allocateTensor(G.GGMLType.F32, [1, m]) for k, m in (("q", 4096), ("up", 11008), ("down", 4096))}
        for t in d.values():
            ga.setTensorBytes(t, np.full(4 * t.ne[1], 0xFF, np.uint8))  # every row must be written
        ranks1.append([(G.shard_view(w["q"], P, r), x, d["q"]), (G.shard_view(w["up"], P, r), x, d["up"])])
        ranks2.append([(G.shard_view(w["down"], P, r), d["up"], d["down"])])
        dsts.append(d)
    group = G.P2PGroup([0] * P)
    assert group.nranks == P
    p1 = G.P2PMulMatPlan(group, ga, ranks1)
    p2 = G.P2PMulMatPlan(group, ga, ranks2)
    p1.launch(s)
    assert p1.signal(0) == P and p1.signal(P - 1) == P  # every rank's push counted on every rank
    p2.launch(s)
    for _ in range(2):
        p1.launch(s); p2.launch(s)
    torch.cuda.synchronize()
    assert all(p.signal(r) == 3 * P for p in (p1, p2) for r in range(P))
    for r in range(P):
        for k in ("q", "up", "down"):
            assert _bytes(ga, dsts[r][k]) == _bytes(ga, refs[k]), (r, k)
    p1.close(); p2.close(); group.close()


def test_p2p_refuses_capture_and_split_streams(gpu, oracle):
    import torch
    import ggml_hip as G
    ga = G.GGMLGraphAllocator(defaultBufferSize=1 << 20)
    a = ga.allocateTensor(G.GGMLType.Q4_0, [256, 64]); ga.setTensorBytes(a, oracle.quantize(2, random_weights(64 * 256, 1)))
    x = ga.allocateTensor(G.GGMLType.F32, [1, 256]); ga.setTensorBytes(x, random_acts(256, 2))
    d0 = ga.allocateTensor(G.GGMLType.F32, [1, 64])
    d1 = ga.allocateTensor(G.GGMLType.F32, [1, 64])
    group = G.P2PGroup([0, 0])
    plan = G.P2PMulMatPlan(group, ga, [[(G.shard_view(a, 2, 0), x, d0)], [(G.shard_view(a, 2, 1), x, d1)]])
    with pytest.raises(G.IllegalArgumentException):
        plan.launch([torch.cuda.Stream(), torch.cuda.Stream()])  # two ranks on one device, two streams
    assert plan.numLaunches == 0
    s = torch.cuda.Stream()
    torch.cuda.synchronize()
    hg = torch.cuda.CUDAGraph()
    with pytest.raises(Exception):
        with torch.cuda.graph(hg, stream=s):
            plan.launch(s)
    assert plan.numLaunches == 0
    plan.launch(s)
    torch.cuda.synchronize()
    assert plan.signal(0) == 2
    with pytest.raises(G.IllegalArgumentException):  # uneven rows
        G.P2PMulMatPlan(group, ga, [[(a, x, d0)], [(a, x, d1)]])
    plan.close(); group.close()
