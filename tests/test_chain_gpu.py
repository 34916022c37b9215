"""Chain plans (lk_plan_create_chain): dependent stages of N = 1 MUL_MAT nodes in one persistent
launch, a device-side grid barrier between stages. Each stage here reads what the previous
stage wrote, so a missing or leaky barrier shows up as wrong values. Results must be
bit-identical to launching the nodes one by one in stage order (every row's dot runs the same
wave code wherever the row lands), launch after launch (the counters re-arm), also when the
launch is replayed from a HIP graph."""
import numpy as np
import pytest

import oracle as O
from _util import parity_ok, random_acts, random_weights


def _chain(G, ga, qt, dims, fanout, seed):
    """dims = [K0, M1, M2, ...]: stage s has `fanout[s]` nodes M_{s+1} x M_s; every node of stage
    s+1 reads the output of node 0 of stage s. Returns (nodes, stages, x0 tensor, outputs)."""
    nodes, stages, outs = [], [], []
    xb = ga.addBuffer(4 * dims[0] + 64)
    x = G.GGMLTensor(G.GGMLType.F32, [1, dims[0]], bufferId=xb)
    ga.setTensorBytes(x, random_acts(dims[0], seed).view(np.uint8))
    cur = x
    host_w = []
    for s in range(len(dims) - 1):
        K, M = dims[s], dims[s + 1]
        stage_out = []
        for f in range(fanout[s]):
            q = O.quantize(qt, random_weights(M * K, seed + 10 * s + f, std=1.0 / np.sqrt(K)))
            a = G.GGMLTensor(G.GGMLType(qt), [K, M], bufferId=ga.addBuffer(q.size))
            ga.setTensorBytes(a, q)
            d = G.GGMLTensor(G.GGMLType.F32, [1, M], bufferId=ga.addBuffer(4 * M + 64))
            nodes.append((a, cur, d))
            stages.append(s)
            stage_out.append(d)
            host_w.append((q, M, K))
        outs.append(stage_out)
        cur = stage_out[0]
    return nodes, stages, x, outs, host_w


CHAINS = [
    (2, [4096, 4096, 11008, 4096], [3, 1, 2]),      # Llama-7B-like: {q,k,v} -> o-ish -> {gate, up}-ish
    (2, [1024, 512, 2048, 1024, 256, 4096], [1, 2, 1, 1, 3]),
    (6, [2048, 2048, 1024], [2, 1]),                # Q8_0
    (3, [4096, 384, 4096], [1, 1]),                 # Q4_1, a 384-row stage: most waves hold no row
    # uneven arrivals: a 256-row stage between two long ones (16 workgroups hold rows there, the
    # rest arrive at once), then an 11008-wide activation read right after it
    (2, [4096, 11008, 256, 11008, 4096], [1, 1, 1, 1]),
]


@pytest.mark.gpu
@pytest.mark.parametrize("case", CHAINS, ids=lambda c: f"{c[0]}-" + "x".join(map(str, c[1])))
def test_chain_equals_stage_by_stage(gpu, case):
    import torch
    import ggml_hip as G
    qt, dims, fanout = case
    ga = G.GGMLGraphAllocator(device="cuda", defaultBufferSize=16)
    nodes, stages, x, outs, host_w = _chain(G, ga, qt, dims, fanout, seed=len(dims) * 7 + qt)
    # reference: one node at a time, in order
    for (a, b, d) in nodes:
        G.computeMatMul(ga, ga.context, a, b, d)
    torch.cuda.synchronize()
    ref = [ga.tensorBytes(d).cpu().numpy().view(np.float32).copy() for (_, _, d) in nodes]
    # the last stage against the oracle too (through the whole chain on the host)
    xs = ga.tensorBytes(x).cpu().numpy().view(np.float32).copy()
    cur = xs
    for s in range(len(dims) - 1):
        idx = [i for i, st in enumerate(stages) if st == s]
        q, M, K = host_w[idx[0]]
        y = O.mat_mul_q(qt, q, M, K, cur.reshape(K, 1)).reshape(-1)
        ok, msg = parity_ok(ref[idx[0]].reshape(-1, 1), y.reshape(-1, 1))
        assert ok, (s, msg)
        cur = ref[idx[0]]  # the GPU's own stage output feeds the next oracle stage
    plan = G.MulMatPlan(ga, nodes, stages=stages)
    assert plan.numLaunches == 1
    for rep in range(3):
        for (_, _, d) in nodes:
            ga.tensorBytes(d).fill_(0xFF)
        plan.launch()
        torch.cuda.synchronize()
        assert not plan.timedOut()
        for i, (_, _, d) in enumerate(nodes):
            got = ga.tensorBytes(d).cpu().numpy().view(np.float32)
            assert np.array_equal(got.view(np.uint32), ref[i].view(np.uint32)), (rep, i, stages[i])


@pytest.mark.gpu
def test_chain_graph_replay(gpu):
    import torch
    import ggml_hip as G
    ga = G.GGMLGraphAllocator(device="cuda", defaultBufferSize=16)
    nodes, stages, x, outs, _ = _chain(G, ga, 2, [4096, 4096, 4096, 4096], [2, 2, 1], seed=3)
    for (a, b, d) in nodes:
        G.computeMatMul(ga, ga.context, a, b, d)
    torch.cuda.synchronize()
    ref = [ga.tensorBytes(d).cpu().numpy().copy() for (_, _, d) in nodes]
    plan = G.MulMatPlan(ga, nodes, stages=stages)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        plan.launch(stream=s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        plan.launch(stream=s)
    for rep in range(4):
        for (_, _, d) in nodes:
            ga.tensorBytes(d).zero_()
        torch.cuda.synchronize()
        with torch.cuda.stream(s):
            g.replay()
        torch.cuda.synchronize()
        for i, (_, _, d) in enumerate(nodes):
            assert np.array_equal(ga.tensorBytes(d).cpu().numpy(), ref[i]), (rep, i)
    assert not plan.timedOut()


@pytest.mark.gpu
def test_chain_rejects_what_it_cannot_stream(gpu):
    import ggml_hip as G
    ga = G.GGMLGraphAllocator(device="cuda", defaultBufferSize=16)
    nodes, stages, *_ = _chain(G, ga, 2, [4096, 512, 512], [1, 1], seed=1)
    with pytest.raises(G.IllegalArgumentException):
        G.MulMatPlan(ga, nodes, stages=[1, 0])
    with pytest.raises(G.IllegalArgumentException):
        G.MulMatPlan(ga, nodes, stages=[0, 2])
    # N = 2 is not a streaming GEMV node
    a, b, d = nodes[0]
    b2 = G.GGMLTensor(G.GGMLType.F32, [2, 4096], bufferId=ga.addBuffer(8 * 4096))
    d2 = G.GGMLTensor(G.GGMLType.F32, [2, 512], bufferId=ga.addBuffer(8 * 512))
    with pytest.raises(NotImplementedError):
        G.MulMatPlan(ga, [(a, b2, d2)], stages=[0])


@pytest.mark.gpu
@pytest.mark.parametrize("qt", [2, 3, 10])
def test_plan_fuses_adjacent_nodes_bit_exactly(gpu, qt):
    """lk_plan_create fuses adjacent nodes that read the same activations and whose weight rows and
    output rows continue each other in memory (a model's q, k, v back to back: one even row split).
    Three such nodes in one weight buffer and one output buffer, plus a fourth whose weights sit
    after a gap (not fused), as a plan and as a chain stage: every output bit-equal to the nodes
    launched one by one (Q4_0, Q4_1, Q4_K)."""
    import ggml_hip as G
    K, Ms = 1024, (512, 256, 768, 512)
    bb = {2: 18, 3: 20, 10: 144}[qt]
    per = 256 if qt == 10 else 32
    row = K // per * bb
    ga = G.GGMLGraphAllocator(device="cuda", defaultBufferSize=16)
    wbuf = ga.addBuffer(sum(Ms) * row + 4096 + 256)
    obuf = ga.addBuffer(4 * sum(Ms) + 256)
    xb = ga.addBuffer(4 * K + 64)
    x = G.GGMLTensor(G.GGMLType.F32, [1, K], bufferId=xb)
    ga.setTensorBytes(x, random_acts(K, 7).view(np.uint8))
    nodes, woff, ooff = [], 0, 0
    for i, M in enumerate(Ms):
        if i == 3:
            woff += 4096  # a gap: not contiguous with the node before
        if qt == 10:  # Q4_K: random codes and scales, small d / dmin
            q = np.random.default_rng(40 + i).integers(0, 256, M * K // 256 * 144, dtype=np.uint8)
            q.reshape(-1, 144)[:, 0:4] = np.frombuffer(np.array([0.01, 0.001], np.float16).tobytes(), np.uint8)
        else:
            q = O.quantize(qt, random_weights(M * K, 40 + i, std=1.0 / np.sqrt(K)))
        a = G.GGMLTensor(G.GGMLType(qt), [K, M], bufferId=wbuf, dataOffset=woff)
        ga.setTensorBytes(a, q)
        d = G.GGMLTensor(G.GGMLType.F32, [1, M], bufferId=obuf, dataOffset=ooff)
        nodes.append((a, x, d))
        woff += M * row
        ooff += 4 * M
    want = []
    for (a, b, d) in nodes:
        G.computeMatMul(ga, None, a, b, d)
        want.append(bytes(ga.tensorBytes(d)))
    for form in ("plan", "chain"):
        ga.setTensorBytes(G.GGMLTensor(G.GGMLType.F32, [1, sum(Ms)], bufferId=obuf), np.zeros(4 * sum(Ms), np.uint8))
        p = G.MulMatPlan(ga, nodes) if form == "plan" else G.MulMatPlan(ga, nodes, stages=[0] * len(nodes))
        p.launch()
        import torch
        torch.cuda.synchronize()
        got = [bytes(ga.tensorBytes(d)) for (_, _, d) in nodes]
        assert got == want, form
        p.close()
