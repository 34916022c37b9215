"""The persistent multi-GPU chain (lk_p2p_chain) on the one GPU of the box: P ranks on
device 0, each on its own CU-masked stream with its own activation buffers, run two Llama-style layers
in the dependent decode order ({q,k,v} -> o -> {gate,up} -> down -> next layer: 8 stages) as ONE launch
per rank. Every rank streams only its row shard of every weight, stores each row into every rank's
copy of the outputs and waits, at each of the 7 stage boundaries, for every rank's stage. Every
rank's every output must equal the same nodes run stage by stage through lk_plan on the whole
weights, bit for bit (each row is the same wave's sequential sum either way)."""
import numpy as np
import pytest

from _util import random_acts, random_weights

pytestmark = pytest.mark.gpu

H, F = 1024, 2816  # hidden / FFN width: rows split evenly over 1, 2 and 4 ranks; K % 64 == 0
LAYER = [("q", H, H, "x"), ("k", H, H, "x"), ("v", H, H, "x"), ("o", H, H, "q"),
         ("gate", F, H, "o"), ("up", F, H, "o"), ("down", H, F, "up")]
STAGE_OF = {"q": 0, "k": 0, "v": 0, "o": 1, "gate": 2, "up": 2, "down": 3}


def _activations(G, ga, buf, layers):
    """x of layer 0 and every node's dst at fixed offsets of buffer `buf` (one layout per rank)."""
    t, off = {}, 0

    def alloc(name, m):
        nonlocal off
        t[name] = G.GGMLTensor(G.GGMLType.F32, [1, m], bufferId=buf, dataOffset=off)
        off += (4 * m + 255) // 256 * 256

    alloc("x0", H)
    for L in range(layers):
        for (name, m, _, _) in LAYER:
            alloc(f"{name}{L}", m)
    return t


def _nodes(w, t, layers, a_of):
    nodes, stages = [], []
    for L in range(layers):
        for (name, m, k, src) in LAYER:
            if src == "x":  # layer L reads the previous layer's down projection
                b = t["x0"] if L == 0 else t[f"down{L - 1}"]
            else:
                b = t[f"{src}{L}"]
            nodes.append((a_of(w[f"{name}{L}"]), b, t[f"{name}{L}"]))
            stages.append(4 * L + STAGE_OF[name])
    return nodes, stages


@pytest.mark.parametrize("P", [1, 2, 4])
def test_p2p_chain_ranks_on_one_gpu(gpu, oracle, P):
    import torch
    import ggml_hip as G
    layers = 2
    ga = G.GGMLGraphAllocator(defaultBufferSize=16)
    wbuf = ga.addBuffer(layers * 7 * F * H * 18 // 32 + 4096)
    w, off = {}, 0
    for L in range(layers):
        for i, (name, m, k, _) in enumerate(LAYER):
            w[f"{name}{L}"] = G.GGMLTensor(G.GGMLType.Q4_0, [k, m], bufferId=wbuf, dataOffset=off)
            ga.setTensorBytes(w[f"{name}{L}"], oracle.quantize(2, random_weights(m * k, 100 * L + i + P)))
            off += (m * k // 32 * 18 + 255) // 256 * 256
    act_bytes = 4 * (H + layers * sum(m for (_, m, _, _) in LAYER)) + 256 * (1 + 7 * layers)
    x0 = random_acts(H, 5 + P)
    # reference: the whole weights, stage by stage
    ref = _activations(G, ga, ga.addBuffer(act_bytes), layers)
    ga.setTensorBytes(ref["x0"], x0)
    nodes, stages = _nodes(w, ref, layers, lambda a: a)
    s = torch.cuda.Stream()
    for st in range(max(stages) + 1):
        G.MulMatPlan(ga, [nd for nd, sg in zip(nodes, stages) if sg == st]).launch(stream=s)
    torch.cuda.synchronize()
    want = {k: ga.tensorBytes(v).cpu().numpy().tobytes() for k, v in ref.items()}
    # P ranks, each with its own activation buffer of the same layout
    ranks, acts = [], []
    for r in range(P):
        t = _activations(G, ga, ga.addBuffer(act_bytes), layers)
        ga.setTensorBytes(t["x0"], x0)
        for k, v in t.items():
            if k != "x0":
                ga.setTensorBytes(v, np.full(4 * v.ne[1], 0xFF, np.uint8))  # every row must be written
        rn, rs = _nodes(w, t, layers, lambda a, r=r: G.shard_view(a, P, r))
        assert rs == stages
        ranks.append(rn)
        acts.append(t)
    group = G.P2PGroup([0] * P)
    chain = G.P2PChain(group, ga, ranks, stages)
    for it in range(3):
        chain.launch()  # the group's CU-partitioned per-rank streams
        torch.cuda.synchronize()
        assert not chain.timedOut(), it
        for r in range(P):
            for k, v in acts[r].items():
                assert ga.tensorBytes(v).cpu().numpy().tobytes() == want[k], (it, r, k)
    assert chain.numLaunches == 3
    chain.close()
    group.close()


def test_p2p_chain_refuses_a_shared_stream_and_uneven_layouts(gpu, oracle):
    import torch
    import ggml_hip as G
    ga = G.GGMLGraphAllocator(defaultBufferSize=16)
    a = G.GGMLTensor(G.GGMLType.Q4_0, [256, 64], bufferId=ga.addBuffer(64 * 256 // 32 * 18 + 256))
    ga.setTensorBytes(a, oracle.quantize(2, random_weights(64 * 256, 1)))
    bufs = [ga.addBuffer(4096), ga.addBuffer(4096)]
    xs = [G.GGMLTensor(G.GGMLType.F32, [1, 256], bufferId=b) for b in bufs]
    ds = [G.GGMLTensor(G.GGMLType.F32, [1, 64], bufferId=b, dataOffset=1024) for b in bufs]
    for x in xs:
        ga.setTensorBytes(x, random_acts(256, 2))
    group = G.P2PGroup([0, 0])
    chain = G.P2PChain(group, ga, [[(G.shard_view(a, 2, r), xs[r], ds[r])] for r in range(2)], [0])
    s = torch.cuda.Stream()
    with pytest.raises(G.IllegalArgumentException):
        chain.launch([s, s])  # two ranks on one device wait for each other: one stream would serialise them
    assert chain.numLaunches == 0
    chain.launch()
    torch.cuda.synchronize()
    assert not chain.timedOut() and chain.numLaunches == 1
    chain.close()
    d_off = G.GGMLTensor(G.GGMLType.F32, [1, 64], bufferId=bufs[1], dataOffset=2048)
    d2 = [G.GGMLTensor(G.GGMLType.F32, [1, 64], bufferId=bufs[0], dataOffset=1536), ds[1]]
    with pytest.raises(G.NotOffloadedError):  # rank 1's two dsts sit at another offset than rank 0's
        G.P2PChain(group, ga, [[(G.shard_view(a, 2, r), xs[r], ds[r]), (G.shard_view(a, 2, r), xs[r], [d2[0], d_off][r])]
                               for r in range(2)], [0, 0])
    group.close()
