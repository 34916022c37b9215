"""Graph residency over host buffers (lk_graph_*): a MUL_MAT graph on
ByteArray-backed tensors computed with the activations kept in HBM between nodes. Every
result must equal the same nodes run one computeMatMul at a time (bit for bit: the same
kernels compute each node), and only graph inputs may cross PCIe on the way in."""
import os

import numpy as np
import pytest

from _util import random_acts, random_weights

pytestmark = pytest.mark.gpu


def _layer(ga, oracle, K=256, F=384, N=1, seed=0):
    """A Llama-style block on host buffers: q,k,v,gate,up from x; o from q; down from up."""
    import ggml_hip as G
    x = ga.allocateTensor(G.GGMLType.F32, [N, K], name="x")
    ga.setTensorBytes(x, random_acts(K * N, seed + 1))
    W, nodes = {}, []

    def weight(name, qt, k, m, s):
        t = ga.allocateTensor(G.GGMLType(qt), [k, m], name=name)
        ga.setTensorBytes(t, oracle.quantize(qt, random_weights(k * m, s)))
        W[name] = t
        return t

    def node(name, a, b, m):
        d = ga.allocateTensor(G.GGMLType.F32, [N, m], name=name)
        nodes.append((a, b, d))
        return d

    q = node("q", weight("wq", 2, K, K, seed + 2), x, K)
    node("k", weight("wk", 3, K, K, seed + 3), x, K)
    node("v", weight("wv", 6, K, K, seed + 4), x, K)
    node("o", weight("wo", 2, K, K, seed + 5), q, K)
    node("g", weight("wg", 2, K, F, seed + 6), x, F)
    u = node("u", weight("wu", 2, K, F, seed + 7), x, F)
    node("d", weight("wd", 2, F, K, seed + 8), u, K)
    return x, nodes


def _sequential(ga, nodes, routes=None):
    import ggml_hip as G
    for a, b, d in nodes:
        G.debugRoute()
        G.computeMatMul(ga, ga.context, a, b, d)
        if routes is not None:
            routes.append(G.debugRoute())
    return [bytes(ga.tensorBytes(d)) for _, _, d in nodes]


NAMES = ["q", "k", "v", "o", "g", "u", "d"]


def _oracle_check(ga, oracle, nodes, x, got):
    """Each node's bytes against the oracle on the inputs the node read (x, or the producing node's
    result in `got`: o reads q, d reads u). Returns {name: (ok, msg)}."""
    from test_gpu_parity import noise_for
    from _util import parity_ok
    out = {}
    xin = np.frombuffer(bytes(ga.tensorBytes(x)), np.float32)
    for i, (a, b, d) in enumerate(nodes):
        N, K, M = b.ne[0], a.ne[0], a.ne[1]
        src = {3: 0, 6: 5}.get(i)
        bv = xin if src is None else np.frombuffer(got[src], np.float32)
        xk = bv.reshape(K, N)
        q = np.frombuffer(bytes(ga.tensorBytes(a)), np.uint8)
        ref = oracle.mat_mul_q(int(a.type), q, M, K, xk)
        g = np.frombuffer(got[i], np.float32).reshape(M, N)
        out[NAMES[i]] = parity_ok(g, ref, noise=noise_for(oracle, int(a.type), q, M, K, xk))
    return out


@pytest.mark.parametrize("N", [1, 4, 32])  # 32: the level's Q4_0 nodes as one grouped pair launch (round 6)
def test_layer_graph_equals_sequential(gpu, oracle, N):
    """The resident graph and the node-by-node path must agree bit for bit, and BOTH must meet the
    parity bar against the oracle: a difference says which side is wrong, and the failure message
    carries the kernel route of every node (lk_debug_route) and the split-K counter state."""
    import ggml_hip as G
    assert G.syncCountersSum() == 0, "split-K counters not re-armed before the test"
    ga = G.GGMLGraphAllocator(device="host", defaultBufferSize=1 << 20)
    x, nodes = _layer(ga, oracle, N=N)
    routes = []
    want = _sequential(ga, nodes, routes)
    seq_ok = _oracle_check(ga, oracle, nodes, x, want)
    for _, _, d in nodes:
        ga.setTensorBytes(d, np.zeros(4 * d.ne[0] * d.ne[1], np.uint8))
    g = G.ResidentGraph(ga, nodes)
    assert g.numLevels == 2
    assert g.transferBytes(True) == 4 * N * 256  # only x goes up: weights pinned, q and u stay in HBM
    assert g.transferBytes(False) == sum(4 * d.ne[0] * d.ne[1] for _, _, d in nodes)
    G.debugRoute()
    g.compute()
    groute = G.debugRoute()
    got = [bytes(ga.tensorBytes(d)) for _, _, d in nodes]
    graph_ok = _oracle_check(ga, oracle, nodes, x, got)
    ctr = G.syncCountersSum()
    if N == 32:  # the first level's three Q4_0 nodes (q, g, u) run as one grouped launch
        assert "pairgroup<2,2>:n3" in groute, groute
    diag = "\n".join(f"  {n}: node-by-node {seq_ok[n]} route [{r}] | graph {graph_ok[n]}"
                      for n, r in zip(NAMES, routes)) + f"\n  graph route [{groute}]\n  counters {ctr}"
    if os.environ.get("LK_DIAG_DUMP") and not all(ok for ok, _ in seq_ok.values()):  # lab diagnostic
        np.savez(os.environ["LK_DIAG_DUMP"], want=np.frombuffer(want[6], np.float32), got=np.frombuffer(got[6], np.float32),
                 u=np.frombuffer(want[5], np.float32), wd=np.frombuffer(bytes(ga.tensorBytes(nodes[6][0])), np.uint8))
    assert all(ok for ok, _ in seq_ok.values()), "node-by-node result off the oracle:\n" + diag
    assert all(ok for ok, _ in graph_ok.values()), "graph result off the oracle:\n" + diag
    assert got == want, "graph != node-by-node (both within the bar):\n" + diag
    assert ctr == 0, diag
    # a new input is picked up by the next compute (the captured replay from here on)
    ga.setTensorBytes(x, random_acts(256 * N, 99))
    want2 = _sequential(ga, nodes)
    g.compute()
    got2 = [bytes(ga.tensorBytes(d)) for _, _, d in nodes]
    assert all(ok for ok, _ in _oracle_check(ga, oracle, nodes, x, got2).values())
    assert got2 == want2
    g.compute()  # replayed again: the same bytes
    assert [bytes(ga.tensorBytes(d)) for _, _, d in nodes] == want2
    assert G.syncCountersSum() == 0


def test_outputs_mask_keeps_intermediates_on_device(gpu, oracle):
    import ggml_hip as G
    ga = G.GGMLGraphAllocator(device="host", defaultBufferSize=1 << 20)
    _, nodes = _layer(ga, oracle)
    want = _sequential(ga, nodes)
    for _, _, d in nodes:
        ga.setTensorBytes(d, np.zeros(4 * d.ne[1], np.uint8))
    outs = [d.name in ("o", "d") for _, _, d in nodes]
    g = G.ResidentGraph(ga, nodes, outputs=outs)
    g.compute()
    for (_, _, d), w, o in zip(nodes, want, outs):
        got = bytes(ga.tensorBytes(d))
        assert got == (w if o else bytes(len(w))), d.name
    assert g.transferBytes(False) == 4 * 256 * 2


def test_f32_chain_and_war_hazard(gpu):
    """An F32 x F32 node whose A is an earlier node's dst, and a node that overwrites the
    bytes an earlier node reads (it must run after the read)."""
    import ggml_hip as G
    rng = np.random.default_rng(1)
    ga = G.GGMLGraphAllocator(device="host", defaultBufferSize=1 << 16)
    a0 = ga.allocateTensor(G.GGMLType.F32, [32, 16])
    b0 = ga.allocateTensor(G.GGMLType.F32, [8, 32])
    d0 = ga.allocateTensor(G.GGMLType.F32, [8, 16])       # = A of node 1 viewed as [K=8, M=16]
    b1 = ga.allocateTensor(G.GGMLType.F32, [3, 8])
    d1 = ga.allocateTensor(G.GGMLType.F32, [3, 16])
    a2 = ga.allocateTensor(G.GGMLType.F32, [8, 4])
    b2 = ga.allocateTensor(G.GGMLType.F32, [3, 8])
    for t in (a0, b0, b1, a2, b2):
        ga.setTensorBytes(t, rng.standard_normal(t.ne[0] * t.ne[1]).astype(np.float32))
    a1 = G.GGMLTensor(G.GGMLType.F32, [8, 16], bufferId=d0.bufferId, dataOffset=d0.dataOffset)
    # node 2 writes into b1's bytes after node 1 read them (WAR): [N=3, M=4] = 48 B of b1's 96
    d2 = G.GGMLTensor(G.GGMLType.F32, [3, 4], bufferId=b1.bufferId, dataOffset=b1.dataOffset)
    nodes = [(a0, b0, d0), (a1, b1, d1), (a2, b2, d2)]
    snap = ga.buffers[0].copy()
    want = _sequential(ga, nodes)
    ga.buffers[0][:] = snap
    g = G.ResidentGraph(ga, nodes)
    assert g.numLevels == 3  # node 2 overwrites the b1 bytes node 1 reads: after node 1
    g.compute()
    assert [bytes(ga.tensorBytes(d)) for _, _, d in nodes] == want


def test_strided_dst_gap_bytes_survive(gpu, oracle):
    import ggml_hip as G
    ga = G.GGMLGraphAllocator(device="host", defaultBufferSize=1 << 16)
    M, K, N = 40, 128, 2
    a = ga.allocateTensor(G.GGMLType.Q4_0, [K, M])
    ga.setTensorBytes(a, oracle.quantize(2, random_weights(M * K, 5)))
    b = ga.allocateTensor(G.GGMLType.F32, [N, K])
    ga.setTensorBytes(b, random_acts(N * K, 6))
    raw = ga.allocateTensor(G.GGMLType.F32, [N + 3, M])  # rows padded by 3 floats of sentinel
    ga.setTensorBytes(raw, np.full((N + 3) * M, 7.25, np.float32))
    d = G.GGMLTensor(G.GGMLType.F32, [N, M], nb=[4, 4 * (N + 3), 4 * (N + 3) * M, 4 * (N + 3) * M],
                     bufferId=raw.bufferId, dataOffset=raw.dataOffset)
    g = G.ResidentGraph(ga, [(a, b, d)])
    g.compute()
    out = np.frombuffer(bytes(ga.tensorBytes(raw)), np.float32).reshape(M, N + 3)
    assert np.all(out[:, N:] == 7.25)
    got = out[:, :N].copy()
    ga.setTensorBytes(raw, np.full((N + 3) * M, 7.25, np.float32))
    G.computeMatMul(ga, ga.context, a, b, d)
    ref = np.frombuffer(bytes(ga.tensorBytes(raw)), np.float32).reshape(M, N + 3)[:, :N]
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


def test_backend_graph_compute_host_uses_resident_graph(gpu, oracle):
    import ggml_hip as G
    ga = G.GGMLGraphAllocator(device="host", defaultBufferSize=1 << 20)
    _, nodes = _layer(ga, oracle)
    want = _sequential(ga, nodes)
    dsts = []
    for a, b, d in nodes:
        d.op, d.src = G.GGMLOp.MUL_MAT, [a, b]
        d.flags = G.tensor.GGML_TENSOR_FLAG_OUTPUT  # every result wanted on the host
        ga.setTensorBytes(d, np.zeros(4 * d.ne[1], np.uint8))
        dsts.append(d)
    be = G.GGMLHipBackend(ga)
    assert be.graphCompute(G.GGMLCGraph(dsts, ga)) == G.GGMLStatus.SUCCESS
    assert [bytes(ga.tensorBytes(d)) for d in dsts] == want


def _mul_mat_nodes(G, nodes):
    dsts = []
    for a, b, d in nodes:
        d.op, d.src = G.GGMLOp.MUL_MAT, [a, b]
        dsts.append(d)
    return dsts


def test_backend_writes_back_only_what_leaves_the_graph(gpu, oracle):
    """With wholeGraphs=True the backend keeps results that only later MUL_MATs consume in HBM
    (q -> o, up -> down); every other result (and anything flagged isOutput) reaches the host
    bytes, equal to the per-node path bit for bit."""
    import ggml_hip as G
    ga = G.GGMLGraphAllocator(device="host", defaultBufferSize=1 << 20)
    _, nodes = _layer(ga, oracle)
    want = _sequential(ga, nodes)
    dsts = _mul_mat_nodes(G, nodes)
    assert G.backend.writeBackMask(dsts, wholeGraph=True) == [d.name not in ("q", "u") for d in dsts]
    dsts[0].flags = G.tensor.GGML_TENSOR_FLAG_OUTPUT  # q is also wanted by the caller
    for d in dsts:
        ga.setTensorBytes(d, np.zeros(4 * d.ne[1], np.uint8))
    be = G.GGMLHipBackend(ga, wholeGraphs=True)
    assert be.graphCompute(G.GGMLCGraph(dsts, ga)) == G.GGMLStatus.SUCCESS
    for d, w in zip(dsts, want):
        got = bytes(ga.tensorBytes(d))
        assert got == (w if d.name != "u" else bytes(len(w))), d.name
    be.free()


def test_backend_cache_keys_on_shapes(gpu):
    """A graph rebuilt per token at the same offsets with another shape (an F32 MUL_MAT whose
    K grows, like attention over a growing KV length) must not hit the old plan."""
    import ggml_hip as G
    rng = np.random.default_rng(3)
    ga = G.GGMLGraphAllocator(device="host", defaultBufferSize=1 << 16)
    a_raw = ga.allocateTensor(G.GGMLType.F32, [64, 16])
    b_raw = ga.allocateTensor(G.GGMLType.F32, [2, 64])
    d_raw = ga.allocateTensor(G.GGMLType.F32, [2, 16])
    ga.setTensorBytes(a_raw, rng.standard_normal(64 * 16).astype(np.float32))
    ga.setTensorBytes(b_raw, rng.standard_normal(2 * 64).astype(np.float32))
    be = G.GGMLHipBackend(ga)
    for K in (8, 16, 32, 16):
        a = G.GGMLTensor(G.GGMLType.F32, [K, 16], bufferId=0, dataOffset=a_raw.dataOffset)
        b = G.GGMLTensor(G.GGMLType.F32, [2, K], bufferId=0, dataOffset=b_raw.dataOffset)
        d = G.GGMLTensor(G.GGMLType.F32, [2, 16], bufferId=0, dataOffset=d_raw.dataOffset,
                         op=G.GGMLOp.MUL_MAT, src=[a, b])
        assert be.graphCompute(G.GGMLCGraph([d], ga)) == G.GGMLStatus.SUCCESS
        got = bytes(ga.tensorBytes(d))
        G.computeMatMul(ga, ga.context, a, b, d)
        assert got == bytes(ga.tensorBytes(d)), K
    be.free()


def test_backend_weight_generation(gpu, oracle):
    """The caller rewrites weight bytes and bumps the backend's generation: the next
    graphCompute reads the new weights."""
    import ggml_hip as G
    ga = G.GGMLGraphAllocator(device="host", defaultBufferSize=1 << 20)
    _, nodes = _layer(ga, oracle)
    dsts = _mul_mat_nodes(G, nodes)
    be = G.GGMLHipBackend(ga)
    assert be.graphCompute(G.GGMLCGraph(dsts, ga)) == G.GGMLStatus.SUCCESS
    a = nodes[0][0]  # wq
    q = oracle.quantize(2, random_weights(256 * 256, 77))
    ga.buffers[a.bufferId][a.dataOffset:a.dataOffset + q.size] = q  # in-place, as the Kotlin caller writes
    be.bumpWeightGeneration()
    assert be.graphCompute(G.GGMLCGraph(dsts, ga)) == G.GGMLStatus.SUCCESS
    got = [bytes(ga.tensorBytes(d)) for d in dsts]
    G.weightsEvictAll()
    want = _sequential(ga, nodes)
    for d, g_, w in zip(dsts, got, want):
        if d.name not in ("q", "u"):
            assert g_ == w, d.name
    be.free()


def test_backend_split_subgraph_results_reach_a_later_cpu_consumer(gpu, oracle):
    """GGMLScheduler.executeGraphSplit (core/GGMLScheduler.kt:245-258) hands the backend one split
    of a larger graph and sets no output flags; a CPU node of a later split may read any result
    (here: ADD(q, o) on the host after the split {q = Wq·x, o = Wo·q}). By default every result of
    the split reaches the ByteArrays, so the CPU consumer reads q's current bytes."""
    import ggml_hip as G
    assert G.backend.writeBackMask([object(), object()]) == [True, True]
    ga = G.GGMLGraphAllocator(device="host", defaultBufferSize=1 << 20)
    _, nodes = _layer(ga, oracle)
    split = [nodes[0], nodes[3]]  # q from x, o from q
    want = _sequential(ga, split)
    dsts = _mul_mat_nodes(G, split)
    for d in dsts:
        ga.setTensorBytes(d, np.zeros(4 * d.ne[1], np.uint8))
    be = G.GGMLHipBackend(ga)
    assert be.graphCompute(G.GGMLCGraph(dsts, ga)) == G.GGMLStatus.SUCCESS
    q = np.frombuffer(bytes(ga.tensorBytes(dsts[0])), np.float32)
    o = np.frombuffer(bytes(ga.tensorBytes(dsts[1])), np.float32)
    assert [q.tobytes(), o.tobytes()] == want
    cpu_add = q + o  # the later split's CPU node
    assert np.array_equal(cpu_add, np.frombuffer(want[0], np.float32) + np.frombuffer(want[1], np.float32))
    be.free()
