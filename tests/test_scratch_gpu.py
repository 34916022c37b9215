"""Lifetimes and states of the batched kernels' device scratch (round 5).

The batched kernels (N > 1) share per-device scratch: activation fragments, split-K slabs and
per-tile counters. A HIP graph captured from them (a ResidentGraph's replay, a caller's capture)
bakes those pointers in, so an outgrown buffer is retired instead of freed (csrc/lk_hip.hip,
GemmScratch); counters are zeroed on the launch's stream when allocated and re-armed by the kernels.
These tests build the states directly rather than hoping a test order recreates them:
  * a graph captured before the scratch grows is replayed after it;
  * counters of every split-K route read zero after every call, results on the oracle;
  * kpart's two K slices into a page-locked host output region (no float atomics there).
Parity is against the oracle (core/GGMLComputeOps.kt:70-145) at the §8c bar."""
import re

import numpy as np
import pytest

from _util import parity_ok, random_acts, random_weights
from test_gpu_parity import gpu_matmul, noise_for
from test_graph_gpu import NAMES, _layer, _oracle_check

pytestmark = pytest.mark.gpu


def _check_oracle(oracle, qt, q, M, K, x, got):
    ref = oracle.mat_mul_q(qt, q, M, K, x, tight=True, threads=16)
    ok, msg = parity_ok(got, ref, noise=noise_for(oracle, qt, q, M, K, x))
    assert ok, msg


def test_captured_graph_survives_scratch_growth(gpu, oracle):
    """A resident graph (N = 4 layer: kpart, skinny and gemm_q_mfma nodes) captured, then calls that
    outgrow the scratch, then the captured replay: the same bytes as before, on the oracle."""
    import ggml_hip as G
    ga = G.GGMLGraphAllocator(device="host", defaultBufferSize=1 << 20)
    x, nodes = _layer(ga, oracle, N=4, seed=40)
    g = G.ResidentGraph(ga, nodes)
    g.compute()
    g.compute()  # the second compute captures the HIP graph and launches it
    before = [bytes(ga.tensorBytes(d)) for _, _, d in nodes]
    for n, (ok, msg) in _oracle_check(ga, oracle, nodes, x, before).items():
        assert ok, (n, msg)
    e0 = G.debugScratchEpoch()
    # activation fragments grow with N·K: wide-kernel calls of growing N until the scratch moves
    M, K = 16, 16384
    q = oracle.quantize(2, random_weights(M * K, 41))
    for N in (256, 1024, 2048):
        xb = random_acts(K * N, 42 + N).reshape(K, N)
        got = gpu_matmul(2, q, M, K, N, xb)
        _check_oracle(oracle, 2, q, M, K, xb, got)
        if G.debugScratchEpoch() > e0:
            break
    assert G.debugScratchEpoch() > e0, "no call outgrew the scratch"
    for _, _, d in nodes:
        ga.setTensorBytes(d, np.zeros(4 * d.ne[0] * d.ne[1], np.uint8))
    g.compute()  # replay of the graph captured before the growth
    after = [bytes(ga.tensorBytes(d)) for _, _, d in nodes]
    assert after == before
    assert G.syncCountersSum() == 0
    g.close()


# every split-K route with counters or slabs, on host and device buffers: (qt, M, K, N, route word)
ROUTES = [
    (2, 256, 384, 4, "gemm_q_"),        # 216-B rows: not skinny-eligible; 12 K slices, tile counters
                                        # (gemm_q_lds with slack past A's bytes, else gemm_q_mfma)
    (2, 4096, 4096, 8, "kpart"),        # two K slices added into dst
    (2, 11008, 4096, 32, "pair"),       # eight slices, reduce launch
    (3, 4096, 4096, 64, "w32<3,2,2,2>"), # Q4_1 at N > 32 (round 6): one slice per tile, no counters
    (2, 512, 4096, 64, "w32<2,2,2,2>"), # few tiles: K split over workgroups, last arriver per tile (tcnt)
    (6, 4096, 4096, 8, "skinny"),       # Q8_0
    (6, 4096, 4096, 64, "wide"),        # Q8_0: last arriver per tile (tcnt)

    (3, 96, 1184, 40, "gemm_q_mfma"),   # Q4_1, 37 blocks per row: neither wide- nor LDS-eligible
]


@pytest.mark.parametrize("host", [True, False])
def test_split_k_counters_zero_after_every_route(gpu, oracle, host):
    """Interleaved split-K routes, each checked against the oracle; after each call every counter
    word (wide tcnt and the gemm_q_mfma / gemm_q_lds tile counters) reads zero."""
    import ggml_hip as G
    cases = []
    for (qt, M, K, N, word) in ROUTES:
        q = oracle.quantize(qt, random_weights(M * K, M + K))
        xb = random_acts(K * N, K + N).reshape(K, N)
        ref = oracle.mat_mul_q(qt, q, M, K, xb, tight=True, threads=16)
        cases.append((qt, M, K, N, word, q, xb, ref))
    for rep in range(2):
        for (qt, M, K, N, word, q, xb, ref) in cases:
            G.debugRoute()
            got = gpu_matmul(qt, q, M, K, N, xb, host=host)
            route = G.debugRoute()
            assert word in route, (word, route)
            ok, msg = parity_ok(got, ref, noise=noise_for(oracle, qt, q, M, K, xb))
            assert ok, (rep, word, route, msg)
            assert G.syncCountersSum() == 0, (rep, word, route)


@pytest.mark.parametrize("N", [4, 16])
def test_kpart_two_slices_into_host_output_region(gpu, oracle, N):
    """Llama q and gate shapes (K = 4096: kpart's two K slices) in a resident graph over host buffers,
    outputs direct (page-locked host memory): the slices go through slabs and a reduce launch there
    (float atomics only into device memory), bit-equal to computeMatMul, on the oracle."""
    import ggml_hip as G
    K = 4096
    ga = G.GGMLGraphAllocator(device="host", defaultBufferSize=1 << 26)
    x = ga.allocateTensor(G.GGMLType.F32, [N, K])
    xb = random_acts(K * N, 50 + N)
    ga.setTensorBytes(x, xb)
    nodes, ws = [], []
    for i, M in enumerate((4096, 11008)):
        w = ga.allocateTensor(G.GGMLType.Q4_0, [K, M])
        q = oracle.quantize(2, random_weights(M * K, 60 + i))
        ga.setTensorBytes(w, q)
        d = ga.allocateTensor(G.GGMLType.F32, [N, M])
        nodes.append((w, x, d))
        ws.append((q, M))
    want = []
    for (w, b, d) in nodes:
        G.debugRoute()
        G.computeMatMul(ga, ga.context, w, b, d)
        r = G.debugRoute()
        assert "kpart<2,1>:s2" in r and r.split("kpart")[1].split()[0].endswith("a"), r  # device scratch dst: atomics
        want.append(bytes(ga.tensorBytes(d)))
        ga.setTensorBytes(d, np.zeros(4 * N * d.ne[1], np.uint8))
    g = G.ResidentGraph(ga, nodes)
    for it in range(3):  # eager, captured, replayed
        G.debugRoute()
        g.compute()
        r = G.debugRoute()
        if it == 0:
            ks = [t for t in r.split() if t.startswith("kpart")]
            assert len(ks) == 2 and all(not t.endswith("a") for t in ks), r  # host region: no atomics
        got = [bytes(ga.tensorBytes(d)) for _, _, d in nodes]
        assert got == want, it
    for (q, M), gb in zip(ws, got):
        _check_oracle(oracle, 2, q, M, K, xb.reshape(K, N), np.frombuffer(gb, np.float32).reshape(M, N))
    g.close()


def test_concurrent_streams_do_not_share_scratch(gpu, oracle):
    """The state behind round 4's intermittent resident-graph failure, built directly: batched calls on a
    torch stream (device buffers) still in flight — queued behind a sleep — while the host path runs
    batched calls of its own on the library stream. Round 4 shared one scratch per device between the
    two (activation fragments, slabs, tile counters), so the host call could read fragments or slabs
    the other stream's launch was writing; scratch is per (device, stream) since round 5. Every result
    on the oracle."""
    import torch
    import ggml_hip as G
    qt, M, K, N = 2, 256, 384, 4  # the graph test's down projection: gemm_q_*, 12 K slices
    q = oracle.quantize(qt, random_weights(M * K, 70))
    xs = [random_acts(K * N, 71 + i).reshape(K, N) for i in range(2)]
    refs = [oracle.mat_mul_q(qt, q, M, K, x) for x in xs]
    noise = [noise_for(oracle, qt, q, M, K, x) for x in xs]
    dga = G.GGMLGraphAllocator(device="cuda", defaultBufferSize=16)
    a = G.GGMLTensor(G.GGMLType.Q4_0, [K, M], bufferId=dga.addBuffer(q.size + 256))
    b = G.GGMLTensor(G.GGMLType.F32, [N, K], bufferId=dga.addBuffer(4 * K * N + 256))
    dsts = [G.GGMLTensor(G.GGMLType.F32, [N, M], bufferId=dga.addBuffer(4 * M * N + 256)) for _ in range(16)]
    dga.setTensorBytes(a, q)
    dga.setTensorBytes(b, np.ascontiguousarray(xs[1]))
    s = torch.cuda.Stream()
    torch.cuda.synchronize()
    with torch.cuda.stream(s):
        torch.cuda._sleep(2_000_000)  # ~1 ms: the device calls below start while the host calls run
        for d in dsts:
            G.computeMatMul(dga, None, a, b, d, stream=s)
    for i in range(8):  # host path on the library stream meanwhile (x0, a different input)
        got = gpu_matmul(qt, q, M, K, N, xs[0], host=True)
        ok, msg = parity_ok(got, refs[0], noise=noise[0])
        assert ok, (i, msg)
    torch.cuda.synchronize()
    for j, d in enumerate(dsts):
        got = dga.tensorBytes(d).cpu().numpy().view(np.float32).reshape(M, N)
        ok, msg = parity_ok(got, refs[1], noise=noise[1])
        assert ok, (j, msg)
    assert G.syncCountersSum() == 0


def test_split_k_behind_a_busy_null_stream(gpu, oracle):
    """Round 4 zeroed newly grown tile counters with hipMemset on the null stream, which the library's
    non-blocking stream does not wait for. Host-path calls of the graph test's
    down-projection shape (gemm_q_*: 12 K slices, a counter per tile, the sc1 hand-off), each queued
    behind ~10 ms of torch work on the default (null) stream, after recycled device memory was filled
    with -1: no tile may come back unwritten, every result on the oracle, counters zero after. Since
    round 5 the counters are zeroed by hipMemsetAsync on the launch stream, at a 4096-tile floor that
    no split-K grid reaches (split K stops at ~2 workgroups per CU)."""
    import torch
    import ggml_hip as G
    K, N, RB = 384, 4, 384 // 32 * 18
    sq = torch.randn(2048, 2048, device="cuda") / 64
    for M in (256, 128 * 40, 128 * 41 + 64):
        q = oracle.quantize(2, random_weights(M * K, M % 1000))
        x = random_acts(K * N, M % 1000 + 1).reshape(K, N)
        junk = torch.full((1 << 22,), -1, dtype=torch.int32, device="cuda")  # recycled memory is not zero
        del junk
        torch.cuda.empty_cache()
        torch.cuda.synchronize()
        y = sq
        for _ in range(60):  # the null stream busy; nothing waits for it
            y = y @ sq
        G.debugRoute()
        got = gpu_matmul(2, q, M, K, N, x, host=True)
        route = G.debugRoute()
        m = re.search(r"gemm_q_\w+<[^>]*>:t\d+s(\d+)", route)
        assert m and int(m.group(1)) > 1, route  # split K
        assert not any((got[t:t + 64] == 0).all() for t in range(0, M, 64)), (M, route)  # no unwritten tile
        _check_oracle(oracle, 2, q, M, K, x, got)
    torch.cuda.synchronize()
    assert G.syncCountersSum() == 0


@pytest.mark.parametrize("value", [1, 5, 11, 1000])
def test_poked_tile_counter_is_rearmed(gpu, oracle, value):
    """VERDICT r5 item 6, the round-4 mechanism made a directed test: a gemm_q_* split-K tile counter
    set non-zero before the call (lk_debug_poke_gemm_counter) must never leave a tile unwritten — the
    library re-arms the counters it uses on the launch stream before every split-K launch. Device
    buffers on an explicit stream (the poke and the call are stream-ordered), result on the oracle, no
    all-zero tile, counters zero after."""
    import torch
    import ggml_hip as G
    qt, M, K, N = 2, 128 * 6, 384, 4  # the graph test's down-projection geometry: 12 K slices per tile
    q = oracle.quantize(qt, random_weights(M * K, 80 + value))
    x = random_acts(K * N, 81 + value).reshape(K, N)
    ref = oracle.mat_mul_q(qt, q, M, K, x)
    dga = G.GGMLGraphAllocator(device="cuda", defaultBufferSize=16)
    a = G.GGMLTensor(G.GGMLType.Q4_0, [K, M], bufferId=dga.addBuffer(q.size + 256))
    b = G.GGMLTensor(G.GGMLType.F32, [N, K], bufferId=dga.addBuffer(4 * K * N + 256))
    d = G.GGMLTensor(G.GGMLType.F32, [N, M], bufferId=dga.addBuffer(4 * M * N + 256))
    dga.setTensorBytes(a, q)
    dga.setTensorBytes(b, np.ascontiguousarray(x))
    s = torch.cuda.Stream()
    torch.cuda.synchronize()
    tiles = 0
    for rep in range(3):  # unpoked (learns the tile count), every tile poked, tile 0 alone poked
        for t in range(tiles if rep == 1 else min(tiles, 1) if rep == 2 else 0):
            G.debugPokeGemmCounter(t, value, stream=s)
        dga.setTensorBytes(d, np.zeros(4 * M * N, np.uint8))
        torch.cuda.synchronize()
        G.debugRoute()
        G.computeMatMul(dga, None, a, b, d, stream=s)
        s.synchronize()
        route = G.debugRoute()
        m = re.search(r"gemm_q_\w+<[^>]*>:t(\d+)s(\d+)", route)
        assert m and int(m.group(2)) > 1, route  # the split-K route with tile counters
        tiles = int(m.group(1))
        got = dga.tensorBytes(d).cpu().numpy().view(np.float32).reshape(M, N)
        assert not any((got[t:t + 64] == 0).all() for t in range(0, M, 64)), (value, route)
        ok, msg = parity_ok(got, ref, noise=noise_for(oracle, qt, q, M, K, x))
        assert ok, (value, rep, route, msg)
    assert G.syncCountersSum() == 0


def test_scratch_release_frees_a_streams_scratch(gpu, oracle):
    """scratch per (device, stream) never shrank. lk_scratch_release frees one
    stream's scratch; calls on that stream afterwards allocate afresh and stay right."""
    import torch
    import ggml_hip as G
    qt, M, K, N = 2, 512, 4096, 256  # wide GEMM: activation fragments + split-K slabs
    q = oracle.quantize(qt, random_weights(M * K, 90))
    x = random_acts(K * N, 91).reshape(K, N)
    ref = oracle.mat_mul_q(qt, q, M, K, x, tight=True, threads=16)
    dga = G.GGMLGraphAllocator(device="cuda", defaultBufferSize=16)
    a = G.GGMLTensor(G.GGMLType.Q4_0, [K, M], bufferId=dga.addBuffer(q.size + 256))
    b = G.GGMLTensor(G.GGMLType.F32, [N, K], bufferId=dga.addBuffer(4 * K * N + 256))
    d = G.GGMLTensor(G.GGMLType.F32, [N, M], bufferId=dga.addBuffer(4 * M * N + 256))
    dga.setTensorBytes(a, q)
    dga.setTensorBytes(b, np.ascontiguousarray(x))
    s = torch.cuda.Stream()
    torch.cuda.synchronize()
    base = G.scratchBytes()
    for rep in range(2):
        G.computeMatMul(dga, None, a, b, d, stream=s)
        s.synchronize()
        held = G.scratchBytes()
        assert held > base, (rep, held, base)
        got = dga.tensorBytes(d).cpu().numpy().view(np.float32).reshape(M, N)
        ok, msg = parity_ok(got, ref, noise=noise_for(oracle, qt, q, M, K, x))
        assert ok, (rep, msg)
        G.scratchRelease(stream=s)
        assert G.scratchBytes() == base, (rep, G.scratchBytes(), base)
