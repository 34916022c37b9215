"""Lab probe (DESIGN §6b budget): the persistent multi-GPU chain (lk_p2p_chain) with P = 1, 2, 4 ranks
on the one GPU of the box against the one-launch chain plan (lk_plan_create_chain) and stream-ordered
launches, over Llama-7B layers in the dependent decode order (4 stages per layer). On one GPU the
ranks split its CUs, so the bytes per stage and the CUs streaming them are those of the single-rank
chain: what changes is the barrier (every rank's stage, announced to every rank) and the row stores
into P copies. One JSON line: us per layer for each form, eager launches timed between events.
Both chains are also timed by host wall clock around launch + synchronize (`*_wall_*`: includes one
launch and one synchronize per rep, the only clock that spans every rank's stream).
Usage: python tools/chain_probe.py [layers]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "llama.kotlin_amd")]

import bench  # noqa: E402


def main():
    import torch
    import ggml_hip as G
    layers = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    T = G.GGMLType
    ga = G.GGMLGraphAllocator(device=str(dev), defaultBufferSize=16)
    # weights once; activations per rank (identical layouts), up to 4 ranks
    wbytes = sum(layers * ((M * K // 32 * 18 + 255) // 256 * 256) for (_, M, K) in bench.LAYER_MATS)
    wbuf = ga.addBuffer(wbytes + 256)
    w, off = [], 0
    for L in range(layers):
        d = {}
        for (name, M, K) in bench.LAYER_MATS:
            t = G.GGMLTensor(T.Q4_0, [K, M], bufferId=wbuf, dataOffset=off)
            ga.buffers[wbuf][off:off + M * K // 32 * 18].copy_(G.quantizeTensor(torch.randn(M * K, device=dev) * 0.02, T.Q4_0))
            off += (M * K // 32 * 18 + 255) // 256 * 256
            d[name] = t
        w.append(d)
    src = {"q": "x", "k": "x", "v": "x", "o": "q", "gate": "o", "up": "o", "down": "up"}
    stage_of = {"q": 0, "k": 0, "v": 0, "o": 1, "gate": 2, "up": 2, "down": 3}
    x0 = torch.randn(bench.HIDDEN, device=dev)

    def acts(buf):
        t, o = {}, 0
        t["x"] = G.GGMLTensor(T.F32, [1, bench.HIDDEN], bufferId=buf, dataOffset=0)
        o = 4 * bench.HIDDEN
        for L in range(layers):
            for (name, M, _) in bench.LAYER_MATS:
                t[(L, name)] = G.GGMLTensor(T.F32, [1, M], bufferId=buf, dataOffset=o)
                o += (4 * M + 255) // 256 * 256
        return t

    act_bytes = 4 * bench.HIDDEN + layers * sum((4 * M + 255) // 256 * 256 for (_, M, _) in bench.LAYER_MATS) + 256

    def nodes_of(t, a_of):
        nodes, stages = [], []
        for L in range(layers):
            for (name, M, K) in bench.LAYER_MATS:
                s = src[name]
                b = (t["x"] if L == 0 else t[(L - 1, "down")]) if s == "x" else t[(L, s)]
                nodes.append((a_of(w[L][name]), b, t[(L, name)]))
                stages.append(4 * L + stage_of[name])
        return nodes, stages

    out = {"layers": layers}
    s = torch.cuda.Stream(device=dev)
    t1 = acts(ga.addBuffer(act_bytes))
    ga.buffers[t1["x"].bufferId][: 4 * bench.HIDDEN].copy_(x0.view(torch.uint8))
    nodes, stages = nodes_of(t1, lambda a: a)

    def timed(fn, reps=10):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(reps):
            fn()
        e1.record(s)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / reps / layers

    import time

    def wall(fn, reps=10):  # launch + synchronize per rep: the form the multi-rank chain is timed in
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
            torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e6 / reps / layers

    # stream-ordered: one plan per stage
    plans = [G.MulMatPlan(ga, [n for n, st in zip(nodes, stages) if st == k]) for k in range(max(stages) + 1)]
    out["stream_ordered_us_per_layer"] = round(timed(lambda: [p.launch(stream=s) for p in plans]), 3)
    chain = G.MulMatPlan(ga, nodes, stages=stages)
    out["chain_plan_us_per_layer"] = round(timed(lambda: chain.launch(stream=s)), 3)
    out["chain_plan_wall_us_per_layer"] = round(wall(lambda: chain.launch(stream=s)), 3)
    out["chain_plan_timed_out"] = chain.timedOut()
    for P in (1, 2, 4):
        ranks = []
        for r in range(P):
            t = acts(ga.addBuffer(act_bytes))
            ga.buffers[t["x"].bufferId][: 4 * bench.HIDDEN].copy_(x0.view(torch.uint8))
            rn, _ = nodes_of(t, lambda a, r=r: G.shard_view(a, P, r))
            ranks.append(rn)
        group = G.P2PGroup([0] * P)
        pc = G.P2PChain(group, ga, ranks, stages)

        def run():
            pc.launch()  # the group's CU-partitioned streams

        out[f"p2p_chain_P{P}_wall_us_per_layer"] = round(wall(run), 3)
        out[f"p2p_chain_P{P}_timed_out"] = pc.timedOut()
        last = ranks[-1][-1][2]
        ref = t1[(layers - 1, "down")]
        out[f"p2p_chain_P{P}_equal"] = bool(torch.equal(ga.tensorBytes(last), ga.tensorBytes(ref)))
        pc.close()
        group.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
