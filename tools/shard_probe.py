"""Lab probe (the P = 8 prediction of the throughput legs): one rank's share of each
bench.py THROUGHPUT_LEGS leg at P = 1, 2, 4, 8 ranks, timed on this one GPU — the rank's M/P rows of
every matrix as its own lk_plan (the `local` form of bench.throughput_leg), rotating over enough distinct
weight copies that every pass streams >= 300 MB from HBM, graph-replayed. What a rank of a P-GPU node
computes per call is exactly this; the all-gather that completes the outputs is added in DESIGN §6 from
an xGMI estimate (it cannot run on one GPU).
Usage: python tools/shard_probe.py [P ...]   One JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "llama.kotlin_amd")]

import bench  # noqa: E402


def main():
    import torch
    import ggml_hip as G
    worlds = [int(a) for a in sys.argv[1:]] or [1, 2, 4, 8]
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    T = G.GGMLType
    out = {"device": torch.cuda.get_device_name(0), "legs": {}}
    for (name, shapes, N) in bench.THROUGHPUT_LEGS:
        leg = {}
        for P in worlds:
            geo = bench.leg_geometry(shapes, N, P)
            copies = geo["copies"]
            ga = G.GGMLGraphAllocator(device=str(dev), defaultBufferSize=16)
            gen = torch.Generator(device=dev)
            gen.manual_seed(7)
            xs = {K: ga.addBuffer(4 * K * N + 256) for K in {k for (_, k) in shapes}}
            for K, xb in xs.items():
                ga.buffers[xb][: 4 * K * N].copy_(torch.randn(K * N, generator=gen, device=dev).view(torch.uint8))
            qs = [G.quantizeTensor(torch.randn((M // P) * K, generator=gen, device=dev) * 0.02, T.Q4_0) for (M, K) in shapes]
            pitch = [(q.numel() + 255) // 256 * 256 for q in qs]
            wb = ga.addBuffer(copies * sum(pitch) + 256)
            db = ga.addBuffer(copies * sum((4 * N * (M // P) + 255) // 256 * 256 for (M, _) in shapes) + 256)
            plans, woff, doff = [], 0, 0
            for _ in range(copies):
                nodes = []
                for i, (M, K) in enumerate(shapes):
                    ga.buffers[wb][woff:woff + qs[i].numel()].copy_(qs[i])
                    nodes.append((G.GGMLTensor(T.Q4_0, [K, M // P], bufferId=wb, dataOffset=woff),
                                  G.GGMLTensor(T.F32, [N, K], bufferId=xs[K]),
                                  G.GGMLTensor(T.F32, [N, M // P], bufferId=db, dataOffset=doff)))
                    woff += pitch[i]
                    doff += (4 * N * (M // P) + 255) // 256 * 256
                plans.append(G.MulMatPlan(ga, nodes))
            s = torch.cuda.Stream(device=dev)

            def run():
                for p in plans:
                    p.launch(stream=s)

            G.debugRoute()  # clear
            per, graphed = bench._graph_time(torch, run, s, 5)
            per /= copies
            leg[f"P{P}"] = {"rank_us_per_call": round(per * 1e6, 3), "rank_alg_bytes": geo["rank_alg_bytes_per_call"],
                            "rank_GBps": round(geo["rank_alg_bytes_per_call"] / per / 1e9, 1),
                            "gather_bytes_in_per_rank": geo["gather_bytes_in_per_rank"],
                            "output_bytes_per_call": geo["output_bytes_per_call"], "copies": copies, "hip_graph": graphed,
                            "route": G.debugRoute()[:160]}
            for p in plans:
                p.close()
            del ga, qs
            torch.cuda.synchronize()
        out["legs"][name] = leg
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
