"""Lab: Q4_K x F32 at batch 1 per launch (rotating copies, graph-replayed, as bench.next_rows) over
several shapes; run once with LK_KQ_STREAM=0 (kquant_n1_kernel) and once with 1 (the stream kernel)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "llama.kotlin_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
import ggml_hip as G  # noqa: E402

G.load_library()
dev = torch.device("cuda", 0)
T = G.GGMLType
out = {}
QN = os.environ.get("KQ_TYPE", "Q4_K")
for M, K in ((4096, 4096), (6144, 4096), (8192, 4096), (11008, 4096), (4096, 11008), (32000, 4096), (1024, 4096)):
    nblk, bb = M * K // 256, {"Q4_K": 144, "Q2_K": 84}[QN]
    so = 0 if QN == "Q4_K" else 80
    nb = nblk * bb
    copies = max(2, min(32, (300 << 20) // nb))
    g = G.GGMLGraphAllocator(device=str(dev), defaultBufferSize=16)
    wb, xb, db = g.addBuffer(copies * nb + 256), g.addBuffer(4 * K + 256), g.addBuffer(4 * M * copies + 256)
    w = g.buffers[wb][: copies * nb].view(copies * nblk, bb)
    w.copy_(torch.randint(0, 256, w.shape, dtype=torch.uint8, device=dev))
    w[:, so:so + 4].copy_(torch.tensor([0.01, 0.001], dtype=torch.float16).view(torch.uint8).to(dev))
    g.buffers[xb][: 4 * K].copy_(torch.randn(K, device=dev).view(torch.uint8))
    nodes = [(G.GGMLTensor(getattr(T, QN), [K, M], bufferId=wb, dataOffset=c * nb), G.GGMLTensor(T.F32, [1, K], bufferId=xb),
              G.GGMLTensor(T.F32, [1, M], bufferId=db, dataOffset=4 * M * c)) for c in range(copies)]
    s = torch.cuda.Stream(device=dev)

    def run_all():
        for (a, b, d) in nodes:
            G.computeMatMul(g, None, a, b, d, stream=s)

    per, _ = bench._graph_time(torch, run_all, s, 20)
    per /= copies
    out["%dx%d" % (M, K)] = round(per * 1e6, 3)
    del g
print(json.dumps({"type": QN, "LK_KQ_STREAM": os.environ.get("LK_KQ_STREAM", "1"), "us": out}))
