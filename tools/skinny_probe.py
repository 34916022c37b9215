"""Lab: time computeMatMul for batched Q4_0 shapes (graph-replayed, rotating weight copies)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "llama.kotlin_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
import ggml_hip as G  # noqa: E402

G.load_library()
dev = torch.device("cuda", 0)
T = G.GGMLType
BB = {"Q4_0": 18, "Q4_1": 20, "Q8_0": 34}
shapes = [("Q4_0", 11008, 4096, 32), ("Q4_1", 11008, 4096, 32), ("Q4_0", 4096, 11008, 32), ("Q4_0", 11008, 4096, 16),
          ("Q4_0", 11008, 4096, 4)]
for (qn, M, K, N) in shapes:
    qt = getattr(T, qn)
    copies = 16
    nb = M * K // 32 * BB[qn]
    g = G.GGMLGraphAllocator(device=str(dev), defaultBufferSize=16)
    wb = g.addBuffer(copies * nb + 256)
    xb = g.addBuffer(4 * K * N + 256)
    db = g.addBuffer(4 * M * N * copies + 256)
    src = torch.randn(M * K, device=dev) * 0.02
    for c in range(copies):
        g.buffers[wb][c * nb:(c + 1) * nb].copy_(G.quantizeTensor(src * (1 + 0.01 * c), qt))
    g.buffers[xb][: 4 * K * N].copy_(torch.randn(K * N, device=dev).view(torch.uint8))
    nodes = [(G.GGMLTensor(qt, [K, M], bufferId=wb, dataOffset=c * nb), G.GGMLTensor(T.F32, [N, K], bufferId=xb),
              G.GGMLTensor(T.F32, [N, M], bufferId=db, dataOffset=4 * M * N * c)) for c in range(copies)]
    s = torch.cuda.Stream(device=dev)

    def run_all():
        for (a, b, d) in nodes:
            G.computeMatMul(g, None, a, b, d, stream=s)

    with torch.cuda.stream(s):
        run_all()
    torch.cuda.synchronize()
    gr = bench.capture(torch, run_all, s)
    with torch.cuda.stream(s):
        gr.replay()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(10):
            gr.replay()
        e1.record(s)
    torch.cuda.synchronize()
    per = e0.elapsed_time(e1) / 1e3 / (10 * copies)
    print(f"{os.environ.get('TAG', '')} {qn} M={M} K={K} N={N}: {per * 1e6:.2f} us  {(nb + 4 * K * N + 4 * M * N) / per / 1e9:.0f} GB/s",
          flush=True)
    del g
