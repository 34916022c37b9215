"""Run the batched configs (C3 N=32, C5 N=512) a few times for rocprof (lab helper)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "llama.kotlin_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
import ggml_hip as G  # noqa: E402

G.load_library()
dev = torch.device("cuda", 0)
print(bench.batched(torch, G, dev, reps=3))
