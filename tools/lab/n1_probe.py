"""Lab: the batch-1 single-launch lines alone (bench.headline + bench.n1_configs), for A/B builds."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "llama.kotlin_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
import ggml_hip as G  # noqa: E402

G.load_library()
dev = torch.device("cuda", 0)
h = bench.headline(torch, G, dev)
n = bench.n1_configs(torch, G, dev)
print({"4096sq": h["avg_launch_us"], "grouped48": h["grouped_48_in_one_launch"]["avg_launch_us"],
       **{k: v["avg_launch_us"] for k, v in n.items()}}, flush=True)
