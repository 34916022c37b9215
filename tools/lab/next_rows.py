"""Prints bench.next_rows() alone (lab: A/B of the §8f rows without the full bench)."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import bench  # noqa: E402
import torch  # noqa: E402
import ggml_hip as G  # noqa: E402

G.load_library()
print(json.dumps(bench.next_rows(torch, G, torch.device("cuda", 0))), flush=True)
