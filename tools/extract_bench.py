"""End-to-end CLIP extraction images/s alone (bench.py extraction_rate), for iterating on the loader path."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpt2-image-captioning_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
from icap.clip import CLIPVisionTower  # noqa: E402

if __name__ == "__main__":
    dev = torch.device("cuda", 0)
    tower = CLIPVisionTower.random_init(seed=0).to(dev)
    t0 = time.perf_counter()
    print(bench.extraction_rate(tower, dev, int(os.environ.get("N", "512"))), f"total {time.perf_counter() - t0:.1f}s")
