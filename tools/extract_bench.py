"""End-to-end CLIP extraction images/s in a process of its own (bench.py runs it as a child process, the way a
user runs the reference's extraction notebook: a dedicated process, so DataLoader workers fork a small parent).
Prints one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpt2-image-captioning_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
from icap.clip import CLIPVisionTower  # noqa: E402

if __name__ == "__main__":
    dev = torch.device("cuda", 0)
    tower = CLIPVisionTower.random_init(seed=0).to(dev)
    print(json.dumps(bench.extraction_rate(tower, dev, int(os.environ.get("N", "512")))), flush=True)
