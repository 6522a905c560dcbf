"""Round 6: the packed B = 128 train step with the mapper's LayerNorm parameter reduces per call (two launches per
layer) vs batched (one ln_param_reduce_batch launch per layer), alternating in one process on the benchmark model
(graph replay, 20 steps per measurement, images/s)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpt2-image-captioning_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from icap import CaptionTrainer  # noqa: E402
from icap import mapper as mapper_mod  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    B = 128
    model, tower, _ = bench.build(B, dev)
    ids, mask, labels, px = bench.synthetic_batch(B, 1, dev)
    trainers = {}
    for mode in (False, True):
        mapper_mod.LN_PARAM_BATCH = mode
        t = CaptionTrainer(model, B, 50, lr=1e-4, num_training_steps=10 ** 6, clip_model=tower, dropout=True,
                           seed=1234, mapper_dw="fused")
        t.load_batch(ids, mask, labels, pixels=px)
        for _ in range(3):
            t.micro_step(use_graph=True)
        trainers[mode] = t
    torch.cuda.synchronize()
    for rep in range(3):
        for mode, t in trainers.items():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(20):
                t.micro_step(use_graph=True)
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            print(f"rep {rep} batch={mode!s:5s} {B * 20 / el:9.1f} images/s  {el / 20 * 1e3:6.3f} ms/step", flush=True)


if __name__ == "__main__":
    main()
