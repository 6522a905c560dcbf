"""Greedy decode (GPT-2 small, bf16, 50 tokens, all steps) with the batch split into 1 / 2 / 4 sub-batch streams
(GPT2Core.decode_streams): captions/s and id equality with the one-chain decode, at B = 128 and 512."""

import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpt2-image-captioning_amd")]

import torch  # noqa: E402

from bench import build  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    model, _, _ = build(8, dev)
    core = model.gpt.core(model.compute_dtype)
    for B in (128, 512):
        g = torch.Generator().manual_seed(5)
        emb = torch.randn((B, 512), generator=g)
        emb = (emb / emb.norm(dim=-1, keepdim=True)).to(dev)
        ref = None
        for parts in (1, 2, 4):
            core.decode_streams = parts
            out = model.generate(emb, max_length=50, temperature=0.0, early_exit=False)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            n = 3
            for _ in range(n):
                out = model.generate(emb, max_length=50, temperature=0.0, early_exit=False)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / n
            same = ref is None or torch.equal(out, ref)
            ref = out if ref is None else ref
            print(f"B={B:4d} streams={parts}  {B / dt:8.1f} captions/s  {dt * 1e3:7.2f} ms/batch  ids_equal={same}",
                  flush=True)


if __name__ == "__main__":
    main()
