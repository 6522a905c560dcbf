"""Profile helper: greedy decode only (B=128, 50 steps, random-init GPT-2 small + mapper), for rocprofv3."""

import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpt2-image-captioning_amd")]

import torch  # noqa: E402


def main():
    from types import SimpleNamespace

    from icap import GPT2LMHeadModel, ImageCaptioningModel, TransformerMappingNetwork

    dev = torch.device("cuda", 0)
    B = int(os.environ.get("B", "128"))
    model = ImageCaptioningModel(TransformerMappingNetwork.random_init(), tokenizer=SimpleNamespace(eos_token_id=50256),
                                 gpt=GPT2LMHeadModel.random_init(), compute_dtype=torch.bfloat16).to(dev)
    emb = torch.randn((B, 512), generator=torch.Generator().manual_seed(5)).to(dev)
    emb = emb / emb.norm(dim=-1, keepdim=True)
    for _ in range(2):
        model.generate(emb, max_length=50, temperature=0.0, early_exit=False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = 5
    for _ in range(n):
        out = model.generate(emb, max_length=50, temperature=0.0, early_exit=False)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / n
    print(f"decode B={B}: {dt * 1e3:.2f} ms/batch, {B / dt:.1f} captions/s, returned {tuple(out.shape)}")


if __name__ == "__main__":
    main()
