"""Round 6: the train step's attention launches in isolation (HIP graph of 20 launches, best of 7 replays, us per
launch): GPT-2's packed short-only pass (128 sequences of 28 tokens in a launch of S = 65, causal, key mask, attention
dropout 0.1) forward / backward, CLIP-B/32 (S = 50, 12 heads, no mask, no dropout) forward, and the mapper (S = 20,
8 heads of 96, dropout 0.1) forward / backward."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpt2-image-captioning_amd"), os.path.dirname(os.path.abspath(__file__))]
import torch  # noqa: E402

from icap import ops  # noqa: E402
from roles_ab import per_launch  # noqa: E402

dev = torch.device("cuda", 0)


def main():
    g = torch.Generator().manual_seed(0)
    r = lambda *s: (torch.randn(s, generator=g) * 0.5).to(dev, torch.bfloat16)  # noqa: E731
    out = {}
    # GPT-2 packed short pass
    B, S, H, hd, live = 128, 65, 12, 64, 28
    qkv, o, do = r(B * S, 3 * H * hd), r(B * S, H * hd), r(B * S, H * hd)
    dqkv = torch.empty_like(qkv)
    lse = torch.empty((B, H, S), device=dev)
    so = torch.arange(B, dtype=torch.int32, device=dev) * live
    sl = torch.full((B,), live, dtype=torch.int32, device=dev)
    km = torch.ones(B * S, dtype=torch.int32, device=dev)
    drop = ops.Dropout(0.1, 3)
    kw = dict(B=B, S=S, H=H, hd=hd, scale=hd ** -0.5, causal=True, key_mask=km, seqs=(so, sl), short_only=True)
    out["gpt2 fwd packed short (28 of 65)"] = per_launch(lambda: ops.attention_fwd(qkv, o, lse=lse, drop=drop, **kw))
    out["gpt2 bwd packed short"] = per_launch(lambda: ops.attention_bwd(qkv, do, lse, dqkv, out=o, drop=drop, **kw))
    # CLIP
    B, S, H, hd = 128, 50, 12, 64
    qkv, o = r(B * S, 3 * H * hd), r(B * S, H * hd)
    lse = torch.empty((B, H, S), device=dev)
    out["clip fwd S50"] = per_launch(lambda: ops.attention_fwd(qkv, o, B=B, S=S, H=H, hd=hd, scale=hd ** -0.5,
                                                               causal=False, lse=lse))
    # mapper
    B, S, H, hd = 128, 20, 8, 96
    qkv, o, do = r(B * S, 3 * H * hd), r(B * S, H * hd), r(B * S, H * hd)
    dqkv = torch.empty_like(qkv)
    lse = torch.empty((B, H, S), device=dev)
    kw = dict(B=B, S=S, H=H, hd=hd, scale=hd ** -0.5, causal=False)
    out["mapper fwd S20 hd96"] = per_launch(lambda: ops.attention_fwd(qkv, o, lse=lse, drop=drop, **kw))
    out["mapper bwd S20 hd96"] = per_launch(lambda: ops.attention_bwd(qkv, do, lse, dqkv, out=o, drop=drop, **kw))
    for k, v in out.items():
        print(f"{k:36s} {v:7.2f} us", flush=True)


if __name__ == "__main__":
    main()
