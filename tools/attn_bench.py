"""Attention microbench at the train step's shapes (GPT-2: B=128, S=65, 12 heads x 64, causal + key mask,
dropout 0.1; mapper: B=128, S=25, 8 heads x 96, dropout 0.1), bf16, HIP-event timing.

Usage: [ICAP_LIB=path/to/other/libicap_hip.so] python tools/attn_bench.py
"""

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpt2-image-captioning_amd")]

import torch  # noqa: E402

from icap import _lib as L  # noqa: E402
from icap import ops  # noqa: E402


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    if os.environ.get("ICAP_LIB"):
        L.load(os.environ["ICAP_LIB"], strict=False)
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(0)
    for (B, S, H, hd, causal) in [(128, 65, 12, 64, True), (128, 25, 8, 96, False)]:
        D = H * hd
        qkv = (torch.randn((B * S, 3 * D), generator=g) * 0.5).to(dev, torch.bfloat16)
        out = torch.empty((B * S, D), device=dev, dtype=torch.bfloat16)
        dout = (torch.randn((B * S, D), generator=g) * 0.5).to(dev, torch.bfloat16)
        dqkv = torch.empty_like(qkv)
        lse = torch.empty((B * H * S,), device=dev)
        km = torch.ones((B, S), dtype=torch.int32, device=dev)
        km[:, 30:] = 0
        drop = ops.Dropout(0.1, seed=3)
        kw = dict(B=B, S=S, H=H, hd=hd, scale=hd ** -0.5, causal=causal, key_mask=km if causal else None, drop=drop)
        f = timeit(lambda: ops.attention_fwd(qkv, out, lse=lse, **kw))
        b = timeit(lambda: ops.attention_bwd(qkv, dout, lse, dqkv, out=out, **kw))
        print(f"attn B={B} S={S} H={H} hd={hd}: fwd {f:7.1f} us  bwd {b:7.1f} us", flush=True)


if __name__ == "__main__":
    main()
