"""Where the GPT-2 LayerNorm backward and the packed attention passes spend their time (packed B = 128 train step
shapes): LN backward over 3584 live rows of an 8320-row capacity vs an exact 3584-row launch, with and without the
dropout-gradient output; packed attention forward / backward with all sequences <= 32 tokens (the short pass does
the work, the long pass only exits) vs the same launch unpacked at S = 32. Median us over 20 launches."""
import os
import statistics
import sys

sys.path[:0] = ["/root/repo", "/root/repo/gpt2-image-captioning_amd"]
import torch  # noqa: E402

from icap import ops  # noqa: E402


def bench(fn, n=20):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(n):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    return statistics.median(ts)


dev = torch.device("cuda", 0)
D, cap, live = 768, 8320, 3584
x = torch.randn((cap, D), device=dev).to(torch.bfloat16)
dy = torch.randn((cap, D), device=dev).to(torch.bfloat16)
dres = torch.randn((cap, D), device=dev).to(torch.bfloat16)
dx = torch.empty_like(x)
dxd = torch.empty_like(x)
g = torch.rand(D, device=dev) + 0.5
mean = torch.randn(cap, device=dev) * 0.1
rstd = torch.rand(cap, device=dev) + 0.5
rd = torch.tensor([live], dtype=torch.int32, device=dev)
drop = ops.Dropout(0.1, 7)
res = {}
res["ln_bwd cap8320 live3584 +dx_drop"] = bench(lambda: ops.layernorm_bwd(x, g, mean, rstd, dy, dx, dres=dres, dx_drop=dxd,
                                                                        drop=drop, rows_dev=rd))
res["ln_bwd cap8320 live3584"] = bench(lambda: ops.layernorm_bwd(x, g, mean, rstd, dy, dx, dres=dres, rows_dev=rd))
res["ln_bwd exact3584 +dx_drop"] = bench(lambda: ops.layernorm_bwd(x[:live], g, mean, rstd, dy[:live], dx[:live],
                                                                  dres=dres[:live], dx_drop=dxd[:live], drop=drop))
res["ln_bwd exact3584"] = bench(lambda: ops.layernorm_bwd(x[:live], g, mean, rstd, dy[:live], dx[:live],
                                                         dres=dres[:live]))
for k, v in res.items():
    print(f"{k:40s} {v:7.2f} us", flush=True)

# packed attention: 128 sequences of 28 tokens in a launch of S = 65 (two passes) vs the same rows unpacked at S = 28
B, S, H, hd, s_live = 128, 65, 12, 64, 28
qkv = (torch.randn((B * S, 3 * H * hd), device=dev) * 0.5).to(torch.bfloat16)
o = torch.empty((B * S, H * hd), device=dev, dtype=torch.bfloat16)
do = torch.randn((B * S, H * hd), device=dev).to(torch.bfloat16)
dqkv = torch.empty_like(qkv)
lse = torch.empty((B, H, S), device=dev)
so = torch.arange(B, dtype=torch.int32, device=dev) * s_live
sl = torch.full((B,), s_live, dtype=torch.int32, device=dev)
sc = 1.0 / hd ** 0.5
r2 = {}
r2["attn fwd packed S65 (28 live)"] = bench(lambda: ops.attention_fwd(qkv, o, B=B, S=S, H=H, hd=hd, scale=sc, causal=True,
                                                                       lse=lse, seqs=(so, sl)))
r2["attn bwd packed S65 (28 live)"] = bench(lambda: ops.attention_bwd(qkv, do, lse, dqkv, B=B, S=S, H=H, hd=hd, scale=sc,
                                                                       causal=True, out=o, seqs=(so, sl)))
lse2 = torch.empty((B, H, s_live), device=dev)
r2["attn fwd unpacked S28"] = bench(lambda: ops.attention_fwd(qkv, o, B=B, S=s_live, H=H, hd=hd, scale=sc, causal=True,
                                                               lse=lse2))
r2["attn bwd unpacked S28"] = bench(lambda: ops.attention_bwd(qkv, do, lse2, dqkv, B=B, S=s_live, H=H, hd=hd, scale=sc,
                                                               causal=True, out=o))
for k, v in r2.items():
    print(f"{k:40s} {v:7.2f} us", flush=True)
