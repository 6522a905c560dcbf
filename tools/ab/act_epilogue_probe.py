import os, sys
ROOT = "/root/repo"
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpt2-image-captioning_amd")]
import torch
from icap import _lib as L, ops
dev = torch.device("cuda", 0)
g = torch.Generator().manual_seed(0)
for M in (6400, 8320):
    A = (torch.rand((M, 768), generator=g) * 2 - 1).to(dev, torch.bfloat16)
    B = (torch.rand((3072, 768), generator=g) * 2 - 1).to(dev, torch.bfloat16)
    C = torch.empty((M, 3072), device=dev, dtype=torch.bfloat16)
    bias = torch.zeros(3072, device=dev)
    for name, kw in (("plain", {}), ("bias", dict(bias=bias)), ("qgelu", dict(bias=bias, act=L.ACT_QUICK_GELU)),
                     ("gelu_new", dict(bias=bias, act=L.ACT_GELU_NEW)), ("relu", dict(bias=bias, act=L.ACT_RELU))):
        for _ in range(3): ops.gemm(A, B, C, **kw)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20): ops.gemm(A, B, C, **kw)
        e1.record(); torch.cuda.synchronize()
        print(f"{M}x3072x768 {name:9s} {e0.elapsed_time(e1) * 1e3 / 20:7.1f} us", flush=True)
