"""What the LayerNorm-statistics producer epilogue costs (diagnostic): the GPT-2 / CLIP residual products with and
without ln_stats_out, graph replay (20 launches, best of 5), automatic plan, kernel names."""
import sys

sys.path[:0] = ["/root/repo", "/root/repo/gpt2-image-captioning_amd", "/root/repo/tests"]
import torch  # noqa: E402

from gemm_helpers import _run  # noqa: E402
from icap import ops  # noqa: E402

dev = torch.device("cuda", 0)
REPS = 20


def per_launch(body):
    body()
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with ops.graph_capture(gr):
        for _ in range(REPS):
            body()
    gr.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(5):
        e0.record()
        gr.replay()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / REPS)
    return best


g = torch.Generator().manual_seed(0)
for (M, live, N, K, what) in ((8320, 3584, 768, 3072, "gpt2 mlp c_proj fwd"), (8320, 3584, 768, 768, "gpt2 attn c_proj fwd"),
                              (6400, None, 768, 3072, "clip fc2"), (6400, None, 768, 768, "clip out_proj")):
    A = (torch.randn((M, K), generator=g) * 0.3).to(dev, torch.bfloat16)
    W = (torch.randn((N, K), generator=g) * 0.05).to(dev, torch.bfloat16)
    C = torch.empty((M, N), device=dev, dtype=torch.bfloat16)
    kw = dict(bias=torch.zeros(N, device=dev), resid=torch.randn((M, N), generator=g).to(dev, torch.bfloat16),
              drop=ops.Dropout(0.1, 1))
    if live:
        kw.update(m_dev=torch.tensor([live], dtype=torch.int32, device=dev), m_hint=live)
    st = torch.empty((M, N // 32, 2), device=dev)
    row = []
    for lab, extra in (("plain", {}), ("ln_stats_out", {"ln_stats_out": st})):
        names = _run(lambda: ops.gemm(A, W, C, **kw, **extra))
        us = per_launch(lambda: ops.gemm(A, W, C, **kw, **extra))
        row.append(f"{lab} {us:6.1f} us {names}")
    print(f"{what} {live or M}x{N}x{K}: " + " | ".join(row), flush=True)
