"""The greedy decode's LM-head product (B = 128 rows x 50304 vocabulary x 768) under each tile form (diagnostic;
ICAP_FORCE_TILE needs the diagnostic build, else only 'auto' is meaningful), graph replay, and the greedy_next pass
after it."""
import os
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
for M in (128, 512):
    A = (torch.randn((M, 768), generator=g) * 0.5).to(dev, torch.bfloat16)
    W = (torch.randn((50304, 768), generator=g) * 0.02).to(dev, torch.bfloat16)
    C = torch.empty((M, 50304), device=dev, dtype=torch.bfloat16)
    for form in ("auto", "0", "4", "5", "12", "13", "16"):
        if form == "auto":
            os.environ.pop("ICAP_FORCE_TILE", None)
        else:
            os.environ["ICAP_FORCE_TILE"] = form
        names = _run(lambda: ops.gemm(A, W, C, split_k=0 if form == "auto" else 1))
        us = per_launch(lambda: ops.gemm(A, W, C, split_k=0 if form == "auto" else 1))
        print(f"M {M} form {form:4s}: {us:7.1f} us ({50304 * 768 * 2 / us / 1e6:.2f} TB/s of weights) {names}", flush=True)
    os.environ.pop("ICAP_FORCE_TILE", None)
    fin = torch.zeros(M, dtype=torch.int32, device=dev)
    tok = torch.zeros((M, 64), dtype=torch.int64, device=dev)
    wpe = (torch.randn((1024, 768), generator=g) * 0.02).to(dev, torch.bfloat16)
    x = torch.empty((M, 768), device=dev, dtype=torch.bfloat16)
    us = per_launch(lambda: ops.greedy_next(C, 50257, 50256, fin, tok, 1, W, wpe, 20, 768, x))
    print(f"M {M} greedy_next: {us:.1f} us", flush=True)
