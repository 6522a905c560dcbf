"""Fixed vs per-k-step cost of each GEMM kernel form (diagnostic): 3584 x 2304 x K for K = 768 .. 6144 in graph
replay (20 launches per graph, best of 5), per form: the automatic plan, the 128 x 128 double-buffered tile (v0,
needs the diagnostic build for ICAP_FORCE_TILE), the 256-row 8-phase kernel at 128 / 256 columns, hipBLASLt. The
slope over K is the main loop's cost per 64-deep k-step; the intercept the prologue + epilogue + launch."""
import os
import sys

sys.path[:0] = ["/root/repo", "/root/repo/gpt2-image-captioning_amd"]
import torch  # noqa: E402

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
for M, N in ((3584, 2304), (6400, 2304), (3584, 768)):
    print(f"M {M} N {N}: us per launch (TF/s)", flush=True)
    for K in (768, 1536, 3072, 6144):
        A = (torch.randn((M, K), generator=g) * 0.1).to(dev, torch.bfloat16)
        B = (torch.randn((N, K), generator=g) * 0.1).to(dev, torch.bfloat16)
        C = torch.empty((M, N), device=dev, dtype=torch.bfloat16)
        row = []
        for name in ("auto", "v0", "r256", "g8p128", "hipblaslt"):
            os.environ.pop("ICAP_FORCE_TILE", None)
            if name == "v0":
                os.environ["ICAP_FORCE_TILE"] = "0"
            if name == "hipblaslt":
                fn = lambda: torch.mm(A, B.t(), out=C)  # noqa: E731
            else:
                g8 = {"g8p128": 128, "g8p256": 256}.get(name, 0)
                fn = lambda g8=g8, name=name: ops.gemm(A, B, C, split_k=0 if name == "auto" else 1, g8p=g8,  # noqa: E731
                                                       r256=name == "r256")
            us = per_launch(fn)
            row.append(f"{name} {us:6.1f} ({2.0 * M * N * K / us / 1e6:4.0f})")
        os.environ.pop("ICAP_FORCE_TILE", None)
        print(f"  K {K:5d}: " + "  ".join(row), flush=True)
