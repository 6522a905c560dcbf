"""Where a one-round tile-GEMM launch loses time (diagnostic): back-to-back launches captured in a HIP graph, per
launch: the packed c_attn product (3584 x 2304 x 768, 504 tiles = one round at 2 blocks per CU), the same at 2x and
4x the rows, two independent copies on two streams, a plain 16.5 MB fill (the product's output bytes) and a minimal
kernel (launch floor)."""
import sys

sys.path[:0] = ["/root/repo", "/root/repo/gpt2-image-captioning_amd"]
import torch  # noqa: E402

from icap import ops  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator().manual_seed(0)
bf = lambda *s: (torch.randn(s, generator=g) * 0.1).to(dev, torch.bfloat16)  # noqa: E731
N, K = 2304, 768
W = bf(N, K)
A = {m: bf(m, K) for m in (3584, 7168, 14336)}
C = {m: torch.empty((m, N), device=dev, dtype=torch.bfloat16) for m in A}
A2, C2 = bf(3584, K), torch.empty((3584, N), device=dev, dtype=torch.bfloat16)
fill = torch.empty(3584 * N, device=dev, dtype=torch.bfloat16)
tiny = torch.empty(256, device=dev)
side = torch.cuda.Stream(dev)
ops.register_side_stream(side)
REPS = 50


def per_launch(body, reps=REPS, label=""):
    body()
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with ops.graph_capture(gr):
        for _ in range(reps):
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
        best = min(best, e0.elapsed_time(e1) * 1e3 / reps)
    return best


def two_streams():
    main = torch.cuda.current_stream()
    ev = torch.cuda.Event()
    ev.record(main)
    side.wait_event(ev)
    with torch.cuda.stream(side):
        ops.gemm(A2, W, C2)
    ops.gemm(A[3584], W, C[3584])
    ev2 = torch.cuda.Event()
    ev2.record(side)
    main.wait_event(ev2)


res = {}
for m in (3584, 7168, 14336):
    us = per_launch(lambda m=m: ops.gemm(A[m], W, C[m]))
    res[m] = us
    print(f"gemm {m}x{N}x{K}: {us:.1f} us per launch, {2.0 * m * N * K / us / 1e6:.0f} TF/s, "
          f"{us / (m / 3584):.1f} us per 3584 rows", flush=True)
us = per_launch(two_streams)
print(f"two independent 3584-row products on two streams: {us:.1f} us per pair ({us / 2:.1f} per product)", flush=True)
us = per_launch(lambda: (ops.gemm(A[3584], W, C[3584]), ops.gemm(A2, W, C2)))
print(f"the same pair on one stream: {us:.1f} us per pair", flush=True)
us = per_launch(lambda: fill.fill_(1.0))
print(f"fill 16.5 MB (the product's output): {us:.1f} us per launch ({fill.numel() * 2 / us / 1e6:.2f} TB/s)", flush=True)
us = per_launch(lambda: tiny.fill_(1.0))
print(f"minimal kernel (1 KB fill): {us:.2f} us per launch", flush=True)

# the vendor library on the same products (torch.mm -> hipBLASLt), for scale
Wt = W.t()
for m in (3584, 7168, 14336):
    us = per_launch(lambda m=m: torch.mm(A[m], Wt, out=C[m]))
    print(f"torch.mm (hipBLASLt) {m}x{N}x{K}: {us:.1f} us per launch, {2.0 * m * N * K / us / 1e6:.0f} TF/s", flush=True)
for (m, n, k) in ((3584, 3072, 768), (3584, 768, 3072), (3584, 768, 768), (8320, 768, 3072)):
    a, w = bf(m, k), bf(n, k)
    c = torch.empty((m, n), device=dev, dtype=torch.bfloat16)
    ours = per_launch(lambda: ops.gemm(a, w, c))
    lib = per_launch(lambda: torch.mm(a, w.t(), out=c))
    print(f"{m}x{n}x{k}: ours {ours:.1f} us ({2.0 * m * n * k / ours / 1e6:.0f} TF/s), hipBLASLt {lib:.1f} us "
          f"({2.0 * m * n * k / lib / 1e6:.0f} TF/s)", flush=True)
