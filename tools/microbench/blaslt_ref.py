"""hipBLASLt (torch.mm) reference times for the gemm_lab shapes: C[M,N] = A[M,K] . B[N,K]^T, bf16, uniform
random operands in [-1, 1), 20 launches per HIP graph, best of 7 replays (the lab's timing form)."""
import sys

import torch

dev = torch.device("cuda", 0)
shapes = [(3584, 2304, k) for k in (768, 1536, 3072, 6144)] + [(3584, 768, k) for k in (768, 2304, 3072)]
shapes += [(3584, 3072, 768), (6400, 2304, 768), (6400, 768, 3072)]
if len(sys.argv) > 1:
    shapes = [tuple(int(x) for x in s.split("x")) for s in sys.argv[1:]]
for M, N, K in shapes:
    A = torch.rand((M, K), device=dev).mul_(2).sub_(1).to(torch.bfloat16)
    B = torch.rand((N, K), device=dev).mul_(2).sub_(1).to(torch.bfloat16)
    C = torch.empty((M, N), device=dev, dtype=torch.bfloat16)
    for _ in range(3):
        torch.mm(A, B.t(), out=C)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(20):
            torch.mm(A, B.t(), out=C)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(7):
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / 20)
    print(f"hipblaslt {M}x{N}x{K}: {best:7.2f} us ({2.0 * M * N * K / best / 1e6:4.0f} TF/s)", flush=True)
