"""Which hipBLASLt kernels torch.mm picks for the step's plain products (run under rocprofv3 --kernel-trace to read
their names: macro tile, wave grid, depth, LDS buffering). Diagnostic; nothing here is on the product path."""
import torch

dev = torch.device("cuda", 0)
SHAPES = [(3584, 2304, 768), (3584, 768, 768), (3584, 768, 2304), (3584, 3072, 768), (3584, 768, 3072),
          (6400, 2304, 768)]
for M, N, K in SHAPES:
    a = torch.randn((M, K), device=dev).to(torch.bfloat16)
    b = torch.randn((N, K), device=dev).to(torch.bfloat16)
    c = torch.empty((M, N), device=dev, dtype=torch.bfloat16)
    for _ in range(10):
        torch.mm(a, b.t(), out=c)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        torch.mm(a, b.t(), out=c)
    e1.record()
    torch.cuda.synchronize()
    print(f"{M}x{N}x{K}: {e0.elapsed_time(e1) * 1e3 / 20:.1f} us per launch (eager)", flush=True)
