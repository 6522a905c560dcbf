"""Reference ceiling: torch.matmul (hipBLASLt/rocBLAS) on the training-step GEMM shapes, bf16, plain epilogue."""

import torch

SHAPES = [(4096, 4096, 4096), (8320, 3072, 768), (8320, 768, 3072), (8320, 2304, 768), (8320, 768, 2304),
          (8320, 768, 768), (8320, 50304, 768), (8320, 768, 50304), (6400, 3072, 768), (3200, 3072, 768),
          (3200, 768, 3072), (768, 3072, 3200), (768, 768, 3200), (128, 2304, 768), (128, 768, 3072)]


def main():
    dev = torch.device("cuda", 0)
    for M, N, K in SHAPES:
        A = (torch.rand((M, K), device=dev) * 2 - 1).to(torch.bfloat16)
        B = (torch.rand((N, K), device=dev) * 2 - 1).to(torch.bfloat16)
        for _ in range(3):
            C = A @ B.t()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            C = A @ B.t()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / 20
        print(f"{M:6d}x{N:6d}x{K:6d} torch.matmul {us:9.1f} us {2 * M * N * K / us / 1e6:8.1f} TF/s", flush=True)
    del C


if __name__ == "__main__":
    main()
