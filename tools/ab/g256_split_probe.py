"""Would a split-K 256x256 kernel beat the fused 128x128 one on the packed N = 768 / long-K products? Emulation:
the 256 kernel over M*S rows and K/S (the same blocks, per-block K range and concurrency as an S-way split of
M x N x K, minus the combine) against the shipped plan of M x N x K. HIP-event timing, random bf16."""

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpt2-image-captioning_amd")]

import torch  # noqa: E402

from icap import ops  # noqa: E402


def t(M, N, K, reps=20, **kw):
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(0)
    A = (torch.rand((M, K), generator=g) * 2 - 1).to(dev, torch.bfloat16)
    B = (torch.rand((N, K), generator=g) * 2 - 1).to(dev, torch.bfloat16)
    C = torch.empty((M, N), device=dev, dtype=torch.bfloat16)
    for _ in range(3):
        ops.gemm(A, B, C, **kw)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        ops.gemm(A, B, C, **kw)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    for M, N, K in [(3584, 768, 3072), (3584, 768, 2304), (3584, 2304, 768), (3584, 3072, 768), (6400, 768, 3072),
                    (3200, 768, 3072), (6400, 3072, 768), (6400, 2304, 768)]:
        base = t(M, N, K)
        fl = 2.0 * M * N * K
        line = f"{M}x{N}x{K}: shipped {base:6.1f} us ({fl / base / 1e6:4.0f} TF/s)"
        line += f" | g256 whole {t(M, N, K, g256=True, split_k=1):6.1f}"
        for S in (2, 3, 4):
            if K % (64 * S) == 0:
                us = t(M * S, N, K // S, g256=True, split_k=1)
                line += f" | g256 S={S} {us:6.1f} ({fl / us / 1e6:4.0f})"
        print(line, flush=True)


if __name__ == "__main__":
    main()
