"""Mapper weight-gradient products (K-outer GEMM, K = 3200 token rows) under split_k settings.
usage: python tools/dw_bench.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpt2-image-captioning_amd")]

import torch  # noqa: E402

from icap.mapper import DWHelper  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    M = 3200
    h = DWHelper(torch.bfloat16, dev, max_rows=M, max_cols=3072, ln_rows=M, ln_D=768)
    g = torch.Generator().manual_seed(0)
    for N, K in [(2304, 768), (768, 768), (3072, 768), (768, 3072)]:
        dY = torch.randn((M, N), generator=g).to(dev, torch.bfloat16)
        X = torch.randn((M, K), generator=g).to(dev, torch.bfloat16)
        out = torch.zeros((N, K), device=dev)
        line = f"dW {N}x{K} over {M} rows:"
        for sk in (0, 1, 2, 4):
            h.split_k = sk
            for _ in range(3):
                h.dW(dY, X, out, M=M)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                h.dW(dY, X, out, M=M)
            e1.record()
            torch.cuda.synchronize()
            line += f"  split_k={sk}: {e0.elapsed_time(e1) * 50:7.1f} us"
        print(line, flush=True)


if __name__ == "__main__":
    main()
