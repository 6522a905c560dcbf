"""Mapper weight-gradient products (K-outer GEMM, K = 3200 token rows) under split_k settings, and the
transpose-then-K-contiguous form (two transposes + one C = A.B^T product) for comparison.
usage: python tools/dw_bench.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpt2-image-captioning_amd")]

import torch  # noqa: E402

from icap import ops  # noqa: E402
from icap.mapper import DWHelper  # noqa: E402


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    dev = torch.device("cuda", 0)
    M = int(os.environ.get("ROWS", "3200"))
    h = DWHelper(torch.bfloat16, dev, max_rows=M, max_cols=3072, ln_rows=M, ln_D=768)
    g = torch.Generator().manual_seed(0)
    for N, K in [(2304, 768), (768, 768), (3072, 768), (768, 3072)]:
        dY = torch.randn((M, N), generator=g).to(dev, torch.bfloat16)
        X = torch.randn((M, K), generator=g).to(dev, torch.bfloat16)
        out = torch.zeros((N, K), device=dev)
        fl = 2.0 * M * N * K
        line = f"dW {N}x{K} over {M} rows:"
        for sk in (0, 1, 2, 3, 4, 6, 8, 12):
            h.split_k = sk
            us = timed(lambda: h.dW(dY, X, out, M=M))
            line += f" sk{sk} {us:5.1f}"
        h.split_k = 0
        Mp = (M + 63) // 64 * 64
        def tform():
            a = h._t(h.tA, dY, M, N, Mp)
            b = h._t(h.tB, X, M, K, Mp)
            ops.gemm(a, b, out, beta=1.0, M=N, N=K, K=Mp)
        us = timed(tform)
        a = h._t(h.tA, dY, M, N, Mp)
        b = h._t(h.tB, X, M, K, Mp)
        us2 = timed(lambda: ops.gemm(a, b, out, beta=1.0, M=N, N=K, K=Mp))
        line += f" | transposed: {us:5.1f} (gemm alone {us2:5.1f}, {fl / us2 / 1e6:4.0f} TF/s)"
        print(line, flush=True)


if __name__ == "__main__":
    main()
