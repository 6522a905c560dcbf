"""GEMM microbenchmark over the shapes/epilogues of one training step (random bf16 operands; HIP-event timing).

Usage: [ICAP_LIB=path/to/other/libicap_hip.so] python tools/gemm_bench.py
       (per shape: the automatic plan and the tile-kernel-only path, interleaved in one process)
"""

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpt2-image-captioning_amd")]

import torch  # noqa: E402

from icap import _lib as L  # noqa: E402
from icap import ops  # noqa: E402

# (M, N, K, epilogue, c dtype)
SHAPES = [
    (4096, 4096, 4096, "plain", torch.bfloat16),
    (8320, 3072, 768, "gelu_aux", torch.bfloat16),
    (8320, 3072, 768, "dgelu", torch.bfloat16),
    (8320, 768, 3072, "resid_drop", torch.bfloat16),
    (8320, 768, 3072, "plain", torch.bfloat16),
    (8320, 2304, 768, "plain", torch.bfloat16),
    (8320, 768, 2304, "plain", torch.bfloat16),
    (8320, 768, 768, "resid_drop", torch.bfloat16),
    (8320, 50304, 768, "plain", torch.bfloat16),
    (8320, 768, 50304, "plain", torch.bfloat16),
    (6400, 3072, 768, "qgelu", torch.bfloat16),
    (3200, 3072, 768, "relu_drop", torch.bfloat16),
    (3200, 768, 3072, "resid_drop", torch.bfloat16),
    (768, 3072, 3200, "beta", torch.float32),
    (768, 768, 3200, "beta", torch.float32),
    (128, 2304, 768, "plain", torch.bfloat16),
    (128, 768, 3072, "resid", torch.bfloat16),
    (8320, 768, 768, "plain", torch.bfloat16),
    (6400, 768, 768, "resid", torch.bfloat16),
    (6400, 2304, 768, "plain", torch.bfloat16),
    (3200, 768, 768, "resid_drop", torch.bfloat16),
    (3200, 2304, 768, "plain", torch.bfloat16),
    (3200, 768, 3072, "plain", torch.bfloat16),
    (3072, 768, 3200, "beta", torch.float32),
]


def main():
    if os.environ.get("ICAP_LIB"):  # A/B against another build of the library
        L.load(os.environ["ICAP_LIB"], strict=False)
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(0)
    reps = int(os.environ.get("REPS", "20"))
    tot_ms = tot_tile = 0.0
    for M, N, K, epi, cdt in SHAPES:
        pad = int(os.environ.get("PAD", "0"))  # row padding (elements) of A and B: L2 channel-stride experiments
        A = (torch.rand((M, K + pad), generator=g) * 2 - 1).to(dev, torch.bfloat16)[:, :K]
        B = (torch.rand((N, K + pad), generator=g) * 2 - 1).to(dev, torch.bfloat16)[:, :K]
        C = torch.zeros((M, N), device=dev, dtype=cdt)
        kw = {}
        if epi == "gelu_aux":
            kw = dict(bias=torch.zeros(N, device=dev), act=L.ACT_GELU_NEW, aux=torch.empty_like(C))
        elif epi == "qgelu":
            kw = dict(bias=torch.zeros(N, device=dev), act=L.ACT_QUICK_GELU)
        elif epi == "relu_drop":
            kw = dict(bias=torch.zeros(N, device=dev), act=L.ACT_RELU, drop=ops.Dropout(0.1, 1))
        elif epi == "dgelu":
            kw = dict(dact=L.ACT_GELU_NEW, dact_src=torch.randn((M, N), device=dev).to(cdt))
        elif epi == "resid_drop":
            kw = dict(bias=torch.zeros(N, device=dev), resid=torch.empty_like(C), drop=ops.Dropout(0.1, 1))
        elif epi == "resid":
            kw = dict(bias=torch.zeros(N, device=dev), resid=torch.empty_like(C))
        elif epi == "beta":
            kw = dict(beta=1.0)
        res = []
        forms = [dict(), dict(tile_only=True)]  # automatic plan vs the 128-row tile kernels
        if M >= 256 and N >= 256 and epi != "beta":
            forms.append(dict(g256=True, split_k=1))  # the 256 x 256 8-phase kernel
        for f in forms:
            for _ in range(3):
                ops.gemm(A, B, C, **f, **kw)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                ops.gemm(A, B, C, **f, **kw)
            e1.record()
            torch.cuda.synchronize()
            res.append(e0.elapsed_time(e1) * 1e3 / reps)
        us = res[0]
        tot_ms += us / 1e3
        tot_tile += res[1] / 1e3
        fl = 2 * M * N * K
        g256 = f" | g256 {res[2]:8.1f} us {fl / res[2] / 1e6:7.1f} TF/s" if len(res) > 2 else ""
        print(f"{M:6d}x{N:6d}x{K:6d} {epi:10s} {str(cdt)[6:]:9s} auto {us:8.1f} us {fl / us / 1e6:7.1f} TF/s | "
              f"tile {res[1]:8.1f} us {fl / res[1] / 1e6:7.1f} TF/s{g256}", flush=True)
    print(f"sum: auto {tot_ms:.3f} ms, tile kernels {tot_tile:.3f} ms")


if __name__ == "__main__":
    main()
