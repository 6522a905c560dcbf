"""Cost of the activation epilogue on the wide K = 768 products (CLIP c_fc 6400x3072x768 quick_gelu, GPT-2 c_fc
8320-row buffer / 3584 live rows gelu_new + aux): the same product without activation, with it, and with it plus
the aux (pre-activation) store. HIP-event timing, random bf16."""

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpt2-image-captioning_amd")]

import torch  # noqa: E402

from icap import _lib as L  # noqa: E402
from icap import ops  # noqa: E402


def t(fn, reps=20):
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
    g = torch.Generator().manual_seed(0)
    for M, live, N, K in [(6400, None, 3072, 768), (8320, 3584, 3072, 768), (3200, None, 3072, 768)]:
        A = (torch.rand((M, K), generator=g) * 2 - 1).to(dev, torch.bfloat16)
        B = (torch.rand((N, K), generator=g) * 2 - 1).to(dev, torch.bfloat16)
        C = torch.empty((M, N), device=dev, dtype=torch.bfloat16)
        aux = torch.empty_like(C)
        bias = torch.zeros(N, device=dev)
        kw = {}
        if live:
            kw = dict(m_dev=torch.tensor([live], dtype=torch.int32, device=dev), m_hint=live)
        line = f"{M}x{N}x{K}{' live ' + str(live) if live else ''}:"
        for tag, extra in [("plain", {}), ("bias", dict(bias=bias)), ("qgelu", dict(bias=bias, act=L.ACT_QUICK_GELU)),
                           ("gelu", dict(bias=bias, act=L.ACT_GELU_NEW)),
                           ("gelu+aux", dict(bias=bias, act=L.ACT_GELU_NEW, aux=aux)),
                           ("relu", dict(bias=bias, act=L.ACT_RELU))]:
            us = t(lambda: ops.gemm(A, B, C, **kw, **extra))
            name = L.load().icap_gemm_kernel_name
            line += f" {tag} {us:6.1f}"
        print(line, flush=True)


if __name__ == "__main__":
    main()
