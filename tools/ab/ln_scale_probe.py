"""Fixed cost vs per-byte cost of the LayerNorm kernels on the packed step's shapes: the GPT-2 backward form (dx =
LN'(dy) + dres, frozen: no dgamma / dbeta), the mapper form (with dgamma / dbeta partials + their reduce), and the
forward, each at 0.5x / 1x / 2x / 4x the step's rows, beside a plain bf16 device copy of the same bytes. Each case is
a HIP graph of REPS back-to-back launches (like the step's replay), timed with HIP events.

    python tools/ab/ln_scale_probe.py            [ROWS=3200,3584] [CASES=mapper,copy]
"""

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpt2-image-captioning_amd")]

import torch  # noqa: E402

from icap import ops  # noqa: E402


def timed(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    dev = torch.device("cuda", 0)
    reps = int(os.environ.get("REPS", "100"))
    D = 768
    print(f"{'case':40s} {'rows':>6s} {'us':>8s} {'MB':>7s} {'TB/s':>6s}")
    only = os.environ.get("CASES")  # comma-separated substrings of the case names (default: all)
    for rows in [int(r) for r in os.environ.get("ROWS", "1792,3584,7168,14336").split(",")]:
        x, dy, dres = (torch.randn((rows, D), device=dev).to(torch.bfloat16) for _ in range(3))
        dx = torch.empty_like(x)
        gam, bet = torch.rand(D, device=dev) + 0.5, torch.randn(D, device=dev)
        mean, rstd = torch.randn(rows, device=dev), torch.rand(rows, device=dev) + 0.5
        dgam, dbet = torch.zeros(D, device=dev), torch.zeros(D, device=dev)
        ws = torch.empty(ops.layernorm_bwd_workspace(rows, D) // 4 + 1, device=dev)
        mb = rows * D * 2 / 1e6
        cases = [
            ("ln bwd dx + dres (GPT-2)", lambda: ops.layernorm_bwd(x, gam, mean, rstd, dy, dx, dres=dres), 4 * mb),
            ("ln bwd dx (no dres)", lambda: ops.layernorm_bwd(x, gam, mean, rstd, dy, dx), 3 * mb),
            ("ln bwd + dgamma/dbeta (mapper)", lambda: ops.layernorm_bwd(x, gam, mean, rstd, dy, dx, dres=dres,
                                                                         dgamma=dgam, dbeta=dbet, workspace=ws),
             4 * mb),
            ("ln fwd + mean/rstd", lambda: ops.layernorm_fwd(x, gam, bet, 1e-5, dx, mean, rstd), 2 * mb),
            ("torch copy bf16", lambda: dx.copy_(x), 2 * mb),
        ]
        for name, fn, nb in cases:
            if only and not any(o in name for o in only.split(",")):
                continue
            us = timed(fn, reps)
            print(f"{name:40s} {rows:6d} {us:8.2f} {nb:7.2f} {nb / us:6.2f}", flush=True)


if __name__ == "__main__":
    main()
