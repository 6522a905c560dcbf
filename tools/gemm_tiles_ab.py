"""Tile-variant A/B over the packed B = 128 train step's GEMM forms: the automatic plan against each tile kernel
forced (ICAP_FORCE_TILE, unsplit) and the automatic plan with split-K off, interleaved in one process
(cdna_hip_programming.md §5.4 rule 24). Random bf16 operands, the step's epilogues. Median / min us over REPS.

    python tools/gemm_tiles_ab.py
"""

import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpt2-image-captioning_amd")]

import torch  # noqa: E402

from icap import _lib as L  # noqa: E402
from icap import ops  # noqa: E402

SHAPES = [  # (M capacity, live rows or None, N, K, epilogue, what)
    (8320, 3584, 768, 768, "resid_drop", "gpt2 attn c_proj fwd"),
    (8320, 3584, 768, 768, "plain", "gpt2 attn c_proj dX"),
    (6400, None, 768, 768, "resid", "clip out_proj"),
    (3200, None, 768, 768, "resid_drop", "mapper out_proj fwd"),
    (8320, 3584, 2304, 768, "plain", "gpt2 c_attn fwd"),
    (8320, 3584, 3072, 768, "gelu_aux", "gpt2 c_fc fwd"),
    (8320, 3584, 3072, 768, "dgelu", "gpt2 mlp c_proj dX"),
    (6400, None, 2304, 768, "plain", "clip qkv"),
    (6400, None, 3072, 768, "qgelu", "clip fc1"),
    (3200, None, 3072, 768, "relu_drop", "mapper linear1"),
    (8320, 3584, 768, 3072, "resid_drop", "gpt2 mlp c_proj fwd"),
    (8320, 3584, 768, 2304, "plain", "gpt2 c_attn dX"),
    (6400, None, 768, 3072, "resid", "clip fc2"),
]
FORMS = [("auto", None, 0), ("g256", "g256", 0), ("auto_ring", "ring", 0), ("split_k8", "mink", 0), ("nosplit", None, 1), ("v0", "0", 1), ("v4", "4", 1), ("v5", "5", 1), ("v12", "12", 1),
         ("v13", "13", 1), ("v16", "16", 1)]


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(0)
    reps = int(os.environ.get("REPS", "10"))
    print(f"{'shape':52s} " + " ".join(f"{f[0]:>13s}" for f in FORMS) + "   (median us; * = auto's kernel)")
    only = os.environ.get("SHAPES")  # comma-separated substrings of the shape names to run (default: all)
    for M, live, N, K, epi, what in SHAPES:
        if only and not any(o in what for o in only.split(",")):
            continue
        A = (torch.rand((M, K), generator=g) * 2 - 1).to(dev, torch.bfloat16)
        B = (torch.rand((N, K), generator=g) * 2 - 1).to(dev, torch.bfloat16)
        C = torch.zeros((M, N), device=dev, dtype=torch.bfloat16)
        kw = {}
        if epi == "gelu_aux":
            kw = dict(bias=torch.zeros(N, device=dev), act=L.ACT_GELU_NEW, aux=torch.empty_like(C))
        elif epi == "qgelu":
            kw = dict(bias=torch.zeros(N, device=dev), act=L.ACT_QUICK_GELU)
        elif epi == "relu_drop":
            kw = dict(bias=torch.zeros(N, device=dev), act=L.ACT_RELU, drop=ops.Dropout(0.1, 1))
        elif epi == "dgelu":
            kw = dict(dact=L.ACT_GELU_NEW, dact_src=torch.randn((M, N), device=dev).to(torch.bfloat16))
        elif epi == "resid_drop":
            kw = dict(bias=torch.zeros(N, device=dev), resid=torch.randn((M, N), device=dev).to(torch.bfloat16),
                      drop=ops.Dropout(0.1, 1))
        elif epi == "resid":
            kw = dict(bias=torch.zeros(N, device=dev), resid=torch.randn((M, N), device=dev).to(torch.bfloat16))
        if live is not None:
            kw.update(m_dev=torch.tensor([live], dtype=torch.int32, device=dev), m_hint=live)
        times = {f[0]: [] for f in FORMS}
        for r in range(reps + 2):
            for name, fv, sk in FORMS:
                os.environ.pop("ICAP_FUSED_NST", None)
                os.environ.pop("ICAP_FUSED_MINK", None)
                g256 = fv == "g256"  # the 256 x 256 8-phase kernel wherever eligible (ops.gemm g256=True)
                if fv is None or g256:
                    os.environ.pop("ICAP_FORCE_TILE", None)
                elif fv == "ring":  # the automatic plan, its in-launch split-K on the 4-stage ring (ICAP_FUSED_NST=4)
                    os.environ.pop("ICAP_FORCE_TILE", None)
                    os.environ["ICAP_FUSED_NST"] = "4"
                elif fv == "mink":  # in-launch split-K down to 8 K stages (the short-K N = 768 products: S = 2)
                    os.environ.pop("ICAP_FORCE_TILE", None)
                    os.environ["ICAP_FUSED_MINK"] = "8"
                else:
                    os.environ["ICAP_FORCE_TILE"] = fv
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                ops.gemm(A, B, C, split_k=sk, g256=g256, **kw)
                e1.record()
                torch.cuda.synchronize()
                if r >= 2:
                    times[name].append(e0.elapsed_time(e1) * 1e3)
        os.environ.pop("ICAP_FORCE_TILE", None)
        os.environ.pop("ICAP_FUSED_NST", None)
        os.environ.pop("ICAP_FUSED_MINK", None)
        rows = live or M
        desc = f"{what} {rows}x{N}x{K}"
        print(f"{desc:52s} " + " ".join(f"{statistics.median(times[f[0]]):13.1f}" for f in FORMS), flush=True)


def kout_splits():
    """The mapper's K-outer weight-gradient products (fp32 C, beta 1, slab + reduce): forced split counts 1-4 and 6 vs
    the automatic rule."""
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(2)
    reps = int(os.environ.get("REPS", "10"))
    forms = [0, 1, 2, 3, 4, 6]
    print(f"{'K-outer dW (rows 3200), split_k':40s} " + " ".join(f"{('auto' if f == 0 else f):>8}" for f in forms))
    for N_out, K_in in ((768, 3072), (3072, 768), (2304, 768), (768, 768)):
        dY = (torch.rand((3200, N_out), generator=g) * 2 - 1).to(dev, torch.bfloat16)
        X = (torch.rand((3200, K_in), generator=g) * 2 - 1).to(dev, torch.bfloat16)
        C = torch.zeros((N_out, K_in), device=dev)
        t = {f: [] for f in forms}
        for r in range(reps + 2):
            for f in forms:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                ops.gemm(dY, X, C, beta=1.0, M=N_out, N=K_in, K=3200, trans_ab=True, split_k=f)
                e1.record()
                torch.cuda.synchronize()
                if r >= 2:
                    t[f].append(e0.elapsed_time(e1) * 1e3)
        print(f"{N_out}x{K_in}x3200{'':27s} " + " ".join(f"{statistics.median(t[f]):8.1f}" for f in forms), flush=True)


def kout():
    """The mapper's K-outer weight-gradient products (fp32 C, beta 1): slab + reduce pass vs in-launch combine."""
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(1)
    reps = int(os.environ.get("REPS", "10"))
    print(f"{'K-outer dW (rows 3200)':40s} {'slab+reduce':>12s} {'in-launch':>12s}")
    for N_out, K_in in ((768, 3072), (3072, 768), (2304, 768), (768, 768)):
        dY = (torch.rand((3200, N_out), generator=g) * 2 - 1).to(dev, torch.bfloat16)
        X = (torch.rand((3200, K_in), generator=g) * 2 - 1).to(dev, torch.bfloat16)
        C = torch.zeros((N_out, K_in), device=dev)
        t = {0: [], 1: []}
        for r in range(reps + 2):
            for f in (0, 1):
                os.environ["ICAP_KOUT_FUSED"] = str(f)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                ops.gemm(dY, X, C, beta=1.0, M=N_out, N=K_in, K=3200, trans_ab=True)
                e1.record()
                torch.cuda.synchronize()
                if r >= 2:
                    t[f].append(e0.elapsed_time(e1) * 1e3)
        os.environ.pop("ICAP_KOUT_FUSED", None)
        print(f"{N_out}x{K_in}x3200{'':25s} {statistics.median(t[0]):12.1f} {statistics.median(t[1]):12.1f}", flush=True)


if __name__ == "__main__":
    main()
    if not os.environ.get("SHAPES"):
        kout()
    if os.environ.get("KOUT_SPLITS", "1") == "1":
        kout_splits()
