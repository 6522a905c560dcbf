"""What the operand traffic costs the train step's GEMM forms: each shape timed with the A / B / both operands'
staging loads dropped (ICAP_GEMM_DIAG zero-record descriptors; outputs wrong, timing only) against the real launch,
interleaved in one process (cdna_hip_programming.md §5.4 rule 24). Random bf16 operands.

    python tools/gemm_diag.py        -> one line per (shape, diag): median / min us over REPS rounds
"""

import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpt2-image-captioning_amd")]

import torch  # noqa: E402

from icap import _lib as L  # noqa: E402
from icap import ops  # noqa: E402

# (M capacity, live rows (m_dev) or None, N, K, epilogue) — the packed B = 128 step's products
SHAPES = [
    (8320, 3584, 768, 3072, "resid_drop"),   # GPT-2 mlp.c_proj fwd
    (8320, 3584, 768, 3072, "plain"),        # c_fc dX
    (8320, 3584, 768, 2304, "plain"),        # c_attn dX
    (8320, 3584, 3072, 768, "gelu_aux"),     # c_fc fwd
    (8320, 3584, 3072, 768, "dgelu"),        # mlp.c_proj dX
    (8320, 3584, 2304, 768, "plain"),        # c_attn fwd
    (8320, 3584, 768, 768, "resid_drop"),    # attn c_proj fwd
    (8320, 3584, 768, 768, "plain"),         # attn c_proj dX
    (6400, None, 768, 3072, "resid"),        # CLIP fc2
    (6400, None, 3072, 768, "qgelu"),        # CLIP fc1
    (3200, None, 3072, 768, "relu_drop"),    # mapper linear1
    (3200, None, 768, 3072, "resid_drop"),   # mapper linear2
    (8320, None, 768, 3072, "plain"),        # padded grid form
]


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(0)
    reps = int(os.environ.get("REPS", "15"))
    diags = [0, 1, 2, 3]
    print(f"{'shape':44s} " + " ".join(f"{'diag' + str(d):>16s}" for d in diags) + "   (median / min us)")
    for M, live, N, K, epi in SHAPES:
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
        times = {d: [] for d in diags}
        for r in range(reps + 2):
            for d in diags:
                os.environ["ICAP_GEMM_DIAG"] = str(d)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                ops.gemm(A, B, C, **kw)
                e1.record()
                torch.cuda.synchronize()
                if r >= 2:
                    times[d].append(e0.elapsed_time(e1) * 1e3)
        os.environ["ICAP_GEMM_DIAG"] = "0"
        rows = live or M
        tf = 2.0 * rows * N * K / (statistics.median(times[0]) * 1e-6) / 1e12
        desc = f"{rows}({M})x{N}x{K} {epi}"
        print(f"{desc:44s} " + " ".join(f"{statistics.median(times[d]):8.1f}/{min(times[d]):7.1f}" for d in diags)
              + f"   real {tf:6.0f} TF/s", flush=True)


if __name__ == "__main__":
    main()
