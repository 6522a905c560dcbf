"""Where a tile-kernel GEMM launch spends its time: per-workgroup phase stamps from the diagnostic build
(`make -C gpt2-image-captioning_amd/csrc stamps` -> libicap_hip_stamps.so, icap_gemm_args.diag_stamps; s_memrealtime
at 100 MHz). For each of the packed B = 128 train step's GEMM forms: when the workgroups start (dispatch spread),
the prologue (first stage landed), the main loop per k-step, the split-K publish / combine, the epilogue, and the
launch span. Random bf16 operands, the step's epilogues, automatic plan.

    python tools/gemm_stamps.py
"""

import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("ICAP_LIB", os.path.join(ROOT, "gpt2-image-captioning_amd", "icap", "libicap_hip_stamps.so"))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpt2-image-captioning_amd"), os.path.join(ROOT, "tools")]

import torch  # noqa: E402

from gemm_tiles_ab import SHAPES  # noqa: E402
from icap import _lib as L  # noqa: E402
from icap import ops  # noqa: E402

TICK_US = 0.01  # s_memrealtime: 100 MHz


def q(xs, f):
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(f * len(xs)))]


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(0)
    st = torch.zeros(8 * 16384, dtype=torch.int64, device=dev)
    print(f"{'shape':40s} {'blocks':>6s} {'span':>6s} {'start50/90/max':>16s} {'prolog':>6s} {'loop':>6s} "
          f"{'/kstep':>6s} {'publ':>5s} {'comb':>5s} {'epil':>5s}   (us; medians over workgroups)")
    for M, live, N, K, epi, what in SHAPES:
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
        for _ in range(5):
            ops.gemm(A, B, C, **kw)
        st.zero_()
        torch.cuda.synchronize()
        ops.gemm(A, B, C, diag_stamps=st, **kw)
        torch.cuda.synchronize()
        s = st.view(-1, 8).cpu().tolist()
        rows = [r for r in s if r[1] != 0]
        if not rows:
            print(f"{what:40s} (no tile-kernel stamps: another kernel form)")
            continue
        t0 = min(r[1] for r in rows)
        span = (max(max(r[3], r[4], r[5]) for r in rows) - t0) * TICK_US
        starts = [(r[1] - t0) * TICK_US for r in rows]
        prolog = [(r[2] - r[1]) * TICK_US for r in rows if r[2]]
        loop = [(r[3] - (r[2] or r[1])) * TICK_US for r in rows if r[3]]
        publ = [(r[4] - r[3]) * TICK_US for r in rows if r[4] and r[5] == 0]
        comb = [(r[4] - r[3]) * TICK_US for r in rows if r[4] and r[5] != 0]
        epil = [(r[5] - r[4]) * TICK_US for r in rows if r[5] and r[4]]
        nk_all = (K + 63) // 64
        splits = max(((r[0] >> 8) & 0xFF) for r in rows) + 1
        kst = statistics.median(loop) / max(1, -(-nk_all // splits)) if loop else 0.0
        med = lambda xs: statistics.median(xs) if xs else 0.0  # noqa: E731
        desc = f"{what} {live or M}x{N}x{K} S{splits}"
        print(f"{desc:40s} {len(rows):6d} {span:6.1f} {q(starts, .5):5.1f}/{q(starts, .9):4.1f}/{max(starts):4.1f} "
              f"{med(prolog):6.2f} {med(loop):6.2f} {kst:6.3f} {med(publ):5.2f} {med(comb):5.2f} {med(epil):5.2f}",
              flush=True)


if __name__ == "__main__":
    main()
