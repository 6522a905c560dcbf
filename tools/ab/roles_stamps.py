"""Round 6: where a split-role ring launch spends its time — per-workgroup phase stamps of the diagnostic build
(`make -C gpt2-image-captioning_amd/csrc stamps`, ICAP_LIB=.../libicap_hip_stamps.so; s_memrealtime, 100 MHz):
dispatch spread, prologue (start -> B_0: the first stage landed), main loop (per k-step), epilogue, launch span.
One tile per workgroup in these shapes (grid = live tiles <= CUs)."""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("ICAP_LIB", os.path.join(ROOT, "gpt2-image-captioning_amd", "icap", "libicap_hip_stamps.so"))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpt2-image-captioning_amd"), os.path.dirname(os.path.abspath(__file__))]
import torch  # noqa: E402

from icap import ops  # noqa: E402
from roles_ab import operands  # noqa: E402

TICK_US = 0.01
CASES = [  # (M, live, N, K, epi, roles, what)
    (8320, 3584, 2304, 768, "plain", 256, "c_attn shape, m_dev"),
    (3584, None, 2304, 768, "plain", 256, "c_attn shape, no m_dev"),
    (3584, None, 2304, 3072, "plain", 256, "K 3072"),
    (8320, 3584, 2304, 768, "lnf", 256, "c_attn fwd (LN fold)"),
    (8320, 3584, 768, 768, "resid_drop_lns", 96, "attn c_proj fwd"),
    (8320, 3584, 768, 768, "plain", 96, "attn c_proj dX"),
    (8320, 3584, 768, 2304, "plain", 96, "c_attn dX"),
    (8320, 3584, 768, 3072, "resid_drop_lns", 96, "mlp c_proj fwd"),
    (8320, 3584, 768, 3072, "plain", 96, "c_fc dX"),
    (3584, None, 3072, 768, "plain", 192, "r192 plain 3584x3072"),
    (8320, 3584, 3072, 768, "lnf_gelu", 192, "r192 c_fc fwd (LN fold, gelu, aux)"),
    (8320, 3584, 3072, 768, "dgelu", 192, "r192 mlp c_proj dX (dgelu)"),
    (3584, None, 3072, 3072, "plain", 192, "r192 K 3072"),
]


def q(xs, f):
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(f * len(xs)))]


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(0)
    st = torch.zeros(8 * 16384, dtype=torch.int64, device=dev)
    med = lambda xs: statistics.median(xs) if xs else 0.0  # noqa: E731
    print(f"{'shape':44s} {'blocks':>6s} {'span':>6s} {'start50/90/max':>16s} {'prolog':>6s} {'loop':>6s} "
          f"{'/kstep':>6s} {'epil':>5s} {'end50/max':>10s}  (us; medians over workgroups)")
    for M, live, N, K, epi, roles, what in CASES:
        A, B, kw = operands(M, N, K, epi, g)
        C = torch.zeros((M, N), device=dev, dtype=torch.bfloat16)
        if live is not None:
            kw.update(m_dev=torch.tensor([live], dtype=torch.int32, device=dev), m_hint=live)
        for _ in range(5):
            ops.gemm(A, B, C, roles=roles, **kw)
        st.zero_()
        torch.cuda.synchronize()
        ops.gemm(A, B, C, roles=roles, diag_stamps=st, **kw)
        torch.cuda.synchronize()
        rows = [r for r in st.view(-1, 8).cpu().tolist() if r[1] != 0]
        t0 = min(r[1] for r in rows)
        ends = [(r[5] - t0) * TICK_US for r in rows]
        starts = [(r[1] - t0) * TICK_US for r in rows]
        prolog = [(r[2] - r[1]) * TICK_US for r in rows]
        loop = [(r[3] - r[2]) * TICK_US for r in rows]
        epil = [(r[5] - r[4]) * TICK_US for r in rows]
        nk = (K + 63) // 64
        desc = f"r{roles} {what} {live or M}x{N}x{K}"
        print(f"{desc:44s} {len(rows):6d} {max(ends):6.1f} {q(starts, .5):5.1f}/{q(starts, .9):4.1f}/{max(starts):4.1f} "
              f"{med(prolog):6.2f} {med(loop):6.2f} {med(loop) / nk:6.3f} {med(epil):5.2f} {q(ends, .5):5.1f}/"
              f"{max(ends):4.1f}", flush=True)


if __name__ == "__main__":
    main()
