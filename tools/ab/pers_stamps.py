"""Round 6: where the persistent split-role GEMM (variant 30, gemm_pers.h) spends its time — per-block timestamps of the
diagnostic build (`make -C gpt2-image-captioning_amd/csrc stamps`, ICAP_LIB=.../libicap_hip_stamps.so): start -> the MFMA
waves past B_0 (first stage landed), then each of the first four tiles' C barrier, and the epilogue waves' end.
(Variant 30 was removed from the library after this measurement, profiles/r06_pers_stamps.txt; commit 76ffabb has it.)"""
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
CASES = [  # (M, live, N, K, epi, what)
    (3584, None, 3072, 768, "plain", "plain 3584x3072x768"),
    (8320, 3584, 3072, 768, "lnf_gelu", "c_fc fwd (LN fold, gelu, aux)"),
    (8320, 3584, 3072, 768, "dgelu", "mlp c_proj dX (dgelu)"),
    (6400, None, 768, 3072, "resid_lns", "clip fc2 (LN stats)"),
    (3584, None, 768, 3072, "plain", "c_fc dX (one round)"),
]


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(0)
    st = torch.zeros(8 * 4096, dtype=torch.int64, device=dev)
    med = statistics.median
    print(f"{'shape':36s} {'blocks':>6s} {'tiles':>5s} {'span':>6s} {'B0':>5s} {'tile0':>6s} {'tile1':>6s} {'tile2':>6s} "
          f"{'tile3':>6s} {'epi_end':>7s}  (us from each block's start; medians over blocks with >= 4 tiles)")
    for M, live, N, K, epi, what in CASES:
        A, B, kw = operands(M, N, K, epi, g)
        C = torch.zeros((M, N), device=dev, dtype=torch.bfloat16)
        if live is not None:
            kw.update(m_dev=torch.tensor([live], dtype=torch.int32, device=dev), m_hint=live)
        for _ in range(5):
            ops.gemm(A, B, C, roles=1, **kw)
        st.zero_()
        torch.cuda.synchronize()
        ops.gemm(A, B, C, roles=1, diag_stamps=st, **kw)
        torch.cuda.synchronize()
        rows = [r for r in st.view(-1, 8).cpu().tolist() if r[1] != 0]
        t0 = min(r[1] for r in rows)
        span = (max(r[7] for r in rows) - t0) * TICK_US
        jmax = max(r[0] for r in rows)
        sel = [r for r in rows if r[0] == jmax]
        rel = lambda i: med([(r[i] - r[1]) * TICK_US for r in sel if r[i] != 0]) if any(r[i] for r in sel) else 0.0  # noqa: E731
        print(f"{what + f' {M if live is None else live}x{N}x{K}':36s} {len(rows):6d} {jmax:5d} {span:6.1f} {rel(2):5.2f} "
              f"{rel(3):6.2f} {rel(4):6.2f} {rel(5):6.2f} {rel(6):6.2f} {rel(7):7.2f}", flush=True)


if __name__ == "__main__":
    main()
