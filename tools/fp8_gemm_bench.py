"""MX fp8 vs bf16 GEMM time on the GPT-2 large (configs[4]) training shapes at B = 128 (M = 8320 tokens), plus the
quantiser. HIP-event timing over REPS launches each; prints TF/s against the bf16 (2.5 PF) and MX-fp8 (5 PF) dense
peaks. Usage: python tools/fp8_gemm_bench.py"""

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpt2-image-captioning_amd")]

import torch  # noqa: E402

from icap import _lib as L  # noqa: E402
from icap import ops  # noqa: E402

M = 8320
SHAPES = [  # (M, N, K, epilogue): GPT-2 large fwd c_attn / c_proj / c_fc / mlp c_proj, then the dX products
    (M, 3840, 1280, "plain"), (M, 1280, 1280, "resid_drop"), (M, 5120, 1280, "gelu_aux"), (M, 1280, 5120, "resid_drop"),
    (M, 1280, 3840, "plain"), (M, 1280, 1280, "plain"), (M, 1280, 5120, "plain"), (M, 5120, 1280, "dgelu"),
    (1792, 50304, 1280, "plain"), (1792, 1280, 50304, "plain"),
]


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3  # us


def main():
    dev = torch.device("cuda", 0)
    reps = int(os.environ.get("REPS", "20"))
    g = torch.Generator(device="cpu").manual_seed(0)
    tb = tf = tq = 0.0
    print(f"{'shape':28s} {'bf16 us':>9s} {'TF/s':>7s} {'fp8 us':>9s} {'TF/s':>7s} {'quant us':>9s} {'speedup':>8s}")
    for Mm, N, K, epi in SHAPES:
        A = (torch.randn((Mm, K), generator=g) * 0.5).to(dev, torch.bfloat16)
        B = (torch.randn((N, K), generator=g) * 0.05).to(dev, torch.bfloat16)
        C = torch.empty((Mm, N), device=dev, dtype=torch.bfloat16)
        kw = {}
        if epi == "gelu_aux":
            kw = dict(bias=torch.zeros(N, device=dev), act=L.ACT_GELU_NEW, aux=torch.empty_like(C))
        elif epi == "dgelu":
            kw = dict(dact=L.ACT_GELU_NEW, dact_src=torch.randn((Mm, N), device=dev).to(torch.bfloat16))
        elif epi == "resid_drop":
            kw = dict(bias=torch.zeros(N, device=dev), resid=torch.randn((Mm, N), device=dev).to(torch.bfloat16),
                      drop=ops.Dropout(0.1, seed=1))
        qA, qB = ops.quantize_mx(A), ops.quantize_mx(B)
        t_b = timed(lambda: ops.gemm(A, B, C, **kw), reps)
        t_f = timed(lambda: ops.gemm(qA, qB, C, **kw), reps)
        t_q = timed(lambda: ops.quantize_mx(A, qA), reps)
        fl = 2.0 * Mm * N * K
        tb, tf, tq = tb + t_b, tf + t_f, tq + t_q
        print(f"{Mm}x{N}x{K} {epi:10s} {t_b:9.1f} {fl / t_b / 1e6:7.0f} {t_f:9.1f} {fl / t_f / 1e6:7.0f} {t_q:9.1f} "
              f"{t_b / (t_f + t_q):8.2f}")
    print(f"sum: bf16 {tb:.0f} us, fp8 {tf:.0f} us + quantise {tq:.0f} us -> {tb / (tf + tq):.2f}x")


if __name__ == "__main__":
    main()
