"""Round 6: the split-role ring kernels (variant 26 = 128 x 256 tiles, ops.gemm(roles=256); variant 27 = 96 x 128,
roles=96; variant 28 = 192 x 256 with 8 MFMA waves, roles=192; variant 32 = 160 x 128, roles=160) against the automatic plan and hipBLASLt (torch.mm, plain products only) on the train step's products,
with the epilogue each one has in the step. Each form is captured as 20 back-to-back launches in a HIP graph and
replayed 7 times (best per-launch us). '!' = not allclose to auto. Usage: python tools/ab/roles_ab.py [skew]
(skew: also the roles forms with K-skew 1, ICAP_ROLES_SKEW, read only by the diagnostic build)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpt2-image-captioning_amd"), os.path.dirname(os.path.abspath(__file__))]
import torch  # noqa: E402

from icap import _lib as L  # noqa: E402
from icap import ops  # noqa: E402
from gemm_helpers_ab import names_of  # noqa: E402

dev = torch.device("cuda", 0)
REPS = 20
SHAPES = [  # (M capacity, live rows or None, N, K, epilogue, what)
    (8320, 3584, 2304, 768, "lnf", "gpt2 c_attn fwd (LN fold)"),
    (8320, 3584, 768, 768, "resid_drop_lns", "gpt2 attn c_proj fwd (LN stats)"),
    (8320, 3584, 3072, 768, "lnf_gelu", "gpt2 c_fc fwd (LN fold, gelu, aux)"),
    (8320, 3584, 768, 3072, "resid_drop_lns", "gpt2 mlp c_proj fwd (LN stats)"),
    (8320, 3584, 3072, 768, "dgelu", "gpt2 mlp c_proj dX (dgelu)"),
    (8320, 3584, 768, 3072, "plain", "gpt2 c_fc dX"),
    (8320, 3584, 768, 768, "plain", "gpt2 attn c_proj dX"),
    (8320, 3584, 768, 2304, "plain", "gpt2 c_attn dX"),
    (8320, 3584, 2304, 768, "plain", "plain 3584x2304x768"),
    (8320, 3584, 3072, 768, "plain", "plain 3584x3072x768"),
    (3200, None, 2304, 768, "plain", "mapper qkv"),
    (3200, None, 768, 768, "resid_drop", "mapper out_proj fwd"),
    (3200, None, 3072, 768, "relu", "mapper linear1 fwd (relu)"),
    (3200, None, 768, 3072, "resid_drop", "mapper linear2 fwd"),
    (6400, None, 2304, 768, "lnf", "clip qkv (LN fold)"),
    (6400, None, 768, 768, "resid_lns", "clip out_proj (LN stats)"),
    (6400, None, 3072, 768, "lnf_qgelu", "clip fc1 (LN fold, quick_gelu)"),
    (6400, None, 768, 3072, "resid_lns", "clip fc2 (LN stats)"),
]


def per_launch(body):
    body()
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with ops.graph_capture(gr):
        for _ in range(REPS):
            body()
    gr.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(7):
        e0.record()
        gr.replay()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / REPS)
    del gr
    return best


def operands(M, N, K, epi, g):
    A = (torch.rand((M, K), generator=g) * 2 - 1).to(dev, torch.bfloat16)
    B = (torch.rand((N, K), generator=g) * 2 - 1).mul_(0.05).to(dev, torch.bfloat16)
    kw = {}
    if epi.startswith("resid"):
        kw = dict(bias=torch.zeros(N, device=dev), resid=torch.randn((M, N), device=dev).to(torch.bfloat16))
        if "drop" in epi:
            kw["drop"] = ops.Dropout(0.1, 1)
        if epi.endswith("lns"):
            kw["ln_stats_out"] = torch.empty((M, N // 32, 2), device=dev)
    elif epi.startswith("lnf"):
        st = torch.stack((torch.zeros(M, K // 32), torch.full((M, K // 32), 32.0)), -1).to(dev).contiguous()
        kw = dict(bias=torch.zeros(N, device=dev), ln_fold=(torch.zeros(N, device=dev), 1e-5), ln_stats_in=st)
        if epi.endswith("_gelu"):
            kw.update(act=L.ACT_GELU_NEW, aux=torch.empty((M, N), device=dev, dtype=torch.bfloat16))
        elif epi.endswith("qgelu"):
            kw.update(act=L.ACT_QUICK_GELU)
    elif epi == "dgelu":
        kw = dict(dact=L.ACT_GELU_NEW, dact_src=torch.randn((M, N), device=dev).to(torch.bfloat16),
                  drop=ops.Dropout(0.1, 1))
    elif epi == "relu":
        kw = dict(bias=torch.zeros(N, device=dev), act=L.ACT_RELU, aux=torch.empty((M, N), device=dev,
                                                                                  dtype=torch.bfloat16))
    return A, B, kw


def main():
    skew = len(sys.argv) > 1 and sys.argv[1] == "skew"
    g = torch.Generator(device="cpu").manual_seed(0)
    forms = [("auto", {}, {}), ("r256", {}, dict(roles=256)), ("r96", {}, dict(roles=96)),
             ("r192", {}, dict(roles=192)), ("r160", {}, dict(roles=160)), ("g8p256", {}, dict(g8p=256))]
    if skew:
        forms += [("r256s", {"ICAP_ROLES_SKEW": "1"}, dict(roles=256)), ("r96s", {"ICAP_ROLES_SKEW": "1"},
                                                                         dict(roles=96))]
    print(f"{'shape':52s} " + " ".join(f"{f[0]:>8s}" for f in forms) + f" {'hipBLASLt':>10s}   (us per launch)")
    for M, live, N, K, epi, what in SHAPES:
        rows = live or M
        A, B, kw = operands(M, N, K, epi, g)
        C = torch.zeros((M, N), device=dev, dtype=torch.bfloat16)
        if live is not None:
            kw.update(m_dev=torch.tensor([live], dtype=torch.int32, device=dev), m_hint=live)
        cells, ref, names = [], None, []
        for name, env, extra in forms:
            os.environ.update(env)
            try:
                fn = lambda: ops.gemm(A, B, C, **kw, **extra)  # noqa: E731
                t = per_launch(fn)
                names.append(names_of(fn).replace("gemm_kernel<bf16, bf16, ", "<"))
            finally:
                for k in env:
                    os.environ.pop(k, None)
            got = C[:rows].float().clone()
            ref = got if ref is None else ref
            ok = torch.allclose(got, ref, rtol=2e-2, atol=2e-2)
            cells.append(f"{t:7.1f}{' ' if ok else '!'}")
        lib = ""
        if epi == "plain":
            a = A[:rows]
            lib = f"{per_launch(lambda: torch.mm(a, B.t(), out=C[:rows])):10.1f}"
        print(f"{what + f' {rows}x{N}x{K}':52s} " + " ".join(cells) + f" {lib:>10s}   " + " | ".join(names),
              flush=True)


if __name__ == "__main__":
    main()
