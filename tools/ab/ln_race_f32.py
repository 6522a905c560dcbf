"""LN backward side-stream victim in fp32 (diagnostic; follows ln_race_probe.py).

ln_race_probe showed the wrong rows differ from the quiet result by <= 1 bf16 ulp in most of their elements, whatever
the order of the mean / rstd loads and with one mean for every row: a perturbation of a row statistic, not of an input
element. With fp32 data the difference vector is exact: fit d = a + b * xhat per wrong row (d = -rs (dm1 + xhat dm2)
when only the row sums m1 = mean(gy), m2 = mean(gy xhat) are off), report the residual, and compare ds1 = D dm1 with the
per-lane partial sums of the half-wave reduction (lane l holds chunks l, l + 32, l + 64 of the row).
"""
import os
import sys

sys.path[:0] = ["/root/repo", "/root/repo/gpt2-image-captioning_amd"]
import torch  # noqa: E402

from icap import ops  # noqa: E402

dev = torch.device("cuda", 0)
M, D, F = 800, 768, 3072
N_V = int(os.environ.get("PROBE_N", "40"))
REPS = int(os.environ.get("PROBE_REPS", "5"))
SHOW = int(os.environ.get("PROBE_SHOW", "6"))
g = torch.Generator().manual_seed(0)
x = torch.randn(M, D, generator=g).to(dev)
gamma = (1 + 0.1 * torch.randn(D, generator=g)).to(dev)
mean = (0.1 * torch.randn(M, generator=g)).to(dev)
rstd = (1 + 0.1 * torch.rand(M, generator=g)).to(dev)
dy = (1e-4 * torch.randn(M, D, generator=g)).to(dev)
bfa = (torch.randn(M, D, generator=g) * 1e-4).to(dev, torch.bfloat16)
f = torch.randn(M, F, generator=g).to(dev, torch.bfloat16)
wt = (0.02 * torch.randn(F, D, generator=g)).to(dev, torch.bfloat16)
ct = torch.empty((M, F), device=dev, dtype=torch.bfloat16)
dW = torch.empty((D, F), device=dev, dtype=torch.float32)
side = torch.cuda.Stream(dev)
ops.register_side_stream(side)
aggressors = {
    "none": lambda: None,
    "tile": lambda: ops.gemm(bfa, wt, ct),
    "kout": lambda: ops.gemm(bfa, f, dW, M=D, N=F, K=M, trans_ab=True),
}
victim = lambda o: ops.layernorm_bwd(x, gamma, mean, rstd, dy, o)  # noqa: E731
BF16 = bool(os.environ.get("PROBE_BF16"))
if BF16:
    # bf16 data whose values the fp32 kernel reproduces exactly: the fp32 launch on the upcast values is the bf16
    # kernel's pre-rounding result, so every wrong element can be classified by how it was rounded
    xb, dyb = x.to(torch.bfloat16), dy.to(torch.bfloat16)
    x, dy = xb.float(), dyb.float()
    o32 = torch.empty((M, D), device=dev)
    ops.layernorm_bwd(x, gamma, mean, rstd, dy, o32)
    victim = lambda o: ops.layernorm_bwd(xb, gamma, mean, rstd, dyb, o)  # noqa: E731


def bf16_round(v, mode):
    """fp32 -> bf16 bits with the given rounding: rne | rtz | up (toward +inf) | down"""
    b = v.contiguous().view(torch.int32).long() & 0xFFFFFFFF
    lo, hi = b & 0xFFFF, b >> 16
    neg = (b >> 31) == 1
    if mode == "rne":
        inc = (lo > 0x8000) | ((lo == 0x8000) & ((hi & 1) == 1))
    elif mode == "rtz":
        inc = torch.zeros_like(lo, dtype=torch.bool)
    elif mode == "up":
        inc = (lo != 0) & ~neg
    else:
        inc = (lo != 0) & neg
    return (hi + inc.long()) & 0xFFFF
for a in aggressors.values():
    a()
ref = torch.empty((M, D), device=dev, dtype=torch.bfloat16 if BF16 else torch.float32)
victim(ref)
torch.cuda.synchronize()
# float64 model of the quiet result and the per-lane partials
xd, dyd, gd = x.double(), dy.double(), gamma.double()
xh = (xd - mean.double()[:, None]) * rstd.double()[:, None]
gy = dyd * gd
lane = torch.arange(D, device=dev) // 8 % 32
P1 = torch.zeros(M, 32, device=dev, dtype=torch.float64).index_add_(1, lane, gy)
P2 = torch.zeros(M, 32, device=dev, dtype=torch.float64).index_add_(1, lane, gy * xh)
print(f"quiet vs float64 model: max |d| {float((ref.double() - (rstd.double()[:, None] * (gy - gy.mean(1, keepdim=True) - xh * (gy * xh).mean(1, keepdim=True)))).abs().max()):.3g}", flush=True)
outs = [torch.empty_like(ref) for _ in range(N_V)]
for an, afn in aggressors.items():
    bad_launch = bad_rows = shown = 0
    for rep in range(REPS):
        torch.cuda.synchronize()
        with torch.cuda.stream(side):
            for _ in range(30):
                afn()
        for o in outs:
            victim(o)
        torch.cuda.synchronize()
        for li, o in enumerate(outs):
            rows = (o != ref).any(1).nonzero().flatten().tolist()
            bad_rows += len(rows)
            bad_launch += bool(rows)
            for r in rows:
                if shown >= SHOW:
                    break
                shown += 1
                if BF16:
                    got = o[r].contiguous().view(torch.int16).long() & 0xFFFF
                    wrong = got != (ref[r].contiguous().view(torch.int16).long() & 0xFFFF)
                    match = {m: int((got == bf16_round(o32[r], m)).sum()) for m in ("rne", "rtz", "up", "down")}
                    print(f"  [{an}] launch {rep}.{li} row {r}: {int(wrong.sum())} of {D} elements wrong; elements equal to "
                          f"the fp32 result rounded {match}; ref == rne(fp32): "
                          f"{bool((bf16_round(o32[r], 'rne') == (ref[r].contiguous().view(torch.int16).long() & 0xFFFF)).all())}",
                          flush=True)
                    continue
                d = (o[r] - ref[r]).double()
                A = torch.stack([torch.ones_like(xh[r]), xh[r]], 1)
                sol = torch.linalg.lstsq(A, d[:, None]).solution.flatten()
                res = float((d - A @ sol).abs().max())
                rs = float(rstd[r])
                ds1, ds2 = -float(sol[0]) / rs * D, -float(sol[1]) / rs * D
                k1 = (P1[r] / ds1).tolist() if ds1 else []
                k2 = (P2[r] / ds2).tolist() if ds2 else []
                best1 = sorted(range(32), key=lambda l: abs(abs(k1[l]) - 1))[:3] if k1 else []
                best2 = sorted(range(32), key=lambda l: abs(abs(k2[l]) - 1))[:3] if k2 else []
                print(f"  [{an}] launch {rep}.{li} row {r} (half {r % 2} of wave, block {r // 8}): max|d| {float(d.abs().max()):.3g}, "
                      f"fit residual {res:.3g}; ds1 {ds1:.4g} (s1 {float(P1[r].sum()):.4g}), ds2 {ds2:.4g} (s2 {float(P2[r].sum()):.4g}); "
                      f"lane partial / ds1 nearest +-1: {[(l, round(k1[l], 4)) for l in best1]}; "
                      f"/ ds2: {[(l, round(k2[l], 4)) for l in best2]}", flush=True)
    print(f"victim ln_bwd_{'bf16' if BF16 else 'f32'} aggressor {an:5s}: {bad_launch:3d} of {N_V * REPS} launches wrong, {bad_rows} rows", flush=True)
