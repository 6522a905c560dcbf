"""Victim kernels beside co-scheduled work on a second stream (diagnostic; follows det_probe5).

det_probe5 localised the side-stream nondeterminism to single rows of the mapper's LN2 backward: the first launch
after the fork is wrong in 1-7 rows, a relaunch on the same inputs right after it and a quiet recomputation agree.
Round-5 call H reproduced it with static inputs: the LayerNorm backward (mapper shape) launched N times on the main
stream while a GEMM runs on a second stream is wrong in a few rows of ~10 % of the launches; a torch copy as the
aggressor, or none, leaves it exact.

Here every (victim, aggressor) pair: the victim is launched N times into N separate outputs on the main stream while
the aggressor is queued 30 times on the side stream; every output is compared with the victim's quiet result.
Victims: ln_bwd, ln_fwd, convert (icap_convert bf16 -> f32), torch_copy. Aggressors: none, tile (row-major tile GEMM,
LDS-DMA staging), kout (K-outer GEMM, LDS-DMA + ds_read_b64_tr_b16), g256 (256 x 256 8-phase kernel), skinny (the
M <= 128 GEMM: loads straight to VGPRs, no LDS-DMA), attn (attention forward), copy (torch copy).
"""
import os
import sys

sys.path[:0] = ["/root/repo", "/root/repo/gpt2-image-captioning_amd"]
import torch  # noqa: E402

from icap import ops  # noqa: E402

dev = torch.device("cuda", 0)
M = int(os.environ.get("PROBE_M", "800"))
D, F = 768, 3072
N_V = int(os.environ.get("PROBE_N", "40"))
REPS = int(os.environ.get("PROBE_REPS", "5"))
g = torch.Generator().manual_seed(0)
bf = lambda *s, sc=1.0: (torch.randn(s, generator=g) * sc).to(dev, torch.bfloat16)  # noqa: E731
x = bf(M, D)
gamma = (1 + 0.1 * torch.randn(D, generator=g)).to(dev)
beta = (0.1 * torch.randn(D, generator=g)).to(dev)
mean = (0.1 * torch.randn(M, generator=g)).to(dev)
if os.environ.get("PROBE_CONST_MEAN"):  # every row the same mean: a mean read from the wrong row would be harmless
    mean.fill_(0.05)
rstd = (1 + 0.1 * torch.rand(M, generator=g)).to(dev)
dy = bf(M, D, sc=1e-4)
dres = bf(M, D, sc=1e-4)
dres_copy = dres.clone()
f = bf(M, F)
dW = torch.empty((D, F), device=dev, dtype=torch.float32)
wt = bf(F, D, sc=0.02)
ct = torch.empty((M, F), device=dev, dtype=torch.bfloat16)
big = bf(4096, 4096, sc=0.05)
bigc = torch.empty_like(big)
sk_a, sk_w = bf(128, 768), bf(3072, 768, sc=0.02)
sk_c = torch.empty((128, 3072), device=dev, dtype=torch.bfloat16)
qkv = bf(128 * 65, 3 * D)
ao = torch.empty((128 * 65, D), device=dev, dtype=torch.bfloat16)
cp_src = torch.randn(32 << 20, device=dev)
cp_dst = torch.empty_like(cp_src)
side = torch.cuda.Stream(dev)
ops.register_side_stream(side)
ws = torch.empty(ops.layernorm_bwd_workspace(M, D), dtype=torch.uint8, device=dev)
dg = torch.zeros(D, device=dev)
db = torch.zeros(D, device=dev)
mo, ro = torch.empty(M, device=dev), torch.empty(M, device=dev)

victims = {
    "ln_bwd": (lambda o: ops.layernorm_bwd(x, gamma, mean, rstd, dy, o, dres=dres, dgamma=dg, dbeta=db, workspace=ws),
               torch.bfloat16),
    "ln_bwd_noparams": (lambda o: ops.layernorm_bwd(x, gamma, mean, rstd, dy, o, dres=dres), torch.bfloat16),
    "ln_bwd_nores": (lambda o: ops.layernorm_bwd(x, gamma, mean, rstd, dy, o, dgamma=dg, dbeta=db, workspace=ws),
                     torch.bfloat16),
    "ln_bwd_bare": (lambda o: ops.layernorm_bwd(x, gamma, mean, rstd, dy, o), torch.bfloat16),
    "ln_fwd": (lambda o: ops.layernorm_fwd(x, gamma, beta, 1e-5, o, mo, ro), torch.bfloat16),
    "convert": (lambda o: ops.convert(dres, o), torch.float32),
    "torch_copy": (lambda o: o.copy_(dres), torch.bfloat16),
}
aggressors = {
    "none": lambda: None,
    "tile": lambda: ops.gemm(dres, wt, ct),
    "kout": lambda: ops.gemm(dres_copy, f, dW, M=D, N=F, K=M, trans_ab=True),
    "tile_nosplit": lambda: ops.gemm(dres, wt, ct, split_k=1),  # (no in-launch split-K: no tickets / fences)
    "kout_nosplit": lambda: ops.gemm(dres_copy, f, dW, M=D, N=F, K=M, trans_ab=True, split_k=1),
    "g256": lambda: ops.gemm(big, big, bigc),
    "skinny": lambda: ops.gemm(sk_a, sk_w, sk_c),
    "attn": lambda: ops.attention_fwd(qkv, ao, B=128, S=65, H=12, hd=64, scale=0.125, causal=True),
    "copy": lambda: cp_dst.copy_(cp_src),
}
only_v = [v for v in os.environ.get("PROBE_VICTIMS", ",".join(victims)).split(",") if v]
only_a = [a for a in os.environ.get("PROBE_AGGRESSORS", ",".join(aggressors)).split(",") if a]
for name in only_a:  # first-use initialisation
    aggressors[name]()
torch.cuda.synchronize()

for vn in only_v:
    vfn, vdt = victims[vn]
    ref = torch.empty((M, D), device=dev, dtype=vdt)
    vfn(ref)
    torch.cuda.synchronize()
    outs = [torch.empty_like(ref) for _ in range(N_V)]
    for an in only_a:
        afn = aggressors[an]
        bad_launch = bad_rows = 0
        shown = False
        for rep in range(REPS):
            torch.cuda.synchronize()
            with torch.cuda.stream(side):
                for _ in range(30):
                    afn()
            for o in outs:
                vfn(o)
            torch.cuda.synchronize()
            for o in outs:
                rows = (o != ref).any(1).nonzero().flatten()
                nb = int(rows.numel())
                bad_rows += nb
                bad_launch += nb > 0
                if nb and not shown:  # forensics of one wrong row: where the differences sit
                    shown = True
                    r = int(rows[0])
                    d = (o[r].float() - ref[r].float()).abs()
                    top = torch.topk(d, 8).indices.sort().values.tolist()
                    # which per-row input explains it: least-squares fit of the kernel's formula with the row's mean
                    # replaced (the output is nearly linear in it), in float64
                    xr, dyr, rr_ = x[r].double(), dy[r].double(), dres[r].double() if "nores" not in vn and "bare" not in vn else 0
                    def model(mu, rsd):
                        xh = (xr - mu) * rsd
                        gy = dyr * gamma.double()
                        return rsd * (gy - gy.mean() - xh * (gy * xh).mean()) + rr_
                    if vn.startswith("ln_bwd"):
                        m0, r0 = float(mean[r]), float(rstd[r])
                        eps_m = 1e-3
                        d0, dm = model(m0, r0), (model(m0 + eps_m, r0) - model(m0 - eps_m, r0)) / (2 * eps_m)
                        dmean = float(((o[r].double() - d0) * dm).sum() / (dm * dm).sum())
                        near = (mean.double() - (m0 + dmean)).abs().argsort()[:3].tolist()
                        print(f"    fit: mean off by {dmean:.4g} (row mean {m0:.4g}); rows whose mean is closest to the fit: "
                              f"{[(i, round(float(mean[i]), 5)) for i in near]}", flush=True)
                    print(f"    first wrong row {r}: {int((d > 0).sum())} elements differ, max {float(d.max()):.3g} "
                          f"(|ref| max {float(ref[r].float().abs().max()):.3g}); largest at columns {top}", flush=True)
        print(f"victim {vn:10s} aggressor {an:7s}: {bad_launch:3d} of {N_V * REPS} launches wrong, {bad_rows} rows",
              flush=True)
