"""LN backward side-stream victim, echo build (diagnostic; follows ln_race_probe.py / ln_race_f32.py).

With ICAP_LIB = a -DICAP_LN_ECHO build of layernorm.hip, ln_bwd8 runs its whole computation but stores the x values
it loaded (o = x + 0 * result), so any difference from x is a wrong load. For each wrong row: the wrong 16-byte
chunks (lane, t) and where their bytes occur in the tensors of the run (x / dy / aggressor buffers, any chunk).
"""
import os
import sys

sys.path[:0] = ["/root/repo", "/root/repo/gpt2-image-captioning_amd"]
import torch  # noqa: E402

from icap import ops  # noqa: E402

dev = torch.device("cuda", 0)
M, D, F = 800, 768, 3072
N_V, REPS, SHOW = 40, int(os.environ.get("PROBE_REPS", "8")), 8
g = torch.Generator().manual_seed(0)
bf = lambda *s, sc=1.0: (torch.randn(s, generator=g) * sc).to(dev, torch.bfloat16)  # noqa: E731
x = bf(M, D)
gamma = (1 + 0.1 * torch.randn(D, generator=g)).to(dev)
mean = (0.1 * torch.randn(M, generator=g)).to(dev)
rstd = (1 + 0.1 * torch.rand(M, generator=g)).to(dev)
dy = bf(M, D, sc=1e-4)
dres = bf(M, D, sc=1e-4)
f = bf(M, F)
wt = bf(F, D, sc=0.02)
ct = torch.empty((M, F), device=dev, dtype=torch.bfloat16)
dW = torch.empty((D, F), device=dev, dtype=torch.float32)
side = torch.cuda.Stream(dev)
ops.register_side_stream(side)
aggressors = {"none": lambda: None, "tile": lambda: ops.gemm(dres, wt, ct),
              "kout": lambda: ops.gemm(dres, f, dW, M=D, N=F, K=M, trans_ab=True)}
victim = lambda o: ops.layernorm_bwd(x, gamma, mean, rstd, dy, o)  # noqa: E731
for a in aggressors.values():
    a()
ref = torch.empty_like(x)
victim(ref)
torch.cuda.synchronize()
print(f"quiet echo == x: {bool(torch.equal(ref, x))}", flush=True)


def chunks(t):
    """16-byte chunks of a bf16/fp32 tensor as rows of 4 int32"""
    return t.contiguous().view(torch.int32).view(-1, 4)


pools = {"x": chunks(x), "dy": chunks(dy), "dres": chunks(dres), "wt": chunks(wt), "f": chunks(f), "ct": chunks(ct)}
outs = [torch.empty_like(x) for _ in range(N_V)]
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
            rows = (o != x).any(1).nonzero().flatten().tolist()
            bad_rows += len(rows)
            bad_launch += bool(rows)
            for r in rows:
                if shown >= SHOW:
                    break
                shown += 1
                oc, xc = chunks(o[r]), chunks(x[r])
                wrong = (oc != xc).any(1).nonzero().flatten().tolist()
                desc = []
                for c in wrong[:6]:
                    hits = []
                    for pn, pool in pools.items():
                        idx = (pool == oc[c]).all(1).nonzero().flatten().tolist()
                        hits += [f"{pn}[{i // (pool.shape[0] // (x.shape[0] if pn in ('x', 'dy', 'dres') else 1))}]"
                                 f"chunk{i}" for i in idx[:2]]
                    desc.append(f"chunk {c} (lane {c % 32}, t {c // 32}): {o[r, 8 * c:8 * c + 8].float().tolist()} "
                                f"vs x {x[r, 8 * c:8 * c + 8].float().tolist()}; found at {hits or 'nowhere'}")
                print(f"  [{an}] launch {rep}.{li} row {r}: {len(wrong)} wrong chunks {wrong[:16]}", flush=True)
                for d_ in desc:
                    print("     ", d_, flush=True)
    print(f"echo victim aggressor {an:5s}: {bad_launch:3d} of {N_V * REPS} launches wrong, {bad_rows} rows", flush=True)
