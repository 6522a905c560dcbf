"""Bitwise determinism of the train step against co-scheduled work.

One fused-trainer forward + backward (GPT-2 small frozen + transformer mapper, bf16, dropout off) runs twice from
the same state: alone, and with a long chain of unrelated GEMMs running concurrently on a second HIP stream (so
the step's kernels share CUs, L2 and HBM with foreign workgroups). No kernel of the step uses atomics or
placement-dependent reductions, so every intermediate and the flat gradient must be bitwise identical. On a
mismatch the test names the first differing buffer in schedule order."""

import pytest
import torch

from icap import ops
from oracle import icap_oracle as O
from test_model_gpu import build

pytestmark = pytest.mark.gpu


def _batch(B, dev):
    ids, mask, labels, _ = O.synthetic_batch(B, 50, 13, seed=3)
    emb = torch.randn((B, 512), generator=torch.Generator().manual_seed(4))
    return ids.to(dev), mask.to(dev), labels.to(dev), (emb / emb.norm(dim=-1, keepdim=True)).to(dev)


def _snapshot(t):
    g = t.gws
    snap = [("mapper prefix", t.mws.out if hasattr(t.mws, "out") else None)]
    snap += [(f"x[{l}]", g.x[l]) for l in range(len(g.x))]
    snap += [("logits/dlogits", g.logits), ("dhf", g.dhf), ("loss", g.loss)]
    snap += [("dx", g.dx), ("dx2", g.dx2), ("dxd", g.dxd), ("dqkv (layer 0)", g.dqkv), ("dff (layer 0)", g.dff)]
    snap += [("mapper dout", t.mws.dout), ("flat_grad", t.flat.flat_grad)]
    return [(n, x.detach().clone()) for n, x in snap if x is not None]


def _same(a, b):
    """Equal values, NaN == NaN (the compact head leaves unused logits rows unwritten: they may hold NaN
    patterns of earlier allocations, whose payload bits are not a value)."""
    if not a.is_floating_point():
        return torch.equal(a, b)
    return bool(((a == b) | (a.isnan() & b.isnan())).all())


def _noise(dev, n):
    s = torch.cuda.Stream(dev)
    a = torch.randn((4096, 4096), device=dev).to(torch.bfloat16)
    c = torch.empty((4096, 4096), device=dev, dtype=torch.bfloat16)
    # a split-K shape with the DEFAULT workspace (one per stream since r03: the noise stream gets its own slabs)
    sa = torch.randn((256, 8192), device=dev).to(torch.bfloat16)
    sc = torch.empty((256, 512), device=dev, dtype=torch.bfloat16)
    # the 128 x 128 tile family (row-major and K-outer): the co-resident waves that exposed the packed-FP32 race
    ta, tw = torch.randn((800, 768), device=dev).to(torch.bfloat16), torch.randn((3072, 768), device=dev).to(torch.bfloat16)
    tc = torch.empty((800, 3072), device=dev, dtype=torch.bfloat16)
    tf, tdw = torch.randn((800, 3072), device=dev).to(torch.bfloat16), torch.empty((768, 3072), device=dev)
    torch.cuda.synchronize(dev)

    def launch():
        with torch.cuda.stream(s):
            for i in range(n):
                ops.gemm(a, a, c)
                ops.gemm(sa, sa[:512], sc)
                ops.gemm(ta, tw, tc)
                ops.gemm(ta, tf, tdw, M=768, N=3072, K=800, trans_ab=True)
    return launch, s


@pytest.mark.parametrize("B", [32])
def test_train_step_bitwise_with_concurrent_stream(dev, B):
    from icap import CaptionTrainer

    model = build(O.GPT2Cfg(), O.MapperCfg(), torch.bfloat16, dev)
    t = CaptionTrainer(model, B, 50, lr=1e-4, num_training_steps=10, dropout=False)
    t.load_batch(*_batch(B, dev))
    t._fwd_bwd(True, 1.0)  # warm-up (first-use initialisation)
    torch.cuda.synchronize(dev)
    t._fwd_bwd(True, 1.0)
    torch.cuda.synchronize(dev)
    ref = _snapshot(t)
    launch, s = _noise(dev, 40)
    for rep in range(3):
        launch()  # ~40 x 4096^3 GEMMs queued on the side stream, running under the step below
        t._fwd_bwd(True, 1.0)
        torch.cuda.synchronize(dev)
        s.synchronize()
        got = _snapshot(t)
        for (name, a), (_, b) in zip(ref, got):
            if not _same(a, b):
                diff = ~((a == b) | (a.isnan() & b.isnan()))
                rows = sorted(set(diff.nonzero()[:, 0].tolist())) if a.dim() > 1 else []
                d = (a.float() - b.float()).abs()
                pytest.fail(f"rep {rep}: first differing buffer '{name}': {int(diff.sum())} elements "
                            f"(NaN before {int(a[diff].isnan().sum())}, now {int(b[diff].isnan().sum())}), rows "
                            f"{rows[:8]} ({len(rows)}), n_valid {int(t.gws.n_valid.item())}, max finite |d| "
                            f"{float(d[d.isfinite()].max()) if d.isfinite().any() else 0.0:.3g}")


def test_layernorm_bwd_exact_beside_tile_gemms(dev):
    """The round-5 race in isolation (tools/ab/ln_race_probe.py): the mapper-shaped LayerNorm backward (800 x 768
    bf16, dgamma / dbeta partials, residual gradient) launched 40 times per rep on the main stream while tile and
    K-outer GEMMs run on a second stream; every output bitwise equal to the quiet launch. With packed-FP32
    instructions in the library ~5 % of these launches had rows off by up to an ulp."""
    g = torch.Generator().manual_seed(0)
    M, D = 800, 768
    bf = lambda *sh, sc=1.0: (torch.randn(sh, generator=g) * sc).to(dev, torch.bfloat16)  # noqa: E731
    x, dy, dres = bf(M, D), bf(M, D, sc=1e-4), bf(M, D, sc=1e-4)
    gamma = (1 + 0.1 * torch.randn(D, generator=g)).to(dev)
    mean = (0.1 * torch.randn(M, generator=g)).to(dev)
    rstd = (1 + 0.1 * torch.rand(M, generator=g)).to(dev)
    ws = torch.empty(ops.layernorm_bwd_workspace(M, D), dtype=torch.uint8, device=dev)
    dg, db = torch.zeros(D, device=dev), torch.zeros(D, device=dev)
    run = lambda o: ops.layernorm_bwd(x, gamma, mean, rstd, dy, o, dres=dres, dgamma=dg, dbeta=db, workspace=ws)  # noqa: E731
    launch, s = _noise(dev, 8)
    ops.register_side_stream(s)
    launch()
    torch.cuda.synchronize(dev)
    ref = torch.empty_like(x)
    run(ref)
    torch.cuda.synchronize(dev)
    outs = [torch.empty_like(x) for _ in range(40)]
    bad = []
    for rep in range(5):
        launch()
        for o in outs:
            run(o)
        torch.cuda.synchronize(dev)
        bad += [(rep, i, (o != ref).any(1).nonzero().flatten()[:4].tolist()) for i, o in enumerate(outs) if not torch.equal(o, ref)]
    assert not bad, f"{len(bad)} of 200 launches differ from the quiet one: {bad[:4]}"
