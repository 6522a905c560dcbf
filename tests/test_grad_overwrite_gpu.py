"""The first micro-batch of an accumulation cycle writes the trained mapper's gradients instead of zeroing the flat
gradient buffer and accumulating (engine.GRAD_OVERWRITE: dW GEMMs at beta 0, column sums / LayerNorm parameter sums
stored): bitwise the zero_() + accumulate result; and a two-micro-batch cycle (overwrite, then accumulate) equals the
sum of the two micro-batches' gradients computed separately (fp32: rel 1e-6 — the accumulating products add their
partial sums into the stored value, a different rounding order than adding two finished gradients)."""

import pytest
import torch

from icap import CaptionTrainer
from oracle import icap_oracle as O
from test_model_gpu import TINY_G, TINY_M, build

pytestmark = pytest.mark.gpu


def _batch(seed, dev, B=6, L=14):
    ids, mask, labels, emb = O.synthetic_batch(B, L, 9, vocab=TINY_G.vocab_size, eos=TINY_G.eos,
                                               embed_dim=TINY_M.embed_dim, seed=seed)
    return ids.to(dev), mask.to(dev), labels.to(dev), emb.to(dev)


def _grads(dev, dtype, monkeypatch, overwrite, batches, zeros):
    import icap.engine as E
    monkeypatch.setattr(E, "GRAD_OVERWRITE", overwrite)
    model = build(TINY_G, TINY_M, dtype, dev)
    t = CaptionTrainer(model, 6, 14, lr=1e-3, num_training_steps=4, dropout=False, seed=3)
    assert t._overwrite_ok() == overwrite
    for v in t.flat.grad_views:  # stale gradients (NaN): the overwrite path must not read them (the alignment gaps
        v.fill_(float("nan"))      # between tensors stay zero, as allocated)
    for b, z in zip(batches, zeros):
        t.load_batch(*b)
        t._fwd_bwd(z, 1.0)
    torch.cuda.synchronize()
    return t.flat.flat_grad.clone()


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_overwrite_equals_zero_then_accumulate(dev, dtype, monkeypatch):
    b = [_batch(1, dev)]
    g1 = _grads(dev, dtype, monkeypatch, True, b, [True])
    g0 = _grads(dev, dtype, monkeypatch, False, b, [True])
    assert torch.isfinite(g1).all()
    assert torch.equal(g1, g0)


def test_cycle_accumulates_after_overwrite(dev, monkeypatch):
    ba, bb = _batch(1, dev), _batch(2, dev)
    acc = _grads(dev, torch.float32, monkeypatch, True, [ba, bb], [True, False])
    ga = _grads(dev, torch.float32, monkeypatch, True, [ba], [True])
    gb = _grads(dev, torch.float32, monkeypatch, True, [bb], [True])
    ref = ga.double() + gb.double()
    err = float((acc.double() - ref).abs().max()) / float(ref.abs().max())
    assert err < 1e-6, err
