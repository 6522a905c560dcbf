"""Grouped mapper weight gradients (CaptionTrainer(mapper_dw="group"), mapper.backward_steps group=): a layer's four K-outer dW
products queued at the end of its backward step, unsplit, one on the main stream and three on registered side
streams, joined before the next layer. Checked: the gradients equal the serial split-K schedule's to fp32 summation
order (rel 1e-5 of the largest entry: the same bf16 products, a different K-sum order), the schedule is bitwise
reproducible, and three graph-replayed steps equal three eager ones bitwise (the four-stream fork / join captures)."""

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


def _trainer(dev, monkeypatch, group):
    """group: True / "group" (four streams), "fused" (one grouped launch), False (serial)."""
    mode = "group" if group is True else group if group else "serial"
    model = build(TINY_G, TINY_M, torch.bfloat16, dev)
    t = CaptionTrainer(model, 6, 14, lr=1e-3, num_training_steps=8, dropout=True, seed=3, mapper_dw=mode)
    assert (t._group is not None) == bool(group)
    return t


def _grads(dev, monkeypatch, group):
    t = _trainer(dev, monkeypatch, group)
    t.load_batch(*_batch(1, dev))
    t._fwd_bwd(True, 1.0)
    torch.cuda.synchronize()
    return t.flat.flat_grad.clone()


@pytest.mark.parametrize("group", [True, "fused"])
def test_grouped_dw_matches_serial(dev, monkeypatch, group):
    g1 = _grads(dev, monkeypatch, group)
    g0 = _grads(dev, monkeypatch, False)
    assert torch.isfinite(g1).all()
    err = float((g1.double() - g0.double()).abs().max()) / float(g0.abs().max())
    assert err < 1e-5, err


@pytest.mark.parametrize("group", [True, "fused"])
def test_grouped_dw_reproducible(dev, monkeypatch, group):
    a = _grads(dev, monkeypatch, group)
    b = _grads(dev, monkeypatch, group)
    assert torch.equal(a, b)


def test_fused_dw_matches_group(dev, monkeypatch):
    """mapper_dw="fused" (one grouped launch on the K-outer split-role body, the bias gradients as products against a
    ones column in the same launch) and "group" (the K-outer tile kernel on four streams + column sums) run each
    weight product unsplit in natural K order — bitwise the same weight gradients — and sum the bias gradients in
    different orders (fp32): equal to rel 1e-6 of the largest entry."""
    a, b = _grads(dev, monkeypatch, "fused"), _grads(dev, monkeypatch, True)
    err = float((a.double() - b.double()).abs().max()) / float(b.abs().max())
    assert err < 1e-6, err
    assert float((a == b).float().mean()) > 0.9  # the weight gradients (most of the buffer) bitwise


@pytest.mark.parametrize("group", [True, "fused"])
def test_grouped_dw_graph_equals_eager(dev, monkeypatch, group):
    out = []
    for use_graph in (True, False):
        t = _trainer(dev, monkeypatch, group)
        for s in range(3):
            t.load_batch(*_batch(10 + s, dev))
            t.micro_step(use_graph=use_graph)
        torch.cuda.synchronize()
        out.append(t.flat.flat.clone())
    assert torch.equal(out[0], out[1])


def test_side_dw_bitwise_serial(dev):
    """mapper_dw="side": the weight-gradient products run beside the dX chain on a second stream. Each is the same
    kernel on the same operands as in the serial schedule, so the flat gradient is bitwise the serial one, on every
    call (round 5: before the library dropped packed-FP32 instructions, the LayerNorm backward co-resident with these
    products broke this — DESIGN.md "Concurrency: the packed-FP32 race")."""
    from test_determinism_gpu import _batch

    from icap import CaptionTrainer as T

    out = {}
    for mode in ("serial", "side"):
        model = build(O.GPT2Cfg(), O.MapperCfg(), torch.bfloat16, dev)
        t = T(model, 32, 50, lr=1e-4, num_training_steps=10, dropout=False, mapper_dw=mode)
        assert (t._side is not None) == (mode == "side")
        t.load_batch(*_batch(32, dev))
        grads = []
        for _ in range(4 if mode == "side" else 1):
            t._fwd_bwd(True, 1.0)
            torch.cuda.synchronize()
            grads.append(t.flat.flat_grad.clone())
        out[mode] = grads
        del t, model
    ref = out["serial"][0]
    for i, gr in enumerate(out["side"]):
        assert torch.equal(gr, ref), f"side call {i}: {int((gr != ref).sum())} gradient entries differ"
