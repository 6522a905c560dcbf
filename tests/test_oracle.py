"""Pin the CPU oracle (oracle/icap_oracle.py) to golden vectors produced by the reference itself
(tools/make_goldens.py: src/models.py ImageCaptioningModel / src/train.py::train over HF GPT-2/CLIP
in this container, dropout off). CPU only."""

import os

import numpy as np
import pytest
import torch

from oracle import icap_oracle as O

GOLD = os.path.join(os.path.dirname(__file__), "golden")

TINY_G = O.GPT2Cfg(n_layer=2, n_embd=128, n_head=2, vocab_size=512, n_positions=128, eos=511)
TINY_M = O.MapperCfg(embed_dim=64, gpt_dim=128, prefix_length=5, hidden_length=4, num_layers=2)


def load(name):
    return dict(np.load(os.path.join(GOLD, name + ".npz")))


def inputs(g):
    return (torch.from_numpy(g["ids"]), torch.from_numpy(g["mask"]), torch.from_numpy(g["labels"]),
            torch.from_numpy(g["emb"]))


def rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


@pytest.fixture(scope="module")
def small_weights():
    return O.gpt2_state_dict(O.GPT2Cfg(), 0), O.mapper_state_dict(O.MapperCfg(), 0)


def test_tiny_forward_and_greedy():
    g = load("tiny")
    ids, mask, labels, emb = inputs(g)
    gsd, msd = O.gpt2_state_dict(TINY_G, 0), O.mapper_state_dict(TINY_M, 0)
    prefix = O.mapper_forward(msd, TINY_M, emb)
    assert rel(prefix, g["prefix"]) < 1e-5
    loss, logits = O.caption_forward(gsd, TINY_G, prefix, ids, mask, labels)
    assert abs(loss.item() - g["loss"][0]) < 1e-5
    assert rel(logits, g["logits"]) < 1e-5
    gen = O.greedy_generate(gsd, TINY_G, prefix, max_length=20)
    assert np.array_equal(gen.numpy(), g["greedy"])


def test_tiny_train_frozen_and_unfrozen():
    g = load("tiny")
    batch = inputs(g)
    gsd, msd = O.gpt2_state_dict(TINY_G, 0), O.mapper_state_dict(TINY_M, 0)
    n = len(g["train_losses"])
    losses, _, new_m, _ = O.train_steps(gsd, TINY_G, msd, TINY_M, [batch] * n, lr0=1e-4, total_steps=n)
    # epoch_losses[k] is the loss of step k (before its update)
    assert rel(losses, g["train_losses"]) < 1e-5
    for k, v in new_m.items():
        # AdamW normalises each gradient element, so elements whose true gradient is ~0 (e.g. the key bias of
        # in_proj_bias, invariant under softmax shifts) move by rounding noise x lr: compare the UPDATE, to 3 %.
        upd = g["trained." + k] - msd[k].numpy()
        assert np.abs(v.numpy() - g["trained." + k]).max() <= 0.03 * np.abs(upd).max(), k
    n2 = len(g["unfrozen_losses"])
    losses2, _, m2, g2 = O.train_steps(gsd, TINY_G, msd, TINY_M, [batch] * n2, lr0=1e-4, total_steps=n2,
                                       freeze_gpt=False)
    assert rel(losses2, g["unfrozen_losses"]) < 1e-5
    for k, v in g2.items():
        ck = g["unfrozen_ck.gpt." + k]
        t = v.double()
        assert rel([t.sum().item(), t.abs().sum().item()], ck[:2]) < 1e-5, k


def test_tiny_mlp_mapper():
    g = load("tiny_mlp")
    ids, mask, labels, emb = inputs(g)
    gsd = O.gpt2_state_dict(TINY_G, 0)
    mcfg = O.MLPMapperCfg(prefix_length=5, embed_dim=64, gpt_dim=128)
    prefix = O.mlp_mapper_forward(O.mlp_mapper_state_dict(mcfg, 0), mcfg, emb)
    assert rel(prefix, g["prefix"]) < 1e-5
    loss, logits = O.caption_forward(gsd, TINY_G, prefix, ids, mask, labels)
    assert abs(loss.item() - g["loss"][0]) < 1e-5
    assert rel(logits, g["logits"]) < 1e-5


def test_small_forward(small_weights):
    g = load("small")
    gsd, msd = small_weights
    ids, mask, labels, emb = inputs(g)
    prefix = O.mapper_forward(msd, O.MapperCfg(), emb)
    assert rel(prefix, g["prefix"]) < 1e-5
    loss, logits = O.caption_forward(gsd, O.GPT2Cfg(), prefix, ids, mask, labels)
    assert abs(loss.item() - g["loss"][0]) < 1e-5
    rows = g["logit_rows"]
    assert rel(logits[:2][:, rows], g["logits_sel"]) < 1e-5
    lse = torch.logsumexp(logits.double(), -1).numpy()
    assert np.abs(lse - g["lse"]).max() < 1e-4
    assert np.mean(logits.argmax(-1).numpy() == g["argmax"]) > 0.99


def test_small_greedy(small_weights):
    g = load("small")
    gsd, msd = small_weights
    emb = torch.from_numpy(g["emb"])[: g["greedy"].shape[0]]
    prefix = O.mapper_forward(msd, O.MapperCfg(), emb)
    gen = O.greedy_generate(gsd, O.GPT2Cfg(), prefix, max_length=g["greedy"].shape[1])
    assert np.array_equal(gen.numpy(), g["greedy"])


def test_small_train(small_weights):
    g = load("small")
    gsd, msd = small_weights
    n = len(g["train_losses"])
    losses, _, new_m, _ = O.train_steps(gsd, O.GPT2Cfg(), msd, O.MapperCfg(), [inputs(g)] * n, total_steps=n)
    assert rel(losses, g["train_losses"]) < 1e-5
    for k, v in new_m.items():
        t = v.double()
        ck = g["trained_ck." + k]
        assert rel([t.sum().item(), t.abs().sum().item()], ck[:2]) < 1e-4, k


def test_clip_b32():
    g = load("clip_b32")
    cfg = O.ClipCfg()
    sd = O.clip_vision_state_dict(cfg, 0)
    px = torch.randn((2, 3, 224, 224), generator=torch.Generator().manual_seed(int(g["pixels_seed"][0])))
    f = O.clip_image_features(sd, cfg, px)
    assert rel(f, g["features"]) < 1e-5
    e = O.clip_embed_normalized(sd, cfg, px)
    assert rel(e, g["embeddings"]) < 1e-5


def test_adamw_restatement_matches_torch():
    """oracle.clip_and_adamw == clip_grad_norm_ + torch.optim.AdamW + LambdaLR (src/train.py:94-103,150-156)."""
    gen = torch.Generator().manual_seed(5)
    ps = {"a": torch.randn(37, generator=gen), "b": torch.randn(5, 7, generator=gen)}
    tp = [torch.nn.Parameter(v.clone()) for v in ps.values()]
    opt = torch.optim.AdamW(tp, lr=1e-3, weight_decay=0.01)
    sched = torch.optim.lr_scheduler.LambdaLR(opt, lambda s: O.linear_schedule(s, 1, 6))
    st = O.AdamWState()
    for k in range(4):
        gr = {n: torch.randn(v.shape, generator=gen) * (0.3 + k) for n, v in ps.items()}
        for p, gg in zip(tp, gr.values()):
            p.grad = gg.clone()
        torch.nn.utils.clip_grad_norm_(tp, 1.0)
        opt.step()
        sched.step()
        O.clip_and_adamw(ps, gr, st, 1e-3, 1, 6)
    for p, v in zip(tp, ps.values()):
        assert torch.allclose(p.detach(), v, rtol=1e-6, atol=1e-7)


MED_G = O.GPT2Cfg(n_layer=24, n_embd=1024, n_head=16)  # BASELINE configs[3]: GPT-2 medium
MED_M = O.MapperCfg(embed_dim=768, gpt_dim=1024)     # mapper over CLIP-L/14 (768-d), head dim 128
L14 = O.ClipCfg(hidden=1024, layers=24, heads=16, patch=14, image=224, inter=4096, proj=768)


def test_medium_forward_greedy_train():
    """configs[3] geometry pinned to the reference (tools/make_goldens.py golden_medium)."""
    g = load("medium")
    gsd, msd = O.gpt2_state_dict(MED_G, 0), O.mapper_state_dict(MED_M, 0)
    ids, mask, labels, emb = inputs(g)
    prefix = O.mapper_forward(msd, MED_M, emb)
    assert rel(prefix, g["prefix"]) < 1e-5
    loss, logits = O.caption_forward(gsd, MED_G, prefix, ids, mask, labels)
    assert abs(loss.item() - g["loss"][0]) < 1e-5
    assert rel(logits[:2][:, g["logit_rows"]], g["logits_sel"]) < 1e-5
    gen = O.greedy_generate(gsd, MED_G, prefix[: g["greedy"].shape[0]], max_length=g["greedy"].shape[1])
    assert np.array_equal(gen.numpy(), g["greedy"])
    n = len(g["train_losses"])
    losses, _, new_m, _ = O.train_steps(gsd, MED_G, msd, MED_M, [inputs(g)] * n, total_steps=n)
    assert rel(losses, g["train_losses"]) < 1e-5
    for k, v in new_m.items():
        t = v.double()
        assert rel([t.sum().item(), t.abs().sum().item()], g["trained_ck." + k][:2]) < 1e-4, k


def test_clip_l14():
    g = load("clip_l14")
    sd = O.clip_vision_state_dict(L14, 0)
    px = torch.randn((2, 3, 224, 224), generator=torch.Generator().manual_seed(int(g["pixels_seed"][0])))
    assert rel(O.clip_image_features(sd, L14, px), g["features"]) < 1e-5
    assert rel(O.clip_embed_normalized(sd, L14, px), g["embeddings"]) < 1e-5


def test_small_train_three_steps_and_unfrozen(small_weights):
    """3 frozen reference train() steps (whole / sampled trained tensors) and 2 unfrozen ones (every GPT-2 tensor)."""
    g = load("small_train")
    gsd, msd = small_weights
    batch = inputs(g)
    losses, _, new_m, _ = O.train_steps(gsd, O.GPT2Cfg(), msd, O.MapperCfg(), [batch] * 3, total_steps=3)
    assert rel(losses, g["train_losses"]) < 1e-5
    for k, v in new_m.items():
        if "trained." + k in g:
            ref, got, init = g["trained." + k], v.numpy(), msd[k].numpy()
        elif "trained_sample." + k in g:
            ref = g["trained_sample." + k]
            got, init = v.numpy().reshape(-1)[::97], msd[k].numpy().reshape(-1)[::97]
        else:
            continue
        assert np.abs(got - ref).max() <= 0.03 * np.abs(ref - init).max() + 1e-9, k
    losses2, _, _, g2 = O.train_steps(gsd, O.GPT2Cfg(), msd, O.MapperCfg(), [batch] * 2, total_steps=2,
                                      freeze_gpt=False)
    assert rel(losses2, g["unfrozen_losses"]) < 1e-5
    for k, v in g2.items():
        t = v.double()
        assert rel([t.sum().item(), t.abs().sum().item()], g["unfrozen_ck.gpt." + k][:2]) < 1e-5, k


def test_topp_filter_matches_reference():
    """The reference's own top-p filter output (src/models.py:400-449 as it ran: probs > 0 after filtering) equals
    the oracle's restatement on the same logits, at every recorded step and row."""
    g = load("topp_filter")
    T, p = float(g["temperature"][0]), float(g["top_p"][0])
    for step in range(g["probs"].shape[0]):
        kept_ref = g["probs"][step] > 0
        kept = O.topp_filter_reference(torch.from_numpy(g["logits"][step]), T, p).numpy()
        assert np.array_equal(kept, kept_ref), step
        # and the kernel's fixed-point restatement keeps the same set
        _, kept_fixed = O.topp_sample_fixed(g["logits"][step], T, p, seed=3, step=step, eos=511)
        assert np.array_equal(kept_fixed, kept_ref), step
