"""Model-level parity of the HIP path against the reference's own outputs (tests/golden, produced by
tools/make_goldens.py from src/models.py + src/train.py) and the CPU oracle on the same inputs.

Tolerances (stated per test):
  fp32 parity mode (exact-fp32 MFMA chains, only summation order differs from the CPU):
    loss |d| <= 2e-5, logits max-rel <= 1e-4, greedy ids exact.
  bf16 perf mode (bf16 storage, fp32 accumulation): loss |d| <= 3e-2, logits max-rel <= 5e-2,
    last-position argmax agreement >= 90 %.
  AdamW steps: the UPDATE (param - init) agrees to 5 % of its max magnitude (AdamW normalises each
    element, so elements with ~0 true gradient move by rounding noise x lr).
"""

import os
from types import SimpleNamespace

import numpy as np
import pytest
import torch

from icap import CaptionTrainer, GPT2Config, GPT2LMHeadModel, ImageCaptioningModel, MLPMappingNetwork
from icap import TransformerMappingNetwork
from icap.clip import CLIPVisionTower
from oracle import icap_oracle as O

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
TINY_G = O.GPT2Cfg(n_layer=2, n_embd=128, n_head=2, vocab_size=512, n_positions=128, eos=511)
TINY_M = O.MapperCfg(embed_dim=64, gpt_dim=128, prefix_length=5, hidden_length=4, num_layers=2)


def load(name):
    return dict(np.load(os.path.join(GOLD, name + ".npz")))


def inputs(g, dev):
    return tuple(torch.from_numpy(g[k]).to(dev) for k in ("ids", "mask", "labels", "emb"))


def rel(a, b):
    a = torch.as_tensor(a).detach().double().cpu()
    b = torch.as_tensor(b).detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def build(gc: O.GPT2Cfg, mc, dtype, dev, mapper="transformer", freeze=True):
    cfg = GPT2Config(vocab_size=gc.vocab_size, n_positions=gc.n_positions, n_embd=gc.n_embd, n_layer=gc.n_layer,
                     n_head=gc.n_head, layer_norm_epsilon=gc.eps, eos_token_id=gc.eos)
    gpt = GPT2LMHeadModel(cfg)
    missing, unexpected = gpt.load_state_dict(O.gpt2_state_dict(gc, 0), strict=False)
    assert not unexpected and missing == ["lm_head.weight"]
    if mapper == "transformer":
        m = TransformerMappingNetwork(mc.embed_dim, mc.gpt_dim, mc.prefix_length, mc.hidden_length, mc.num_layers)
        m.load_state_dict(O.mapper_state_dict(mc, 0))
    else:
        m = MLPMappingNetwork(mc.prefix_length, mc.embed_dim, mc.gpt_dim)
        m.load_state_dict(O.mlp_mapper_state_dict(mc, 0))
    model = ImageCaptioningModel(m, tokenizer=SimpleNamespace(eos_token_id=gc.eos), gpt=gpt,
                                 freeze_gpt_weights=freeze, compute_dtype=dtype)
    return model.to(dev)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_tiny_forward(dev, dtype):
    g = load("tiny")
    ids, mask, labels, emb = inputs(g, dev)
    model = build(TINY_G, TINY_M, dtype, dev).eval()
    with torch.no_grad():
        prefix = model.mapping_network(emb.to(dtype))
        out = model(ids, emb, mask, labels)
    if dtype == torch.float32:
        assert rel(prefix, g["prefix"]) < 1e-4
        assert abs(out.loss.item() - g["loss"][0]) < 2e-5
        assert rel(out.logits, g["logits"]) < 1e-4
    else:
        assert abs(out.loss.item() - g["loss"][0]) < 3e-2
        assert rel(out.logits, g["logits"]) < 5e-2


def test_tiny_greedy_exact(dev):
    g = load("tiny")
    _, _, _, emb = inputs(g, dev)
    model = build(TINY_G, TINY_M, torch.float32, dev)
    gen = model.generate(emb, max_length=20, temperature=0.0)
    assert np.array_equal(gen.cpu().numpy(), g["greedy"])


def test_tiny_generate_sampling_branch(dev):
    """generate(temperature > 0, top_p < 1) runs the HIP nucleus sampler (src/models.py:400-449): reproducible
    under torch.manual_seed, ids inside the vocabulary, EOS latched once emitted; temperature 0 stays greedy."""
    g = load("tiny")
    _, _, _, emb = inputs(g, dev)
    model = build(TINY_G, TINY_M, torch.float32, dev)
    torch.manual_seed(0)
    a = model.generate(emb, max_length=12, temperature=1.2, top_p=0.9).cpu()
    torch.manual_seed(0)
    b = model.generate(emb, max_length=12, temperature=1.2, top_p=0.9).cpu()
    assert torch.equal(a, b)
    assert a.min() >= 0 and a.max() < TINY_G.vocab_size
    for row in a.tolist():
        if TINY_G.eos in row:
            assert all(t == TINY_G.eos for t in row[row.index(TINY_G.eos):])
    gc = model._gcore()
    gc.graph_decode = False  # the eager loop draws the same tokens as the graph-chunk runner for one seed
    try:
        torch.manual_seed(0)
        c = model.generate(emb, max_length=12, temperature=1.2, top_p=0.9).cpu()
    finally:
        gc.graph_decode = True
    assert torch.equal(a, c)
    torch.manual_seed(1)
    d = model.generate(emb, max_length=12, temperature=1.2, top_p=0.9).cpu()
    assert not torch.equal(a, d)  # the seed reaches the captured graphs through device memory
    gen = model.generate(emb, max_length=20, temperature=0.0)
    assert np.array_equal(gen.cpu().numpy(), g["greedy"])


def test_tiny_mlp_mapper(dev):
    g = load("tiny_mlp")
    ids, mask, labels, emb = inputs(g, dev)
    mc = O.MLPMapperCfg(prefix_length=5, embed_dim=64, gpt_dim=128)
    model = build(TINY_G, mc, torch.float32, dev, mapper="mlp").eval()
    with torch.no_grad():
        out = model(ids, emb, mask, labels)
        prefix = model.mapping_network(emb)
    assert rel(prefix, g["prefix"]) < 1e-4
    assert abs(out.loss.item() - g["loss"][0]) < 2e-5
    assert rel(out.logits, g["logits"]) < 1e-4


@pytest.mark.parametrize("graph", [False, True])
def test_tiny_mlp_fused_train_matches_reference(dev, graph):
    """MLPMappingNetwork trained through the fused trainer (tanh-epilogue forward, dtanh backward, dW / bias grads,
    AdamW) vs 3 steps of the reference train() with that mapper (src/models.py:14-74, train.py:119-166)."""
    g = load("tiny_mlp")
    mc = O.MLPMapperCfg(prefix_length=5, embed_dim=64, gpt_dim=128)
    model = build(TINY_G, mc, torch.float32, dev, mapper="mlp")
    init = {k: v.detach().clone().cpu() for k, v in model.mapping_network.state_dict().items()}
    losses, _ = _trainer_steps(model, inputs(g, dev), len(g["train_losses"]), graph=graph)
    assert rel(losses, g["train_losses"]) < 1e-5
    _check_updates(model, g, init)


def _trainer_steps(model, batch, n, graph=False):
    ids, mask, labels, emb = batch
    t = CaptionTrainer(model, ids.shape[0], ids.shape[1], lr=1e-4, num_training_steps=n, dropout=False)
    t.load_batch(ids, mask, labels, emb)
    losses = []
    for _ in range(n):
        t.micro_step(use_graph=graph)
        losses.append(t.last_loss.item())
    return losses, t


def _check_updates(model, g, init_sd, key_prefix="trained."):
    for k, v in model.mapping_network.state_dict().items():
        ref = torch.from_numpy(g[key_prefix + k]).double()
        upd = (ref - init_sd[k].double()).abs().max()
        assert (v.detach().double().cpu() - ref).abs().max() <= 0.05 * upd + 1e-7, k


def test_tiny_fused_train_matches_reference(dev):
    """src/train.py::train inner loop (3 AdamW steps, frozen GPT-2) vs the fused HIP trainer (fp32)."""
    g = load("tiny")
    batch = inputs(g, dev)
    model = build(TINY_G, TINY_M, torch.float32, dev)
    losses, _ = _trainer_steps(model, batch, 3)
    assert rel(losses, g["train_losses"]) < 1e-5
    _check_updates(model, g, O.mapper_state_dict(TINY_M, 0))


def test_graph_replay_equals_eager(dev):
    g = load("tiny")
    batch = inputs(g, dev)
    m1 = build(TINY_G, TINY_M, torch.float32, dev)
    m2 = build(TINY_G, TINY_M, torch.float32, dev)
    l1, _ = _trainer_steps(m1, batch, 4, graph=False)
    l2, _ = _trainer_steps(m2, batch, 4, graph=True)
    assert l1 == l2
    for (k, a), b in zip(m1.mapping_network.state_dict().items(), m2.mapping_network.state_dict().values()):
        assert torch.equal(a, b), k


def test_tiny_autograd_dropin_unfrozen(dev):
    """Reference-style loop (loss.backward, clip_grad_norm_, torch AdamW, linear schedule) over the icap model with
    GPT-2 UNfrozen: the custom autograd backward supplies every grad (incl. tied wte, wpe)."""
    g = load("tiny")
    ids, mask, labels, emb = inputs(g, dev)
    model = build(TINY_G, TINY_M, torch.float32, dev, freeze=False)
    n = len(g["unfrozen_losses"])
    opt = torch.optim.AdamW(model.parameters(), lr=1e-4, weight_decay=0.01)
    sched = torch.optim.lr_scheduler.LambdaLR(opt, lambda s: O.linear_schedule(s, 0, n))
    model.train()
    for p in model.modules():
        if hasattr(p, "dropout_p"):
            p.dropout_p = 0.0
    model.gpt.config.resid_pdrop = model.gpt.config.embd_pdrop = model.gpt.config.attn_pdrop = 0.0
    losses = []
    for _ in range(n):
        model.eval()  # dropout off (goldens are dropout-free); eval() does not stop autograd
        out = model(ids, emb, mask, labels)
        out.loss.backward()
        torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=1.0)
        opt.step()
        sched.step()
        opt.zero_grad()
        losses.append(out.loss.item())
    assert rel(losses, g["unfrozen_losses"]) < 1e-5
    for k, v in model.gpt.state_dict().items():
        if k == "lm_head.weight":
            continue
        ck = g["unfrozen_ck.gpt." + k]
        t = v.detach().double()
        assert rel(torch.tensor([t.sum().item(), t.abs().sum().item()]), torch.tensor(ck[:2])) < 1e-4, k


def _check_gpt_checksums(model, g, tol):
    for k, v in model.gpt.state_dict().items():
        if k == "lm_head.weight":  # tied to transformer.wte.weight
            continue
        t = v.detach().double()
        ck = g["unfrozen_ck.gpt." + k]
        assert rel(torch.tensor([t.sum().item(), t.abs().sum().item()]), torch.tensor(ck[:2])) < tol, k


@pytest.mark.parametrize("graph", [False, True])
def test_tiny_fused_train_unfrozen_matches_reference(dev, graph):
    """freeze_gpt_weights=False through the fused trainer (src/train.py:94-96,150-153: AdamW over all parameters)
    vs the reference train() golden: every GPT-2 tensor (tied wte, wpe, LayerNorms, biases) after the steps."""
    g = load("tiny")
    model = build(TINY_G, TINY_M, torch.float32, dev, freeze=False)
    n = len(g["unfrozen_losses"])
    losses, t = _trainer_steps(model, inputs(g, dev), n, graph=graph)
    assert t.gpt_trainable
    assert rel(losses, g["unfrozen_losses"]) < 1e-5
    _check_gpt_checksums(model, g, 1e-4)
    # the trainer's refreshed GPT-2 copies and the masters the inference path rebuilds from agree: one more
    # forward/backward in the trainer gives the model's own forward loss at the trained weights
    ids, mask, labels, emb = inputs(g, dev)
    t._fwd_bwd(True, 1.0)
    with torch.no_grad():
        out = model.eval()(ids, emb, mask, labels)
    assert abs(t.last_loss.item() - out.loss.item()) < 1e-5


@pytest.fixture(scope="module")
def small_f32(dev):
    return build(O.GPT2Cfg(), O.MapperCfg(), torch.float32, dev)


def test_small_forward_f32(dev, small_f32):
    g = load("small")
    ids, mask, labels, emb = inputs(g, dev)
    model = small_f32.eval()
    with torch.no_grad():
        out = model(ids, emb, mask, labels)
        prefix = model.mapping_network(emb)
    assert rel(prefix, g["prefix"]) < 1e-4
    assert abs(out.loss.item() - g["loss"][0]) < 2e-5
    rows = torch.from_numpy(g["logit_rows"])
    assert rel(out.logits[:2][:, rows], g["logits_sel"]) < 1e-4  # north star: logits within 1e-3 rel
    lse = torch.logsumexp(out.logits.double(), -1).cpu().numpy()
    assert np.abs(lse - g["lse"]).max() < 1e-4


def test_small_greedy_exact_f32(dev, small_f32):
    g = load("small")
    emb = torch.from_numpy(g["emb"]).to(dev)[: g["greedy"].shape[0]]
    gen = small_f32.generate(emb, max_length=g["greedy"].shape[1], temperature=0.0)
    assert np.array_equal(gen.cpu().numpy(), g["greedy"])  # token-id exact


def test_small_forward_bf16(dev):
    g = load("small")
    ids, mask, labels, emb = inputs(g, dev)
    model = build(O.GPT2Cfg(), O.MapperCfg(), torch.bfloat16, dev).eval()
    with torch.no_grad():
        out = model(ids, emb, mask, labels)
    assert abs(out.loss.item() - g["loss"][0]) < 3e-2
    rows = torch.from_numpy(g["logit_rows"])
    assert rel(out.logits[:2][:, rows], g["logits_sel"]) < 5e-2
    agree = (out.logits.argmax(-1).cpu().numpy() == g["argmax"]).mean()
    assert agree >= 0.9


def test_small_fused_train_f32(dev):
    g = load("small")
    batch = inputs(g, dev)
    model = build(O.GPT2Cfg(), O.MapperCfg(), torch.float32, dev)
    n = len(g["train_losses"])
    losses, _ = _trainer_steps(model, batch, n)
    assert rel(losses, g["train_losses"]) < 1e-5
    for k, v in model.mapping_network.state_dict().items():
        t = v.detach().double()
        ck = g["trained_ck." + k]
        assert rel(torch.tensor([t.sum().item(), t.abs().sum().item()]), torch.tensor(ck[:2])) < 1e-4, k


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_clip_b32(dev, dtype):
    g = load("clip_b32")
    tower = CLIPVisionTower()
    tower.load_state_dict(O.clip_vision_state_dict(O.ClipCfg(), 0))
    tower = tower.to(dev)
    px = torch.randn((2, 3, 224, 224), generator=torch.Generator().manual_seed(int(g["pixels_seed"][0]))).to(dev)
    f = tower.get_image_features(px, compute_dtype=dtype)
    e = tower.embed(px, compute_dtype=dtype)
    if dtype == torch.float32:
        assert rel(f, g["features"]) < 1e-4
        assert rel(e, g["embeddings"]) < 1e-4
    else:
        cos = torch.nn.functional.cosine_similarity(e.cpu().double(), torch.from_numpy(g["embeddings"]).double())
        assert cos.min() > 0.995


def test_bf16_train_with_clip_dropout_decreases(dev):
    """The benchmarked configuration at small batch: CLIP fwd on pixels + dropout + bf16; loss falls."""
    B = 16
    torch.manual_seed(0)
    gpt = GPT2LMHeadModel.random_init()
    mapper = TransformerMappingNetwork.random_init()
    model = ImageCaptioningModel(mapper, tokenizer=SimpleNamespace(eos_token_id=50256), gpt=gpt,
                                 compute_dtype=torch.bfloat16).to(dev)
    tower = CLIPVisionTower.random_init().to(dev)
    t = CaptionTrainer(model, B, 50, lr=1e-3, num_training_steps=100, clip_model=tower)
    ids, mask, labels, _ = O.synthetic_batch(B, 50, 13, seed=3)
    px = torch.randn((B, 3, 224, 224), generator=torch.Generator().manual_seed(4))
    t.load_batch(ids.to(dev), mask.to(dev), labels.to(dev), pixels=px.to(dev))
    losses = []
    for _ in range(8):
        t.micro_step(use_graph=True)
        losses.append(t.last_loss.item())
    assert all(np.isfinite(losses))
    assert losses[-1] < losses[0] - 0.5, losses


@pytest.mark.parametrize("dropout", [False, True])
def test_compact_head_equals_full_head(dev, dropout):
    """The trainer's LM head over the target rows only (compact_head, the default) gives the loss and parameter
    updates of the full 65-row head: the skipped rows have label -100 and contribute exactly nothing. (Packed
    token rows off here: with dropout on, packing draws the masks by packed row; tests/test_pack_gpu.py checks
    packing against the padded layout with dropout off.)"""
    g = load("tiny")
    batch = inputs(g, dev)
    ids, mask, labels, emb = batch
    res = []
    for compact in (True, False):
        model = build(TINY_G, TINY_M, torch.float32, dev)
        t = CaptionTrainer(model, ids.shape[0], ids.shape[1], lr=1e-3, num_training_steps=4, dropout=dropout,
                           compact_head=compact, pack_rows=False, seed=5)
        t.load_batch(ids, mask, labels, emb)
        losses = []
        for _ in range(3):
            t.micro_step()
            losses.append(t.last_loss.item())
        res.append((losses, {k: v.detach().clone() for k, v in model.mapping_network.state_dict().items()}))
    assert np.allclose(res[0][0], res[1][0], rtol=1e-6, atol=0), (res[0][0], res[1][0])
    for k in res[0][1]:
        assert torch.allclose(res[0][1][k], res[1][1][k], rtol=1e-6, atol=1e-9), k

