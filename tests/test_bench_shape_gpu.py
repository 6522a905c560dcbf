"""The benchmarked shape pinned to the reference: tests/golden/bench128.npz is the
reference's own B = 128 step (tools/make_goldens.py golden_bench128): HF CLIP ViT-B/32 features of seeded 224x224
pixels -> the reference's ImageCaptioningModel (GPT-2 small frozen + transformer mapper, S = 65) -> 2 src/train.py
steps. Here the fused trainer runs exactly as bench.py does (CLIP forward from pixels inside the step, compact LM
head, split-K / tile-kernel choices of M = 8320, first step eager, second a HIP-graph replay), dropout off.

fp32 parity mode: CLIP embeddings max-rel <= 1e-4, losses rel <= 1e-5, every mapper tensor's (sum, |sum|) rel <= 1e-4.
bf16 (the benchmarked precision): loss |d| <= 3e-2 per step; the mapper update (param - init; small tensors whole,
large ones every 997th element) per tensor: cosine >= COS_MIN and |u - u_ref| / |u_ref| <= REL_MAX, values measured
at this shape and written below."""

import os

import numpy as np
import pytest
import torch

from icap import CaptionTrainer
from icap.clip import CLIPVisionTower
from oracle import icap_oracle as O
from test_model_gpu import build, load, rel

pytestmark = pytest.mark.gpu
B = 128


def _run(dtype, dev):
    g = load("bench128")
    model = build(O.GPT2Cfg(), O.MapperCfg(), dtype, dev)
    tower = CLIPVisionTower.random_init(seed=0).to(dev)
    ref_sd = O.clip_vision_state_dict(O.ClipCfg(), 0)
    sd = tower.state_dict()
    assert all(torch.equal(sd[k].cpu(), v) for k, v in ref_sd.items() if k in sd)
    ids, mask, labels, _ = O.synthetic_batch(B, 50, 13, seed=int(g["batch_seed"][0]))
    px = torch.randn((B, 3, 224, 224), generator=torch.Generator().manual_seed(int(g["pixels_seed"][0])))
    init = {k: v.detach().clone() for k, v in model.mapping_network.state_dict().items()}
    t = CaptionTrainer(model, B, 50, lr=1e-4, num_training_steps=2, dropout=False, clip_model=tower)
    assert t.gws.compact  # the benchmark's compact LM head
    t.load_batch(ids.to(dev), mask.to(dev), labels.to(dev), pixels=px.to(dev))
    losses = []
    for _ in range(2):
        t.micro_step(use_graph=True)  # eager, then a captured-graph replay (bench.py's timed form)
        losses.append(t.last_loss.item())
    emb = t.emb_c.float()
    return g, model, init, losses, emb


def test_bench_shape_fp32_parity(dev):
    g, model, _, losses, emb = _run(torch.float32, dev)
    assert rel(emb, g["emb"]) < 1e-4
    assert rel(losses, g["train_losses"]) < 1e-5, (losses, g["train_losses"])
    for k, v in model.mapping_network.state_dict().items():
        t = v.detach().double()
        assert rel(torch.tensor([t.sum().item(), t.abs().sum().item()]), torch.tensor(g["trained_ck." + k][:2])) < 1e-4, k


# measured at this shape (r03, profiles/r03_bench128_bf16_update_stats.txt): overall cosine 0.891, per tensor min 0.805
# and max relative norm 0.672 (both the layer-0 in_proj_bias: AdamW's per-element normalisation makes near-zero
# bias gradients take full-size steps whose sign bf16 rounding can flip); loss |d| 8e-5 / 4.3e-3
COS_MIN, REL_MAX, COS_ALL_MIN = 0.78, 0.72, 0.87  # measured at this shape: see the printed line in the GPU log


def test_bench_shape_bf16_bounds(dev):
    g, model, init, losses, emb = _run(torch.bfloat16, dev)
    dl = [abs(a - b) for a, b in zip(losses, g["train_losses"])]
    cos_t, rel_t, ua, ra = {}, {}, [], []
    for k, v in model.mapping_network.state_dict().items():
        step = 1 if v.numel() <= 20000 else 997  # the golden keeps small tensors whole, every 997th element else
        u = (v.detach().double().reshape(-1)[::step] - init[k].double().reshape(-1)[::step]).cpu()
        r = torch.from_numpy(g["trained_sample." + k]).double() - init[k].double().reshape(-1)[::step].cpu()
        if r.norm() == 0:
            continue
        cos_t[k] = float(torch.nn.functional.cosine_similarity(u, r, dim=0))
        rel_t[k] = float((u - r).norm() / r.norm())
        ua.append(u)
        ra.append(r)
    cos_all = float(torch.nn.functional.cosine_similarity(torch.cat(ua), torch.cat(ra), dim=0))
    kmin = min(cos_t, key=cos_t.get)
    kmax = max(rel_t, key=rel_t.get)
    print(f"bench128 bf16: loss |d| {dl}, update cosine all {cos_all:.4f}, min {cos_t[kmin]:.4f} ({kmin}), "
          f"max rel {rel_t[kmax]:.4f} ({kmax})")
    print("bench128 bf16 worst cosines:", sorted((round(c, 4), k) for k, c in cos_t.items())[:6])
    print("bench128 bf16 worst rel:", sorted(((round(r, 4), k) for k, r in rel_t.items()), reverse=True)[:6])
    assert max(dl) < 3e-2
    assert cos_all >= COS_ALL_MIN and min(cos_t.values()) >= COS_MIN and max(rel_t.values()) <= REL_MAX
