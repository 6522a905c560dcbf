"""BASELINE configs[3] end to end on the device: seeded 224x224 pixels -> CLIP ViT-L/14 (frozen, 257 tokens) ->
transformer mapper at gpt_dim 1024 (head dim 128, trained) -> GPT-2 medium (24 layers, d 1024, frozen) fwd + dX bwd,
LM head + CE, clip + AdamW — the fused trainer with `clip_model=` (no precomputed embeddings), against the oracle's
restatement of src/train.py:119-166 with the CLIP tower in front (src/embeddings/clip.py:10-12 model_name, :132-137
get_image_features + L2 normalisation).

The oracle pieces are each pinned to reference goldens (tests/test_oracle.py: GPT-2 medium, mapper 1024, CLIP
ViT-L/14); here they run chained, on the CPU, for the same seeded batch.

Tolerances: fp32 parity mode — losses rel <= 1e-5, trained mapper checksums (sum, sum |.|) rel <= 1e-4;
bf16 perf mode — first step loss |d| <= 5e-2 (the forward at identical weights: 24 layers of bf16 rounding, as
test_parity_gpu's medium forward); second step |d| <= 0.15 (after one AdamW update from bf16 gradients: AdamW
normalises each element, so bf16 noise on near-zero gradients becomes full-size steps; measured 0.076 against the
reference's 1.43 loss drop); the mapper's update direction (param - init) cosine over all tensors >= 0.75
(measured 0.807)."""

import pytest
import torch

from icap import CaptionTrainer
from icap.clip import CLIPVisionConfig, CLIPVisionTower
from oracle import icap_oracle as O
from test_model_gpu import build, rel

pytestmark = pytest.mark.gpu

MED_G = O.GPT2Cfg(n_layer=24, n_embd=1024, n_head=16)
MED_M = O.MapperCfg(embed_dim=768, gpt_dim=1024)
L14 = O.ClipCfg(hidden=1024, layers=24, heads=16, patch=14, image=224, inter=4096, proj=768)
B, STEPS = 2, 2


@pytest.fixture(scope="module")
def batch():
    ids, mask, labels, _ = O.synthetic_batch(B, 50, 13, seed=31)
    px = torch.randn((B, 3, 224, 224), generator=torch.Generator().manual_seed(32))
    return ids, mask, labels, px


@pytest.fixture(scope="module")
def oracle_run(batch):
    """(losses, trained mapper state) of the oracle: CLIP-L/14 embed -> mapper -> GPT-2 medium, 2 AdamW steps."""
    torch.set_num_threads(16)
    losses, _, map_sd, _ = O.train_steps(O.gpt2_state_dict(MED_G, 0), MED_G, O.mapper_state_dict(MED_M, 0), MED_M,
                                         [batch] * STEPS, total_steps=STEPS,
                                         clip=(O.clip_vision_state_dict(L14, 0), L14))
    return losses, map_sd


def _run(dev, dtype, batch):
    model = build(MED_G, MED_M, dtype, dev)
    tower = CLIPVisionTower(CLIPVisionConfig.vit_l14())
    tower.load_state_dict(O.clip_vision_state_dict(L14, 0))
    tower = tower.to(dev)
    t = CaptionTrainer(model, B, 50, lr=1e-4, num_training_steps=STEPS, dropout=False, clip_model=tower)
    ids, mask, labels, px = (x.to(dev) for x in batch)
    t.load_batch(ids, mask, labels, pixels=px)
    losses = []
    for _ in range(STEPS):
        t.micro_step()
        losses.append(t.last_loss.item())
    return model, losses


def test_configs3_pixels_train_f32(dev, batch, oracle_run):
    ref_losses, ref_sd = oracle_run
    model, losses = _run(dev, torch.float32, batch)
    assert rel(losses, ref_losses) < 1e-5, (losses, ref_losses)
    for k, v in model.mapping_network.state_dict().items():
        t, r = v.detach().double().cpu(), ref_sd[k].double()
        assert rel(torch.tensor([t.sum().item(), t.abs().sum().item()]),
                   torch.tensor([r.sum().item(), r.abs().sum().item()])) < 1e-4, k


def test_configs3_pixels_train_bf16(dev, batch, oracle_run):
    ref_losses, ref_sd = oracle_run
    model, losses = _run(dev, torch.bfloat16, batch)
    init = O.mapper_state_dict(MED_M, 0)
    num = den_a = den_b = 0.0
    for k, v in model.mapping_network.state_dict().items():
        du = (v.detach().double().cpu() - init[k].double()).flatten()
        dr = (ref_sd[k].double() - init[k].double()).flatten()
        num += float(du @ dr)
        den_a += float(du @ du)
        den_b += float(dr @ dr)
    cos = num / max((den_a * den_b) ** 0.5, 1e-30)
    print(f"configs[3] bf16: losses {losses} vs reference {ref_losses}; update cosine {cos:.4f}")
    assert abs(losses[0] - ref_losses[0]) < 5e-2, (losses, ref_losses)
    assert abs(losses[1] - ref_losses[1]) < 0.15, (losses, ref_losses)
    assert cos >= 0.75, cos
