"""BASELINE configs[4] end to end on the device: seeded 224x224 pixels -> DINOv3 ViT-L/16 backbone (frozen, 201
tokens: CLS + 4 registers + 196 patches, RoPE, LayerScale) -> transformer mapper 1024 -> gpt_dim 1280 (heads of 160,
trained) -> GPT-2 large (36 layers, d 1280, frozen) fwd + dX bwd, LM head + CE, clip + AdamW: the fused trainer with
`clip_model=DINOv3ImageTower` (no precomputed embeddings), against the oracle's restatement of src/train.py:119-166
with the backbone in front (src/embeddings/dino.py:138-185: encode_image, then the L2 normalisation of :177-179).

The dino.txt vision head that the reference's encode_image adds on top of the backbone has neither code nor weights
offline, so the image embedding here is the backbone's pooled CLS on both sides: that head is
parity unpinned. The oracle pieces are each pinned to goldens (tests/test_oracle.py: DINOv3 vs HF DINOv3ViTModel,
GPT-2 large + mapper 1280 vs the reference's train()); here they run chained on the CPU for the same seeded batch.

Tolerances: fp32 parity mode — losses rel <= 1e-5, trained mapper checksums (sum, sum |.|) rel <= 1e-4.
bf16 perf mode — step-1 loss |d| <= 5e-2 vs the fp32 oracle (the forward at identical weights, 24 + 36 layers of
bf16 rounding). MX fp8 (gpt_fp8=True: every frozen GPT-2 product block-scaled e4m3) — step-1 loss |d| <= 5e-2 vs the
fp32 oracle; step 2 and the mapper update against the bf16 trainer on the same batch (the benchmarked precision; bf16
itself drifts from fp32 after one AdamW update, as tests/test_fp8_gpu.py::test_large_train_fp8 records): loss
|d| <= 5e-2, update cosine >= 0.8."""

import pytest
import torch

from icap import CaptionTrainer
from icap.dino import DINOv3ImageTower
from oracle import icap_oracle as O
from test_model_gpu import build, rel

pytestmark = pytest.mark.gpu

LRG_G = O.GPT2Cfg(n_layer=36, n_embd=1280, n_head=20)
LRG_M = O.MapperCfg(embed_dim=1024, gpt_dim=1280)
L16 = O.DinoCfg()
B, STEPS = 2, 2


@pytest.fixture(scope="module")
def batch():
    ids, mask, labels, _ = O.synthetic_batch(B, 50, 13, seed=41)
    px = torch.randn((B, 3, 224, 224), generator=torch.Generator().manual_seed(42))
    return ids, mask, labels, px


@pytest.fixture(scope="module")
def oracle_run(batch):
    """(losses, trained mapper state) of the oracle: DINOv3 embed -> mapper -> GPT-2 large, 2 AdamW steps."""
    torch.set_num_threads(16)
    losses, _, map_sd, _ = O.train_steps(O.gpt2_state_dict(LRG_G, 0), LRG_G, O.mapper_state_dict(LRG_M, 0), LRG_M,
                                         [batch] * STEPS, total_steps=STEPS, clip=(O.dinov3_state_dict(L16, 0), L16))
    return losses, map_sd


def _run(dev, dtype, batch, fp8=False):
    model = build(LRG_G, LRG_M, dtype, dev)
    if fp8:
        model.gpt.fp8_mx = True
    tower = DINOv3ImageTower()
    tower.load_state_dict(O.dinov3_state_dict(L16, 0), strict=True)
    tower = tower.to(dev)
    t = CaptionTrainer(model, B, 50, lr=1e-4, num_training_steps=STEPS, dropout=False, clip_model=tower)
    ids, mask, labels, px = (x.to(dev) for x in batch)
    t.load_batch(ids, mask, labels, pixels=px)
    init = {k: v.detach().clone() for k, v in model.mapping_network.state_dict().items()}
    losses = []
    for _ in range(STEPS):
        t.micro_step()
        losses.append(t.last_loss.item())
    upd = torch.cat([(v.detach() - init[k]).double().reshape(-1).cpu()
                     for k, v in model.mapping_network.state_dict().items()])
    if fp8:
        assert model.gpt.core(torch.bfloat16).fp8
    return model, losses, upd


def test_configs4_pixels_train_f32(dev, batch, oracle_run):
    ref_losses, ref_sd = oracle_run
    model, losses, _ = _run(dev, torch.float32, batch)
    assert rel(losses, ref_losses) < 1e-5, (losses, ref_losses)
    for k, v in model.mapping_network.state_dict().items():
        t, r = v.detach().double().cpu(), ref_sd[k].double()
        assert rel(torch.tensor([t.sum().item(), t.abs().sum().item()]),
                   torch.tensor([r.sum().item(), r.abs().sum().item()])) < 1e-4, k


def test_configs4_pixels_train_bf16_fp8(dev, batch, oracle_run):
    ref_losses, _ = oracle_run
    _, lb, ub = _run(dev, torch.bfloat16, batch)
    _, l8, u8 = _run(dev, torch.bfloat16, batch, fp8=True)
    cos = float(torch.nn.functional.cosine_similarity(u8, ub, dim=0))
    print(f"configs[4] pixels: bf16 losses {lb}, fp8 losses {l8}, reference {ref_losses}; fp8 update cosine vs "
          f"bf16 {cos:.4f}")
    assert abs(lb[0] - ref_losses[0]) < 5e-2, (lb, ref_losses)
    assert abs(l8[0] - ref_losses[0]) < 5e-2, (l8, ref_losses)
    assert abs(l8[1] - lb[1]) < 5e-2, (l8, lb)
    assert cos >= 0.8, cos
