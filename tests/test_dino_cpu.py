"""DINOv3 ViT-L/16 tower (BASELINE configs[4]; src/embeddings/dino.py) — CPU side: the oracle restatement pinned to
the golden produced by HF DINOv3ViTModel (tools/make_goldens.py golden_dinov3; the reference's own torch.hub model
is gated and offline), the product tower's weights / key layout, its RoPE tables, the kernel schedule's bounds (dry
run) and the reference's FileNotFoundError rule."""

import os

import numpy as np
import pytest
import torch

from oracle import icap_oracle as O

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_oracle_dinov3_matches_hf_golden():
    g = dict(np.load(os.path.join(GOLD, "dinov3_l16.npz")))
    px = torch.randn((2, 3, 224, 224), generator=torch.Generator().manual_seed(int(g["pixels_seed"][0])))
    cfg = O.DinoCfg()
    sd = O.dinov3_state_dict(cfg, 0)
    out = O.dinov3_forward(sd, cfg, px)
    assert float((out[:, 0] - torch.from_numpy(g["pooler"])).abs().max()) < 2e-5
    assert float((out[:, 5:].mean(1) - torch.from_numpy(g["patch_mean"])).abs().max()) < 2e-5
    assert float((out[:, 1:5] - torch.from_numpy(g["registers"])).abs().max()) < 2e-5
    e = O.dinov3_embed_normalized(sd, cfg, px)
    assert float((e - torch.from_numpy(g["embeddings"])).abs().max()) < 2e-6


def test_product_tower_weights_key_layout_and_rope():
    from icap.dino import DINOv3ImageTower, DinoConfig, rope_tables

    t = DINOv3ImageTower.random_init(seed=0)
    ref = O.dinov3_state_dict(O.DinoCfg(), 0)
    sd = t.state_dict()
    assert set(sd) == set(ref)  # HF DINOv3ViTModel key names
    for k, v in ref.items():
        assert torch.equal(sd[k], v), k
    c, s = rope_tables(DinoConfig(), 14, 14)
    oc, os_ = O.dinov3_rope_tables(O.DinoCfg(), 14, 14)
    assert c.shape == (196, 64) and torch.equal(c, oc) and torch.equal(s, os_)
    pre = {"backbone." + k: v for k, v in ref.items()}
    t2 = DINOv3ImageTower()
    t2.load_backbone_state_dict(pre)
    assert torch.equal(t2.state_dict()["norm.weight"], ref["norm.weight"])


def test_dino_schedule_in_bounds():
    import icap.weights
    from dryrun import dry_run
    from icap.dino import DINOv3ImageTower, DinoConfig

    with dry_run() as rec:
        icap.weights.ops.call = rec
        t = DINOv3ImageTower(DinoConfig(num_hidden_layers=3))
        for dt in (torch.float32, torch.bfloat16):
            t.core(dt).features(torch.randn(3, 3, 224, 224))
        bad = rec.check()
        names = [c[0] for c in rec.calls]
    assert not bad, bad[:10]
    assert names.count("icap_rope_patches") == 2 * 3 and names.count("icap_prefix_embed") == 2


def test_load_dinov3_models_requires_both_files(tmp_path):
    from icap.dino import load_dinov3_models

    with pytest.raises(FileNotFoundError):
        load_dinov3_models(str(tmp_path), device=torch.device("cpu"))


def test_processor_geometry():
    from icap.dino import get_dinov3_preprocessor

    img = (np.arange(300 * 400 * 3) % 251).astype(np.uint8).reshape(300, 400, 3)
    px = get_dinov3_preprocessor()(images=[img, img[:, :300]]).pixel_values
    assert px.shape == (2, 3, 224, 224) and px.dtype == torch.float32
    assert torch.isfinite(px).all()
