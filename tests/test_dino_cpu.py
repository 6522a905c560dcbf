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
    # fp32: im2col + GEMM + icap_prefix_embed; bf16: one icap_patch_embed (the GEMM gathers the pixels itself)
    assert names.count("icap_rope_patches") == 2 * 3 and names.count("icap_prefix_embed") == 1
    assert names.count("icap_patch_embed") == 1 and names.count("icap_im2col_patches") == 1


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


def _to_meta(sd, D):
    """HF DINOv3ViTModel keys -> Meta's native DINOv3 checkpoint layout (what BACKBONE_WEIGHTS_FILE holds): the
    inverse of icap.dino.meta_to_hf_state_dict, written out key by key from the Meta module names."""
    out = {"cls_token": sd["embeddings.cls_token"].clone(), "mask_token": sd["embeddings.mask_token"].reshape(1, D),
           "storage_tokens": sd["embeddings.register_tokens"].clone(),
           "patch_embed.proj.weight": sd["embeddings.patch_embeddings.weight"],
           "patch_embed.proj.bias": sd["embeddings.patch_embeddings.bias"],
           "norm.weight": sd["norm.weight"], "norm.bias": sd["norm.bias"]}
    i = 0
    while f"model.layer.{i}.norm1.weight" in sd:
        p, b = f"model.layer.{i}.", f"blocks.{i}."
        a = p + "attention."
        out[b + "attn.qkv.weight"] = torch.cat([sd[a + "q_proj.weight"], sd[a + "k_proj.weight"],
                                                sd[a + "v_proj.weight"]], 0)
        # Meta stores a (masked) key bias: garbage there must not leak into the model
        out[b + "attn.qkv.bias"] = torch.cat([sd[a + "q_proj.bias"], torch.full((D,), 123.0), sd[a + "v_proj.bias"]])
        out[b + "attn.qkv.bias_mask"] = torch.cat([torch.ones(D), torch.zeros(D), torch.ones(D)])
        out[b + "attn.proj.weight"], out[b + "attn.proj.bias"] = sd[a + "o_proj.weight"], sd[a + "o_proj.bias"]
        out[b + "ls1.gamma"], out[b + "ls2.gamma"] = sd[p + "layer_scale1.lambda1"], sd[p + "layer_scale2.lambda1"]
        out[b + "mlp.fc1.weight"], out[b + "mlp.fc1.bias"] = sd[p + "mlp.up_proj.weight"], sd[p + "mlp.up_proj.bias"]
        out[b + "mlp.fc2.weight"], out[b + "mlp.fc2.bias"] = sd[p + "mlp.down_proj.weight"], sd[p + "mlp.down_proj.bias"]
        for nm in ("norm1", "norm2"):
            out[b + nm + ".weight"], out[b + nm + ".bias"] = sd[p + nm + ".weight"], sd[p + nm + ".bias"]
        i += 1
    return out


def test_meta_checkpoint_layout_loads_into_hf_layout():
    """BACKBONE_WEIGHTS_FILE ships in Meta's key layout; load_backbone_state_dict converts it (qkv split,
    masked key bias dropped, LayerScale / MLP / patch-embed renames, periods checked and dropped). The converted
    weights equal the HF-layout ones and the oracle forward over them is the same function."""
    from icap.dino import DINOv3ImageTower, DinoConfig, is_meta_layout

    cfg = DinoConfig(num_hidden_layers=2, image_size=64)
    t = DINOv3ImageTower.random_init(cfg, seed=3)
    hf = {k: v.clone() for k, v in t.state_dict().items()}
    meta = _to_meta(hf, cfg.hidden_size)
    hd = cfg.hidden_size // cfg.num_attention_heads
    meta["rope_embed.periods"] = cfg.rope_theta ** torch.arange(0, 1, 4 / hd, dtype=torch.float32)
    assert is_meta_layout(meta) and not is_meta_layout(hf)
    t2 = DINOv3ImageTower(cfg)
    t2.load_backbone_state_dict({"backbone." + k: v for k, v in meta.items()})
    got = t2.state_dict()
    assert set(got) == set(hf)
    for k, v in hf.items():
        assert torch.equal(got[k], v), k
    ocfg = O.DinoCfg(layers=2, image=64)
    px = torch.randn((2, 3, 64, 64), generator=torch.Generator().manual_seed(0))
    assert torch.equal(O.dinov3_forward(got, ocfg, px), O.dinov3_forward(hf, ocfg, px))
    bad = dict(meta)
    bad["rope_embed.periods"] = bad["rope_embed.periods"] * 2
    with pytest.raises(ValueError):
        DINOv3ImageTower(cfg).load_backbone_state_dict(bad)
    unknown = dict(meta)
    unknown["blocks.0.attn.extra"] = torch.zeros(1)
    with pytest.raises(RuntimeError):
        DINOv3ImageTower(cfg).load_backbone_state_dict(unknown)
