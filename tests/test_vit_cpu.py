"""ViT-B/16 image tower (src/embeddings/vit.py) — CPU side: the oracle restatement pinned to
the golden produced by HF ViTModel (tools/make_goldens.py golden_vit_b16), the product tower's weights / key
layouts, the host ViTImageProcessor against transformers', the kernel schedule's bounds (dry run), and the
extraction loop's .pt format (decode in DataLoader workers, the reference's file order)."""

import os

import numpy as np
import pytest
import torch

from oracle import icap_oracle as O

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_oracle_vit_matches_reference_golden():
    g = dict(np.load(os.path.join(GOLD, "vit_b16.npz")))
    px = torch.randn((2, 3, 224, 224), generator=torch.Generator().manual_seed(int(g["pixels_seed"][0])))
    sd = O.vit_state_dict(O.ViTCfg(), 0)
    pooled = O.vit_pooler_output(sd, O.ViTCfg(), px)
    assert float((pooled - torch.from_numpy(g["pooler"])).abs().max()) < 2e-5
    e = O.vit_embed_normalized(sd, O.ViTCfg(), px)
    assert float((e - torch.from_numpy(g["embeddings"])).abs().max()) < 2e-6


def test_product_tower_weights_and_key_layouts():
    from icap.vit import ViTImageTower

    t = ViTImageTower.random_init(seed=0)
    ref = O.vit_state_dict(O.ViTCfg(), 0)
    sd = t.state_dict()
    assert set(sd) == set(ref)  # transformers 4.57 key names (the reference's pin)
    for k, v in ref.items():
        assert torch.equal(sd[k], v), k
    # a transformers 5.x-layout checkpoint (and the ViTForImageClassification 'vit.' prefix) loads into it
    five = {}
    for k, v in ref.items():
        n = k
        if k.startswith("encoder.layer."):
            i, rest = k[len("encoder.layer."):].split(".", 1)
            rest = (rest.replace("attention.attention.query", "attention.q_proj")
                    .replace("attention.attention.key", "attention.k_proj")
                    .replace("attention.attention.value", "attention.v_proj")
                    .replace("attention.output.dense", "attention.o_proj")
                    .replace("intermediate.dense", "mlp.fc1").replace("output.dense", "mlp.fc2"))
            n = f"layers.{i}.{rest}"
        five["vit." + n] = v * 2
    t2 = ViTImageTower()
    t2.load_hf_state_dict(five)
    for k, v in ref.items():
        assert torch.equal(t2.state_dict()[k], v * 2), k


def test_host_processor_matches_transformers():
    from transformers import ViTImageProcessor as HFProc
    from PIL import Image

    from icap.vit import ViTImageProcessor

    rng = np.random.default_rng(0)
    ims = [Image.fromarray(rng.integers(0, 256, (h, w, 3), dtype=np.uint8)) for h, w in ((480, 640), (224, 224),
                                                                                        (300, 199))]
    ours = ViTImageProcessor()(ims).pixel_values
    ref = HFProc()(images=ims, return_tensors="pt").pixel_values
    assert ours.shape == ref.shape == (3, 3, 224, 224)
    assert float((ours - ref).abs().max()) < 1e-5
    arr = ViTImageProcessor()([np.asarray(im) for im in ims]).pixel_values  # uint8 arrays from the loader
    assert torch.equal(arr, ours)


def test_vit_schedule_in_bounds():
    import icap.weights
    from dryrun import dry_run
    from icap.vit import ViTConfig, ViTImageTower

    with dry_run() as rec:
        icap.weights.ops.call = rec
        t = ViTImageTower(ViTConfig())
        for dt in (torch.float32, torch.bfloat16):
            t.core(dt).features(torch.randn(3, 3, 224, 224))
        bad = rec.check()
        names = [c[0] for c in rec.calls]
    assert not bad, bad[:10]
    assert names.count("icap_attention_fwd") == 2 * 12


def _fake_embed(px):
    return px.float().mean(dim=(2, 3)).repeat(1, 4)[:, :8]  # deterministic per image, shape [B, 8]


def test_extract_directory_format_and_order(tmp_path):
    from PIL import Image

    from icap.images import extract_directory
    from icap.vit import ViTImageProcessor

    d = tmp_path / "imgs"
    d.mkdir()
    rng = np.random.default_rng(1)
    for i in range(7):
        Image.fromarray(rng.integers(0, 256, (64 + 8 * i, 80, 3), dtype=np.uint8)).save(d / f"COCO_{i:012d}.jpg")
    (d / "notes.txt").write_text("not an image")
    out = tmp_path / "emb.pt"
    n = extract_directory(str(d), str(out), _fake_embed, ViTImageProcessor(), 8, batch_size=3, num_workers=2)
    assert n == 7
    data = torch.load(str(out), weights_only=True)
    listed = [f for f in os.listdir(d) if f.endswith(".jpg")]  # src/utils.py:131-135 order
    assert data["filenames"] == listed
    assert data["embeddings"].shape == (7, 8) and data["embeddings"].dtype == torch.float32
    single = torch.cat([_fake_embed(ViTImageProcessor()([Image.open(d / f)]).pixel_values) for f in listed])
    assert torch.allclose(data["embeddings"], single)
    # the dataset file the reference's CocoDataset reads (src/dataset.py:127-137) loads these rows back
    from icap.dataset import CocoDataset

    assert [CocoDataset.get_image_id_from_filename(f) for f in data["filenames"]] == [int(f[5:17]) for f in listed]
