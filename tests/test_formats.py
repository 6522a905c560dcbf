"""On-disk formats shared with the reference: checkpoint files of
save_parameters / load_saved_parameters (src/models.py:489-547), the extraction .pt read by CocoDataset
(src/embeddings/clip.py:147-149 <-> src/dataset.py:127-137) and the evaluation JSON files (src/eval.py:366-386).

The reference's key sets come from its own save_parameters() output (tools/make_goldens.py golden_ckpt_keys ->
tests/golden/ckpt_keys.json: 99 keys for the transformer mapper with GPT-2 frozen, 247 unfrozen, 4 for the MLP
mapper). CPU only: the modules are parameter storage, nothing here runs a kernel."""

import json
import os
from types import SimpleNamespace

import pytest
import torch

from icap import GPT2Config, GPT2LMHeadModel, ImageCaptioningModel, MLPMappingNetwork, TransformerMappingNetwork
from oracle import icap_oracle as O

GOLD = os.path.join(os.path.dirname(__file__), "golden", "ckpt_keys.json")


def _model(tag):
    mc = O.MapperCfg()
    if tag.startswith("mlp"):
        m = MLPMappingNetwork(O.MLPMapperCfg().prefix_length, O.MLPMapperCfg().embed_dim, O.MLPMapperCfg().gpt_dim)
    else:
        m = TransformerMappingNetwork(mc.embed_dim, mc.gpt_dim, mc.prefix_length, mc.hidden_length, mc.num_layers)
    torch.manual_seed(0)
    with torch.no_grad():
        for p in m.parameters():
            p.copy_(torch.randn_like(p) * 0.02)
    return ImageCaptioningModel(m, tokenizer=SimpleNamespace(eos_token_id=50256), gpt=GPT2LMHeadModel(GPT2Config()),
                                freeze_gpt_weights=not tag.endswith("unfrozen"))


@pytest.fixture(scope="module")
def ref_keys():
    with open(GOLD) as f:
        return json.load(f)


@pytest.mark.parametrize("tag", ["transformer_frozen", "transformer_unfrozen", "mlp_frozen"])
def test_save_parameters_matches_reference_key_set(tmp_path, ref_keys, tag):
    model = _model(tag)
    path = tmp_path / "ckpt.pt"
    model.save_parameters(str(path))
    sd = torch.load(str(path), weights_only=True)
    assert {k: list(v.shape) for k, v in sd.items()} == ref_keys[tag]


@pytest.mark.parametrize("tag", ["transformer_frozen", "transformer_unfrozen"])
def test_checkpoint_round_trip_and_reference_files(tmp_path, ref_keys, tag):
    a, b = _model(tag), _model(tag)
    with torch.no_grad():
        for p in b.mapping_network.parameters():
            p.add_(1.0)
    path = str(tmp_path / "a.pt")
    a.save_parameters(path)
    b.load_saved_parameters(path, device=torch.device("cpu"))
    for k, v in a.state_dict().items():
        assert torch.equal(v, b.state_dict()[k]), k
    # a file with exactly the reference's keys and shapes (what its save_parameters writes) loads
    g = torch.Generator().manual_seed(1)
    ref = {k: torch.randn(s, generator=g) for k, s in ref_keys[tag].items()}
    if "gpt.lm_head.weight" in ref:  # tied to wte in both implementations: one tensor under two names
        ref["gpt.lm_head.weight"] = ref["gpt.transformer.wte.weight"]
    torch.save(ref, str(tmp_path / "ref.pt"))
    b.load_saved_parameters(str(tmp_path / "ref.pt"), device=torch.device("cpu"))
    sd = b.state_dict()
    for k, v in ref.items():
        assert torch.equal(sd[k], v), k
    # the reference's error behaviour (src/models.py:535-545)
    torch.save({**ref, "mapping_network.not_a_key": torch.zeros(1)}, str(tmp_path / "extra.pt"))
    with pytest.raises(ValueError, match="Unexpected keys"):
        b.load_saved_parameters(str(tmp_path / "extra.pt"), device=torch.device("cpu"))
    drop = dict(ref)
    drop.pop(next(k for k in ref if k.startswith("mapping_network.")))
    torch.save(drop, str(tmp_path / "missing.pt"))
    with pytest.raises(ValueError, match="Missing keys"):
        b.load_saved_parameters(str(tmp_path / "missing.pt"), device=torch.device("cpu"))


class _Enc(dict):
    __getattr__ = dict.__getitem__


class _Tok:
    """Character-level stand-in with the tokenizer call the dataset makes (src/dataset.py:181-188)."""

    eos_token = "<eos>"
    eos_token_id = 3
    pad_token_id = 3
    padding_side = "right"
    truncation_side = "right"

    def __call__(self, texts, max_length, padding, truncation, return_tensors=None, **_):
        single = isinstance(texts, str)
        rows = [texts] if single else texts
        ids = torch.full((len(rows), max_length), self.pad_token_id, dtype=torch.long)
        mask = torch.zeros((len(rows), max_length), dtype=torch.long)
        for i, t in enumerate(rows):
            body = t[: -len(self.eos_token)] if t.endswith(self.eos_token) else t
            seq = [4 + (ord(c) % 50) for c in body] + ([self.eos_token_id] if t.endswith(self.eos_token) else [])
            seq = seq[:max_length]
            ids[i, : len(seq)] = torch.tensor(seq, dtype=torch.long)
            mask[i, : len(seq)] = 1
        return _Enc(input_ids=ids, attention_mask=mask)


def test_extraction_pt_feeds_coco_dataset(tmp_path):
    """extract_directory's .pt (filenames in os.listdir order + fp32 [N, D] embeddings) is the file CocoDataset
    reads: every caption item carries its image's row and id."""
    from PIL import Image

    from icap.dataset import CocoDataset
    from icap.images import extract_directory
    from icap.vit import ViTImageProcessor

    d = tmp_path / "imgs"
    d.mkdir()
    ids = [391895, 522418, 184613]
    for i, iid in enumerate(ids):
        Image.new("RGB", (40 + 8 * i, 32), color=(10 * i, 100, 200)).save(d / f"COCO_val2014_{iid:012d}.jpg")
    emb_path = tmp_path / "emb.pt"
    n = extract_directory(str(d), str(emb_path), lambda px: px.float().mean(dim=(2, 3)).repeat(1, 3)[:, :8],
                          ViTImageProcessor(), 8, batch_size=2, num_workers=0)
    assert n == 3
    ann = {"annotations": [{"image_id": iid, "caption": f"caption {j} of {iid}", "id": j}
                           for j, iid in enumerate(ids * 2)]}
    (tmp_path / "ann.json").write_text(json.dumps(ann))
    for pre in (False, True):
        ds = CocoDataset(str(emb_path), str(tmp_path / "ann.json"), tokenizer=_Tok(), max_length=20, pretokenize=pre)
        data = torch.load(str(emb_path), weights_only=True)
        row = {CocoDataset.get_image_id_from_filename(f): i for i, f in enumerate(data["filenames"])}
        assert len(ds) == 6
        for j in range(len(ds)):
            it = ds[j]
            assert it["image_id"] == ids[j % 3]
            assert torch.equal(it["image_embedding"], data["embeddings"][row[it["image_id"]]])
            assert it["caption_text"] == f"caption {j} of {ids[j % 3]}"


def test_evaluation_json_files_match_reference_layout(tmp_path):
    """evaluate_epoch writes the reference's two files (src/eval.py:366-386): epoch_{e}_{split}_predictions.json
    (a list of {"image_id", "caption"}, one per image) and epoch_{e}_{split}_metrics.json."""
    from icap.evaluate import evaluate_epoch

    items = [{"image_id": iid, "image_embedding": torch.zeros(4)} for iid in (7, 7, 9, 11, 9)]

    class DS(torch.utils.data.Dataset):
        def __len__(self):
            return len(items)

        def __getitem__(self, i):
            return items[i]

    class M:
        device = torch.device("cpu")
        tokenizer = SimpleNamespace(batch_decode=lambda ids, skip_special_tokens: [f"t{int(r[0])}" for r in ids])

        def eval(self):
            return self

        def generate(self, emb, **_):
            return torch.arange(emb.shape[0]).unsqueeze(1) + 100

    m = evaluate_epoch(M(), DS(), None, 3, "val", 2, 0, 50, 0.0, 0.9, torch.device("cpu"), str(tmp_path))
    with open(tmp_path / "epoch_3_val_predictions.json") as f:
        preds = json.load(f)
    assert [p["image_id"] for p in preds] == [7, 9, 11]
    assert all(set(p) == {"image_id", "caption"} and isinstance(p["caption"], str) for p in preds)
    with open(tmp_path / "epoch_3_val_metrics.json") as f:
        meta = json.load(f)
    assert meta["epoch"] == 3 and meta["split"] == "val" and meta["num_images"] == 3
    assert m == {}  # pycocoevalcap absent: no metric keys (present: EvalMetrics.to_dict's six)


def test_val_metrics_summary_written_by_train(tmp_path):
    """src/train.py:229-235 -> src/eval.py:479-491: after training with a validation set, train() writes
    eval_results/val_metrics_summary.json = the list of per-epoch {"epoch", "loss", **metrics} dicts (indent 2),
    the same list it returns as "val_metrics"."""
    import icap
    import icap.weights
    from dryrun import dry_run
    from icap.dataset import SyntheticCaptionDataset
    from test_dryrun_bounds import tiny_model

    ds = SyntheticCaptionDataset(4, max_length=12, real=5, vocab_size=512, eos=511, embed_dim=64)
    ann = tmp_path / "ann.json"
    ann.write_text(json.dumps({"annotations": []}))
    with dry_run() as rec:
        icap.weights.ops.call = rec
        model = tiny_model()
        model.generate = lambda emb, **_: torch.full((emb.shape[0], 3), 7, dtype=torch.int64)
        res = icap.train(ds, model, batch_size=2, num_epochs=2, num_workers=0, device=torch.device("cpu"),
                         outputs_dir=str(tmp_path / "out"), save_every_epoch=5, use_graph=False,
                         val_dataset=ds, val_annotations_path=str(ann))
    path = tmp_path / "out" / "eval_results" / "val_metrics_summary.json"
    with open(path) as f:
        summary = json.load(f)
    assert summary == res["val_metrics"]
    assert [e["epoch"] for e in summary] == [1, 2]
    assert all(set(e) >= {"epoch", "loss"} for e in summary)
    assert path.read_text().startswith("[\n  {")  # json.dump(..., indent=2)
    for e in (1, 2):
        assert (tmp_path / "out" / "eval_results" / f"epoch_{e}_val_predictions.json").exists()


def test_extraction_packed_batches(tmp_path):
    """The device processor's loader path (icap.images: ImageDirectoryDataset.packed_collate in the workers, one
    packed uint8 buffer per batch): with a host stand-in for preprocess_packed, every image arrives byte-exact and in
    the reference's os.listdir order, over 2 worker processes."""
    import numpy as np
    from PIL import Image

    from icap.images import ImageDirectoryDataset, extract_directory

    d = tmp_path / "imgs"
    d.mkdir()
    rng = np.random.default_rng(0)
    arrays = {}
    for i in range(7):
        a = rng.integers(0, 256, (20 + 3 * i, 30 + i, 3), dtype=np.uint8)
        name = f"COCO_val2014_{100 + i:012d}.png"  # lossless, so the decoded bytes are the array
        Image.fromarray(a).save(d / name)
        arrays[name] = a
    seen = []

    class PackedStandIn:
        def preprocess_packed(self, packed, sizes):
            off = 0
            feats = []
            for h, w in sizes:
                img = packed[off: off + h * w * 3].view(h, w, 3)
                off += h * w * 3
                seen.append(img.numpy().copy())
                feats.append(img.float().mean(dim=(0, 1)))
            assert off == packed.numel()
            return torch.stack(feats)

    out = tmp_path / "emb.pt"
    n = extract_directory(str(d), str(out), lambda px: px, PackedStandIn(), 3, batch_size=3, num_workers=2)
    assert n == 7
    names = ImageDirectoryDataset(str(d)).filenames
    data = torch.load(str(out), weights_only=True)
    assert data["filenames"] == names
    for name, img, row in zip(names, seen, data["embeddings"]):
        assert np.array_equal(img, arrays[name])
        assert torch.allclose(row, torch.from_numpy(arrays[name]).float().mean(dim=(0, 1)))
