"""Generate tests/golden/*.npz by running the REFERENCE itself (build container only).

Imports /root/reference/src (read-only) with the unavailable third-party modules
stubbed (faiss, objectbox -> src/database only; pycocoevalcap -> src/eval.py
metrics; tensorboard -> train.py:6,15-17), builds the reference's own modules
(ImageCaptioningModel, TransformerMappingNetwork, MLPMappingNetwork over HF
GPT2LMHeadModel/CLIPModel) with weights from oracle.gen_tensor, and records their
outputs. Dropout is disabled (GPT2Config *_pdrop=0 and the mapper's dropout
modules set to p=0) so outputs are deterministic. Only inputs + outputs are
written: no reference source travels.

Run:  PYTHONDONTWRITEBYTECODE=1 python tools/make_goldens.py
"""

from __future__ import annotations

import os
import sys
import tempfile
import types
from unittest import mock

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
OUT = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, ROOT)

from oracle import icap_oracle as O  # noqa: E402


def stub_modules():
    for name in ("faiss", "objectbox"):
        sys.modules[name] = mock.MagicMock()
    for name in ("pycocoevalcap", "pycocoevalcap.bleu", "pycocoevalcap.bleu.bleu", "pycocoevalcap.cider",
                 "pycocoevalcap.cider.cider", "pycocoevalcap.rouge", "pycocoevalcap.rouge.rouge"):
        sys.modules[name] = mock.MagicMock()
    tb = types.ModuleType("torch.utils.tensorboard")
    tb.SummaryWriter = mock.MagicMock()
    sys.modules["torch.utils.tensorboard"] = tb


class Tok:
    """Only eos_token_id is read by generate (src/models.py:348)."""

    def __init__(self, eos):
        self.eos_token_id = eos
        self.eos_token = "<|endoftext|>"


class ListDataset(torch.utils.data.Dataset):
    def __init__(self, ids, mask, labels, emb):
        self.t = (ids, mask, labels, emb)

    def __len__(self):
        return self.t[0].shape[0]

    def __getitem__(self, i):
        ids, mask, labels, emb = self.t
        return {"token_ids": ids[i], "labels": labels[i], "image_embedding": emb[i], "attention_mask": mask[i],
                "caption_text": "", "image_id": i}


def build_ref(gcfg: O.GPT2Cfg, mcfg, seed: int, mapper: str = "transformer"):
    from transformers import GPT2Config, GPT2LMHeadModel

    import src.models as RM

    hf = GPT2Config(vocab_size=gcfg.vocab_size, n_positions=gcfg.n_positions, n_embd=gcfg.n_embd,
                    n_layer=gcfg.n_layer, n_head=gcfg.n_head, resid_pdrop=0.0, embd_pdrop=0.0, attn_pdrop=0.0,
                    layer_norm_epsilon=gcfg.eps, bos_token_id=gcfg.eos, eos_token_id=gcfg.eos)
    gpt = GPT2LMHeadModel(hf)
    gsd = O.gpt2_state_dict(gcfg, seed)
    missing, unexpected = gpt.load_state_dict(gsd, strict=False)
    assert not unexpected and all(k == "lm_head.weight" for k in missing), (missing, unexpected)
    if mapper == "transformer":
        m = RM.TransformerMappingNetwork(embed_dim=mcfg.embed_dim, gpt_dim=mcfg.gpt_dim,
                                         prefix_length=mcfg.prefix_length, hidden_length=mcfg.hidden_length,
                                         num_layers=mcfg.num_layers)
        msd = O.mapper_state_dict(mcfg, seed)
        for layer in m.transformer.layers:  # deterministic goldens: dropout off
            layer.dropout.p = layer.dropout1.p = layer.dropout2.p = 0.0
            layer.self_attn.dropout = 0.0
    else:
        m = RM.MLPMappingNetwork(prefix_length=mcfg.prefix_length, embed_dim=mcfg.embed_dim, gpt_dim=mcfg.gpt_dim)
        msd = O.mlp_mapper_state_dict(mcfg, seed)
    m.load_state_dict(msd, strict=True)
    model = RM.ImageCaptioningModel(mapping_network=m, tokenizer=Tok(gcfg.eos), gpt=gpt, freeze_gpt_weights=True)
    return model, gsd, msd


def checksum(t: torch.Tensor):
    t = t.detach().double()
    return np.array([t.sum().item(), t.abs().sum().item(), (t * t).sum().item()])


def run_ref_train(model, batch, steps, lr, freeze: bool, workdir):
    import src.train as RT

    for p in model.gpt.parameters():
        p.requires_grad = not freeze
    ds = ListDataset(*batch)
    torch.manual_seed(0)
    hist = RT.train(train_dataset=ds, model=model, batch_size=len(ds), num_epochs=steps, num_workers=0,
                    learning_rate=lr, num_warmup_steps=0, save_every_epoch=10 ** 6, device=torch.device("cpu"),
                    outputs_dir=os.path.join(workdir, "ckpt"))
    return hist["epoch_losses"]


def golden_config(tag, gcfg, mcfg, B, L, real, gen_B, gen_len, logit_rows, train_steps, unfrozen_steps, workdir,
                  full_logits):
    torch.manual_seed(0)
    model, gsd, msd = build_ref(gcfg, mcfg, seed=0)
    model.eval()
    ids, mask, labels, emb = O.synthetic_batch(B, L, real, gcfg.vocab_size, gcfg.eos, mcfg.embed_dim, seed=1)
    out = {"ids": ids.numpy(), "mask": mask.numpy(), "labels": labels.numpy(), "emb": emb.numpy()}
    with torch.no_grad():
        prefix = model.mapping_network(emb)
        res = model.forward(caption_token_ids=ids, image_embeddings=emb, attention_mask=mask, labels=labels)
    out["prefix"] = prefix.numpy()
    out["loss"] = np.array([res.loss.item()])
    lg = res.logits.double()
    out["lse"] = torch.logsumexp(lg, -1).numpy()
    out["argmax"] = lg.argmax(-1).numpy()
    if full_logits:
        out["logits"] = res.logits.numpy()
    else:
        rows = torch.tensor(logit_rows)
        out["logit_rows"] = rows.numpy()
        out["logits_sel"] = res.logits[:2][:, rows].numpy()
    with torch.no_grad():
        gen = model.generate(emb[:gen_B], max_length=gen_len, temperature=0.0)
    out["greedy"] = gen.numpy()
    # training: reference src/train.py::train, same batch every epoch (1 batch / epoch)
    losses = run_ref_train(model, (ids, mask, labels, emb), train_steps, 1e-4, True, workdir)
    out["train_losses"] = np.array(losses)
    for k, v in model.mapping_network.state_dict().items():
        out["trained_ck." + k] = checksum(v)
    if full_logits:
        for k, v in model.mapping_network.state_dict().items():
            out["trained." + k] = v.numpy()
    if unfrozen_steps:
        model2, _, _ = build_ref(gcfg, mcfg, seed=0)
        losses2 = run_ref_train(model2, (ids, mask, labels, emb), unfrozen_steps, 1e-4, False, workdir)
        out["unfrozen_losses"] = np.array(losses2)
        for k, v in model2.state_dict().items():
            if k == "gpt.lm_head.weight":
                continue
            out["unfrozen_ck." + k] = checksum(v)
    np.savez_compressed(os.path.join(OUT, f"{tag}.npz"), **out)
    print(tag, "loss", out["loss"], "train", out["train_losses"], "greedy", out["greedy"][0][:10])


def golden_mlp(workdir):
    gcfg = O.GPT2Cfg(n_layer=2, n_embd=128, n_head=2, vocab_size=512, n_positions=128, eos=511)
    mcfg = O.MLPMapperCfg(prefix_length=5, embed_dim=64, gpt_dim=128)
    model, _, _ = build_ref(gcfg, mcfg, 0, mapper="mlp")
    model.eval()
    ids, mask, labels, emb = O.synthetic_batch(3, 12, 7, 512, 511, 64, seed=1)
    with torch.no_grad():
        res = model.forward(caption_token_ids=ids, image_embeddings=emb, attention_mask=mask, labels=labels)
        prefix = model.mapping_network(emb)
    np.savez_compressed(os.path.join(OUT, "tiny_mlp.npz"), ids=ids.numpy(), mask=mask.numpy(),
                        labels=labels.numpy(), emb=emb.numpy(), prefix=prefix.numpy(), loss=np.array([res.loss.item()]),
                        logits=res.logits.numpy())
    print("tiny_mlp loss", res.loss.item())


def golden_clip():
    from transformers import CLIPConfig, CLIPModel

    cfg = O.ClipCfg()
    hf = CLIPModel(CLIPConfig())
    sd = O.clip_vision_state_dict(cfg, seed=0)
    missing, unexpected = hf.load_state_dict(sd, strict=False)
    assert not unexpected
    assert all(not k.startswith("vision_model.") and k != "visual_projection.weight" for k in missing)
    hf.eval()
    g = torch.Generator().manual_seed(3)
    px = torch.randn((2, 3, 224, 224), generator=g)
    with torch.no_grad():
        feats = hf.get_image_features(pixel_values=px)
        # transformers 5.x returns an output object (SURVEY.md §7 version skew): pooler_output == 4.57 tensor
        feats = getattr(feats, "pooler_output", feats)
        normed = feats / feats.norm(p=2, dim=-1, keepdim=True)  # src/embeddings/clip.py:135-137
    np.savez_compressed(os.path.join(OUT, "clip_b32.npz"), pixels_seed=np.array([3]), features=feats.numpy(),
                        embeddings=normed.numpy())
    print("clip", normed[0, :5])


def main():
    os.makedirs(OUT, exist_ok=True)
    stub_modules()
    sys.path.insert(0, REF)
    work = tempfile.mkdtemp(prefix="icap_golden_")
    cwd = os.getcwd()
    os.chdir(work)  # train.py:15-17 creates ./logs at import
    try:
        tiny_g = O.GPT2Cfg(n_layer=2, n_embd=128, n_head=2, vocab_size=512, n_positions=128, eos=511)
        tiny_m = O.MapperCfg(embed_dim=64, gpt_dim=128, prefix_length=5, hidden_length=4, num_layers=2)
        golden_config("tiny", tiny_g, tiny_m, B=3, L=12, real=7, gen_B=3, gen_len=20, logit_rows=[4, 10, 16],
                      train_steps=3, unfrozen_steps=2, workdir=work, full_logits=True)
        golden_mlp(work)
        golden_config("small", O.GPT2Cfg(), O.MapperCfg(), B=4, L=50, real=13, gen_B=2, gen_len=12,
                      logit_rows=[14, 27, 64], train_steps=2, unfrozen_steps=0, workdir=work, full_logits=False)
        golden_clip()
    finally:
        os.chdir(cwd)


if __name__ == "__main__":
    main()
