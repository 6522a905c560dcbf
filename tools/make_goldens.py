"""Generate tests/golden/*.npz by running the REFERENCE itself (build container only).

Imports /root/reference/src (read-only) with the unavailable third-party modules
stubbed (faiss, objectbox -> src/database only; pycocoevalcap -> src/eval.py
metrics; tensorboard -> train.py:6,15-17), builds the reference's own modules
(ImageCaptioningModel, TransformerMappingNetwork, MLPMappingNetwork over HF
GPT2LMHeadModel/CLIPModel) with weights from oracle.gen_tensor, and records their
outputs. Dropout is disabled (GPT2Config *_pdrop=0 and the mapper's dropout
modules set to p=0) so outputs are deterministic. Only inputs + outputs are
written: no reference source travels.

Run:  PYTHONDONTWRITEBYTECODE=1 python tools/make_goldens.py [tiny small clip vit clip_l14 dino topp small_train medium ckpt
                                                            small_bf16w bench128_bf16w]
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
    # 3 reference train() steps through the MLP mapper (GPT-2 frozen): losses + every trained tensor
    model2, _, msd = build_ref(gcfg, mcfg, 0, mapper="mlp")
    losses = run_ref_train(model2, (ids, mask, labels, emb), 3, 1e-4, True, workdir)
    trained = {"trained." + k: v.detach().numpy() for k, v in model2.mapping_network.state_dict().items()}
    np.savez_compressed(os.path.join(OUT, "tiny_mlp.npz"), ids=ids.numpy(), mask=mask.numpy(),
                        labels=labels.numpy(), emb=emb.numpy(), prefix=prefix.numpy(), loss=np.array([res.loss.item()]),
                        logits=res.logits.numpy(), train_losses=np.array(losses), **trained)
    print("tiny_mlp loss", res.loss.item(), "train", losses)


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


def vit_keys_to_installed(sd):
    """transformers 4.57 ViT names (oracle.vit_state_dict; the reference's pin) -> the installed 5.x layout."""
    out = {}
    for k, v in sd.items():
        n = k
        if k.startswith("encoder.layer."):
            i, rest = k[len("encoder.layer."):].split(".", 1)
            rest = (rest.replace("attention.attention.query", "attention.q_proj")
                    .replace("attention.attention.key", "attention.k_proj")
                    .replace("attention.attention.value", "attention.v_proj")
                    .replace("attention.output.dense", "attention.o_proj")
                    .replace("intermediate.dense", "mlp.fc1").replace("output.dense", "mlp.fc2"))
            n = f"layers.{i}.{rest}"
        out[n] = v
    return out


def golden_vit_b16():
    """ViT-B/16 pooler embedding (src/embeddings/vit.py:63-72): HF ViTModel(ViTConfig()) = google/vit-base-patch16-224
    geometry, deterministic weights, 2 seeded images."""
    from transformers import ViTConfig, ViTModel

    cfg = O.ViTCfg()
    hf = ViTModel(ViTConfig())
    missing, unexpected = hf.load_state_dict(vit_keys_to_installed(O.vit_state_dict(cfg, 0)), strict=False)
    assert not missing and not unexpected, (missing, unexpected)
    hf.eval()
    px = torch.randn((2, 3, 224, 224), generator=torch.Generator().manual_seed(4))
    with torch.no_grad():
        out = hf(pixel_values=px)
        pooled = out.pooler_output
        normed = pooled / pooled.norm(p=2, dim=-1, keepdim=True)  # vit.py:71
    np.savez_compressed(os.path.join(OUT, "vit_b16.npz"), pixels_seed=np.array([4]), pooler=pooled.numpy(),
                        embeddings=normed.numpy())
    print("vit_b16", normed[0, :5])


def golden_clip_l14():
    """CLIP ViT-L/14 image features (BASELINE configs[3]: load_clip_model("openai/clip-vit-large-patch14"),
    src/embeddings/clip.py:10-12): HF CLIPModel with that vision geometry, deterministic weights, 2 images."""
    from transformers import CLIPConfig, CLIPModel

    cfg = O.ClipCfg(hidden=1024, layers=24, heads=16, patch=14, image=224, inter=4096, proj=768)
    hf = CLIPModel(CLIPConfig(vision_config=dict(hidden_size=1024, num_hidden_layers=24, num_attention_heads=16,
                                                 intermediate_size=4096, patch_size=14, image_size=224),
                              projection_dim=768))
    missing, unexpected = hf.load_state_dict(O.clip_vision_state_dict(cfg, seed=0), strict=False)
    assert not unexpected
    assert all(not k.startswith("vision_model.") and k != "visual_projection.weight" for k in missing)
    hf.eval()
    px = torch.randn((2, 3, 224, 224), generator=torch.Generator().manual_seed(5))
    with torch.no_grad():
        feats = hf.get_image_features(pixel_values=px)
        feats = getattr(feats, "pooler_output", feats)
        normed = feats / feats.norm(p=2, dim=-1, keepdim=True)
    np.savez_compressed(os.path.join(OUT, "clip_l14.npz"), pixels_seed=np.array([5]), features=feats.numpy(),
                        embeddings=normed.numpy())
    print("clip_l14", normed[0, :5])


def golden_dinov3():
    """DINOv3 ViT-L/16 backbone (BASELINE configs[4]; src/embeddings/dino.py loads it from torch.hub, which is gated
    and offline here): HF DINOv3ViTModel (transformers 5.15) at the ViT-L/16 geometry with 4 register tokens,
    key_bias=False and LayerScale, deterministic weights, 2 seeded images. The dino.txt vision head that
    encode_image adds on top of the backbone is not available offline (parity unpinned for that head)."""
    from transformers import DINOv3ViTConfig, DINOv3ViTModel

    cfg = O.DinoCfg()
    hf = DINOv3ViTModel(DINOv3ViTConfig(hidden_size=cfg.hidden, num_hidden_layers=cfg.layers,
                                        num_attention_heads=cfg.heads, intermediate_size=cfg.inter,
                                        num_register_tokens=cfg.registers, key_bias=False, layerscale_value=1.0,
                                        patch_size=cfg.patch, image_size=cfg.image, rope_theta=cfg.rope_theta,
                                        layer_norm_eps=cfg.eps))
    missing, unexpected = hf.load_state_dict(O.dinov3_state_dict(cfg, 0), strict=True)
    assert not missing and not unexpected, (missing, unexpected)
    hf.eval()
    px = torch.randn((2, 3, 224, 224), generator=torch.Generator().manual_seed(6))
    with torch.no_grad():
        out = hf(pixel_values=px)
        pooled = out.pooler_output
        normed = pooled / pooled.norm(p=2, dim=-1, keepdim=True)
        patch_mean = out.last_hidden_state[:, 1 + cfg.registers:].mean(dim=1)
    np.savez_compressed(os.path.join(OUT, "dinov3_l16.npz"), pixels_seed=np.array([6]), pooler=pooled.numpy(),
                        embeddings=normed.numpy(), patch_mean=patch_mean.numpy(),
                        registers=out.last_hidden_state[:, 1:1 + cfg.registers].numpy())
    print("dinov3_l16", normed[0, :5])


def golden_topp():
    """The reference's top-p filter (src/models.py:400-449) as the reference runs it: generate(temperature 0.8,
    top_p 0.9) at the tiny config with torch.multinomial replaced by a recorder that returns the most probable kept
    token (so the path is deterministic); records the filter's input logits (recomputed by the reference forward)
    and its output distribution (probs > 0 = the kept set) for every step."""
    import src.models as RM

    gcfg = O.GPT2Cfg(n_layer=2, n_embd=128, n_head=2, vocab_size=512, n_positions=128, eos=511)
    mcfg = O.MapperCfg(embed_dim=64, gpt_dim=128, prefix_length=5, hidden_length=4, num_layers=2)
    model, _, _ = build_ref(gcfg, mcfg, 0)
    model.eval()
    _, _, _, emb = O.synthetic_batch(4, 12, 7, 512, 511, 64, seed=7)
    probs_log, logits_log = [], []
    real_softmax = torch.nn.functional.softmax

    def multinomial(probs, num_samples=1):
        probs_log.append(probs.detach().clone())
        return probs.argmax(-1, keepdim=True)

    orig_forward = model.gpt.forward

    def forward(*a, **k):
        out = orig_forward(*a, **k)
        logits_log.append(out.logits[:, -1, :].detach().clone())
        return out

    model.gpt.forward = forward
    with mock.patch.object(RM.torch, "multinomial", multinomial):
        with torch.no_grad():
            ids = model.generate(emb, max_length=6, temperature=0.8, top_p=0.9)
    del real_softmax
    np.savez_compressed(os.path.join(OUT, "topp_filter.npz"), emb=emb.numpy(), ids=ids.numpy(),
                        logits=torch.stack(logits_log[: len(probs_log)]).numpy(),
                        probs=torch.stack(probs_log).numpy(), temperature=np.array([0.8]), top_p=np.array([0.9]))
    print("topp steps", len(probs_log), "kept per row", (torch.stack(probs_log) > 0).sum(-1)[0].tolist())


def hf_beam(gcfg, gsd, prefix, max_new, num_beams=4):
    """transformers' own beam search (GPT2LMHeadModel.generate, HF/generation/utils.py:3208-3540) on the
    caption prefix: the definition the device beam search and oracle.beam_generate are pinned to (the reference
    itself has greedy / top-p only, src/models.py:327-477)."""
    from transformers import GPT2Config, GPT2LMHeadModel

    hf = GPT2Config(vocab_size=gcfg.vocab_size, n_positions=gcfg.n_positions, n_embd=gcfg.n_embd,
                    n_layer=gcfg.n_layer, n_head=gcfg.n_head, resid_pdrop=0.0, embd_pdrop=0.0, attn_pdrop=0.0,
                    layer_norm_epsilon=gcfg.eps, bos_token_id=gcfg.eos, eos_token_id=gcfg.eos)
    gpt = GPT2LMHeadModel(hf)
    gpt.load_state_dict(gsd, strict=False)
    gpt.tie_weights()
    gpt.eval()
    with torch.no_grad():
        return gpt.generate(inputs_embeds=prefix, attention_mask=torch.ones(prefix.shape[:2], dtype=torch.long),
                            num_beams=num_beams, max_new_tokens=max_new, do_sample=False, early_stopping=False,
                            length_penalty=1.0, num_return_sequences=1, pad_token_id=gcfg.eos,
                            eos_token_id=gcfg.eos)


def golden_beam():
    """Beam-4 ids from transformers' generate on the tiny and small goldens' prefixes.
    `eos_scale` multiplies wte[eos] (the tied LM-head row) so captions finish at different steps and the
    finished-hypothesis / early-stop paths are exercised; 1.0 = the plain weights."""
    out = {}
    tiny_g = O.GPT2Cfg(n_layer=2, n_embd=128, n_head=2, vocab_size=512, n_positions=128, eos=511)
    tiny = np.load(os.path.join(OUT, "tiny.npz"))
    small = np.load(os.path.join(OUT, "small.npz"))
    # the tiny golden's 3 mapper prefixes + 5 seeded ones of the same scale (more captions, more finishing steps)
    g = torch.Generator().manual_seed(11)
    extra = torch.randn((5,) + tiny["prefix"].shape[1:], generator=g) * float(tiny["prefix"].std())
    tiny_pre = np.concatenate([tiny["prefix"], extra.numpy()]).astype(np.float32)
    for tag, gcfg, pre, L, scales in (("tiny", tiny_g, tiny_pre, 20, (1.0, 4.0, 5.0, 6.0)),
                                      ("small", O.GPT2Cfg(), small["prefix"][:2], 12, (1.0, 3.0, 4.0))):
        for s in scales:
            gsd = O.gpt2_state_dict(gcfg, 0)
            gsd["transformer.wte.weight"] = gsd["transformer.wte.weight"].clone()
            gsd["transformer.wte.weight"][gcfg.eos] *= s
            ids = hf_beam(gcfg, gsd, torch.from_numpy(pre), L)
            k = f"{tag}_s{s:g}"
            out[k + "_ids"] = ids.numpy()
            out[k + "_scale"] = np.array([s])
            n_eos = [(int((r == gcfg.eos).nonzero()[0][0]) + 1 if (r == gcfg.eos).any() else -1) for r in ids]
            print("beam", k, tuple(ids.shape), "eos at", n_eos)
    out["tiny_prefix"] = tiny_pre
    out["small_prefix"] = small["prefix"][:2]
    np.savez_compressed(os.path.join(OUT, "beam4.npz"), **out)


def golden_small_train(workdir):
    """GPT-2 small + transformer mapper: 3 frozen train() steps with the trained mapper tensors kept whole (bf16
    update-direction tests), 2 unfrozen steps (every GPT-2 tensor's checksum), and greedy decode at the
    benchmarked decode shape (128 captions x 50 tokens, the reference's full-recompute loop)."""
    gcfg, mcfg = O.GPT2Cfg(), O.MapperCfg()
    torch.manual_seed(0)
    model, _, _ = build_ref(gcfg, mcfg, seed=0)
    ids, mask, labels, emb = O.synthetic_batch(4, 50, 13, gcfg.vocab_size, gcfg.eos, mcfg.embed_dim, seed=1)
    out = {"ids": ids.numpy(), "mask": mask.numpy(), "labels": labels.numpy(), "emb": emb.numpy()}
    losses = run_ref_train(model, (ids, mask, labels, emb), 3, 1e-4, True, workdir)
    out["train_losses"] = np.array(losses)
    for k, v in model.mapping_network.state_dict().items():
        out["trained_ck." + k] = checksum(v)
        if not k.startswith("transformer.layers.") or k.startswith("transformer.layers.0."):
            a = v.numpy()  # whole (small tensors) or every 97th element (matrices): a fixture of ~0.6 MB
            if a.size > 20000:
                out["trained_sample." + k] = a.reshape(-1)[::97].copy()
            else:
                out["trained." + k] = a
    model2, _, _ = build_ref(gcfg, mcfg, seed=0)
    losses2 = run_ref_train(model2, (ids, mask, labels, emb), 2, 1e-4, False, workdir)
    out["unfrozen_losses"] = np.array(losses2)
    for k, v in model2.state_dict().items():
        if k != "gpt.lm_head.weight":
            out["unfrozen_ck." + k] = checksum(v)
    np.savez_compressed(os.path.join(OUT, "small_train.npz"), **out)
    print("small_train", losses, losses2)
    model3, _, _ = build_ref(gcfg, mcfg, seed=0)
    model3.eval()
    g = torch.Generator().manual_seed(5)
    e = torch.randn((128, mcfg.embed_dim), generator=g)
    e = e / e.norm(dim=-1, keepdim=True)
    with torch.no_grad():
        gen = model3.generate(e, max_length=50, temperature=0.0)
    np.savez_compressed(os.path.join(OUT, "small_greedy128.npz"), emb_seed=np.array([5]), greedy=gen.numpy())
    print("small_greedy128", tuple(gen.shape))


def golden_medium(workdir):
    """BASELINE configs[3] geometry: GPT-2 medium (24 layers, d 1024, 16 heads) + transformer mapper at gpt_dim 1024
    (head dim 128) over 768-d CLIP-L/14 embeddings."""
    golden_config("medium", O.GPT2Cfg(n_layer=24, n_embd=1024, n_head=16),
                  O.MapperCfg(embed_dim=768, gpt_dim=1024), B=2, L=12, real=7, gen_B=2, gen_len=8,
                  logit_rows=[14, 17, 26], train_steps=2, unfrozen_steps=0, workdir=workdir, full_logits=False)


def golden_large(workdir):
    """BASELINE configs[4] caption model: GPT-2 large (36 layers, d 1280, 20 heads) + transformer mapper at
    gpt_dim 1280 (8 heads of 160) over 1024-d DINOv3 ViT-L/16 embeddings; plus transformers' beam-4 ids on its
    caption prefix (the configs[4] decode)."""
    gcfg, mcfg = O.GPT2Cfg(n_layer=36, n_embd=1280, n_head=20), O.MapperCfg(embed_dim=1024, gpt_dim=1280)
    golden_config("large", gcfg, mcfg, B=2, L=12, real=7, gen_B=2, gen_len=6, logit_rows=[14, 17, 26],
                  train_steps=2, unfrozen_steps=0, workdir=workdir, full_logits=False)
    model, gsd, _ = build_ref(gcfg, mcfg, 0)
    model.eval()
    _, _, _, emb = O.synthetic_batch(2, 12, 7, gcfg.vocab_size, gcfg.eos, mcfg.embed_dim, seed=1)
    with torch.no_grad():
        prefix = model.mapping_network(emb)
    ids = hf_beam(gcfg, gsd, prefix, 8, num_beams=4)
    np.savez_compressed(os.path.join(OUT, "large_beam4.npz"), prefix=prefix.numpy(), ids=ids.numpy())
    print("large beam4", ids.tolist())


def golden_bench128(workdir):
    """The benchmarked shape itself (bench.py / BASELINE configs[1]): B = 128 images, CLIP
    ViT-B/32 features from seeded 224x224 pixels (HF CLIPModel.get_image_features -> pooler_output, L2-normalised as
    src/embeddings/clip.py:132-137), COCO-shaped 50-token captions (13 tokens + EOS), S = 65, GPT-2 small frozen +
    transformer mapper, 2 reference train() steps (src/train.py, lr 1e-4, dropout off). Stored small: the
    embeddings, the forward loss, the train losses, per-tensor checksums of the trained mapper and each trained
    tensor whole (<= 20000 elements) or every 997th element (update-direction bounds for the bf16 run)."""
    from transformers import CLIPConfig, CLIPModel

    gcfg, mcfg = O.GPT2Cfg(), O.MapperCfg()
    hf = CLIPModel(CLIPConfig())
    missing, unexpected = hf.load_state_dict(O.clip_vision_state_dict(O.ClipCfg(), seed=0), strict=False)
    assert not unexpected
    hf.eval()
    B = 128
    px = torch.randn((B, 3, 224, 224), generator=torch.Generator().manual_seed(21))
    with torch.no_grad():
        feats = hf.get_image_features(pixel_values=px)
        feats = getattr(feats, "pooler_output", feats)
        emb = feats / feats.norm(p=2, dim=-1, keepdim=True)
    ids, mask, labels, _ = O.synthetic_batch(B, 50, 13, gcfg.vocab_size, gcfg.eos, mcfg.embed_dim, seed=22)
    torch.manual_seed(0)
    model, _, _ = build_ref(gcfg, mcfg, seed=0)
    model.eval()
    with torch.no_grad():
        res = model.forward(caption_token_ids=ids, image_embeddings=emb, attention_mask=mask, labels=labels)
    out = {"pixels_seed": np.array([21]), "batch_seed": np.array([22]), "emb": emb.numpy(),
           "loss": np.array([res.loss.item()]), "lse_row0": torch.logsumexp(res.logits[0].double(), -1).numpy()}
    losses = run_ref_train(model, (ids, mask, labels, emb), 2, 1e-4, True, workdir)
    out["train_losses"] = np.array(losses)
    for k, v in model.mapping_network.state_dict().items():
        out["trained_ck." + k] = checksum(v)
        a = v.detach().numpy().reshape(-1)
        out["trained_sample." + k] = a.copy() if a.size <= 20000 else a[::997].copy()
    np.savez_compressed(os.path.join(OUT, "bench128.npz"), **out)
    print("bench128 loss", out["loss"], "train", losses)


def bf16_round_(module):
    """Every floating parameter of `module` rounded to bf16 in place (kept fp32): the weights the bf16 perf mode
    computes with (frozen GPT-2 / CLIP weights are stored bf16; the trained mapper's compute copy is its bf16
    rounding). The reference then computes in fp32 on them: SURVEY.md §8(c) "bf16-rounded-weights" variant."""
    with torch.no_grad():
        for prm in module.parameters():
            if prm.is_floating_point():
                prm.copy_(prm.to(torch.bfloat16).float())


def golden_small_bf16w(workdir):
    """The 'small' golden (GPT-2 small + transformer mapper, B = 4, L = 50) and the benchmarked greedy shape (128 x 50)
    with every weight pre-rounded to bf16: the reference's own forward (loss, every position's logsumexp and argmax,
    selected logit rows) and generate() in fp32 on those weights -> tests/golden/small_bf16w.npz. The bf16 perf mode's
    remaining difference from it is the rounding of activations, not of weights."""
    gcfg, mcfg = O.GPT2Cfg(), O.MapperCfg()
    torch.manual_seed(0)
    model, _, _ = build_ref(gcfg, mcfg, seed=0)
    bf16_round_(model)
    model.eval()
    ids, mask, labels, emb = O.synthetic_batch(4, 50, 13, gcfg.vocab_size, gcfg.eos, mcfg.embed_dim, seed=1)
    out = {"ids": ids.numpy(), "mask": mask.numpy(), "labels": labels.numpy(), "emb": emb.numpy()}
    with torch.no_grad():
        res = model.forward(caption_token_ids=ids, image_embeddings=emb, attention_mask=mask, labels=labels)
        out["prefix"] = model.mapping_network(emb).numpy()
    out["loss"] = np.array([res.loss.item()])
    lg = res.logits.double()
    out["lse"] = torch.logsumexp(lg, -1).numpy()
    out["argmax"] = lg.argmax(-1).numpy()
    rows = torch.tensor([14, 27, 64])
    out["logit_rows"] = rows.numpy()
    out["logits_sel"] = res.logits[:2][:, rows].numpy()
    g = torch.Generator().manual_seed(5)  # the small_greedy128 embeddings
    e = torch.randn((128, mcfg.embed_dim), generator=g)
    e = e / e.norm(dim=-1, keepdim=True)
    with torch.no_grad():
        out["greedy128"] = model.generate(e, max_length=50, temperature=0.0).numpy()
    np.savez_compressed(os.path.join(OUT, "small_bf16w.npz"), **out)
    print("small_bf16w loss", out["loss"], "greedy128", out["greedy128"].shape)


def golden_bench128_bf16w(workdir):
    """bench128 (the benchmarked B = 128 step) with every weight — CLIP tower, GPT-2, mapper init — pre-rounded to
    bf16 and the reference computing in fp32: CLIP features, forward loss, 2 train() steps, trained mapper samples
    -> tests/golden/bench128_bf16w.npz (the bf16 train step's update-direction bounds)."""
    from transformers import CLIPConfig, CLIPModel

    gcfg, mcfg = O.GPT2Cfg(), O.MapperCfg()
    hf = CLIPModel(CLIPConfig())
    missing, unexpected = hf.load_state_dict(O.clip_vision_state_dict(O.ClipCfg(), seed=0), strict=False)
    assert not unexpected
    bf16_round_(hf.vision_model)
    bf16_round_(hf.visual_projection)
    hf.eval()
    B = 128
    px = torch.randn((B, 3, 224, 224), generator=torch.Generator().manual_seed(21))
    with torch.no_grad():
        feats = hf.get_image_features(pixel_values=px)
        feats = getattr(feats, "pooler_output", feats)
        emb = feats / feats.norm(p=2, dim=-1, keepdim=True)
    ids, mask, labels, _ = O.synthetic_batch(B, 50, 13, gcfg.vocab_size, gcfg.eos, mcfg.embed_dim, seed=22)
    torch.manual_seed(0)
    model, _, _ = build_ref(gcfg, mcfg, seed=0)
    bf16_round_(model)
    model.eval()
    with torch.no_grad():
        res = model.forward(caption_token_ids=ids, image_embeddings=emb, attention_mask=mask, labels=labels)
    out = {"pixels_seed": np.array([21]), "batch_seed": np.array([22]), "emb": emb.numpy(),
           "loss": np.array([res.loss.item()])}
    # the first step's gradient of the mean loss w.r.t. every mapper tensor (before clip_grad_norm / AdamW: the
    # update direction after AdamW's per-element normalisation is dominated by the elements whose gradient is ~0)
    model.train()
    for prm in model.gpt.parameters():
        prm.requires_grad = False
    model.zero_grad(set_to_none=True)
    model.forward(caption_token_ids=ids, image_embeddings=emb, attention_mask=mask, labels=labels).loss.backward()
    for k, prm in model.mapping_network.named_parameters():
        if prm.grad is None:
            continue
        a = prm.grad.detach().numpy().reshape(-1)
        out["grad_sample." + k] = a.copy() if a.size <= 20000 else a[::997].copy()
    model.zero_grad(set_to_none=True)
    init = {k: v.detach().clone() for k, v in model.mapping_network.state_dict().items()}
    losses = run_ref_train(model, (ids, mask, labels, emb), 2, 1e-4, True, workdir)
    out["train_losses"] = np.array(losses)
    for k, v in model.mapping_network.state_dict().items():
        a = (v.detach() - init[k]).numpy().reshape(-1)  # the update of this (rounded-init) run
        out["update_sample." + k] = a.copy() if a.size <= 20000 else a[::997].copy()
    np.savez_compressed(os.path.join(OUT, "bench128_bf16w.npz"), **out)
    print("bench128_bf16w loss", out["loss"], "train", losses)


def golden_ckpt_keys(workdir):
    """Key sets + shapes of the reference's save_parameters() files (src/models.py:489-519) for the transformer
    mapper with GPT-2 frozen / unfrozen and the MLP mapper (GPT-2 small geometry), and of its extraction .pt
    (src/embeddings/clip.py:147-149) -> tests/golden/ckpt_keys.json."""
    import json

    out = {}
    for tag, mapper, mcfg, freeze in (("transformer_frozen", "transformer", O.MapperCfg(), True),
                                      ("transformer_unfrozen", "transformer", O.MapperCfg(), False),
                                      ("mlp_frozen", "mlp", O.MLPMapperCfg(), True)):
        model, _, _ = build_ref(O.GPT2Cfg(), mcfg, 0, mapper)
        if not freeze:
            for p in model.gpt.parameters():
                p.requires_grad = True
        path = os.path.join(workdir, f"{tag}.pt")
        model.save_parameters(path)
        sd = torch.load(path, map_location="cpu", weights_only=True)
        out[tag] = {k: list(v.shape) for k, v in sd.items()}
        print(tag, len(sd), "keys")
    with open(os.path.join(OUT, "ckpt_keys.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


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
        only = set(sys.argv[1:])  # optional subset: tiny small clip vit clip_l14 topp small_train medium
        if not only or "tiny" in only:
            golden_config("tiny", tiny_g, tiny_m, B=3, L=12, real=7, gen_B=3, gen_len=20, logit_rows=[4, 10, 16],
                          train_steps=3, unfrozen_steps=2, workdir=work, full_logits=True)
        if not only or "tiny" in only or "mlp" in only:
            golden_mlp(work)
        if not only or "small" in only:
            golden_config("small", O.GPT2Cfg(), O.MapperCfg(), B=4, L=50, real=13, gen_B=2, gen_len=12,
                          logit_rows=[14, 27, 64], train_steps=2, unfrozen_steps=0, workdir=work, full_logits=False)
        if not only or "clip" in only:
            golden_clip()
        if not only or "vit" in only:
            golden_vit_b16()
        if not only or "clip_l14" in only:
            golden_clip_l14()
        if not only or "dino" in only:
            golden_dinov3()
        if not only or "topp" in only:
            golden_topp()
        if not only or "beam" in only:
            golden_beam()
        if not only or "small_train" in only:
            golden_small_train(work)
        if not only or "medium" in only:
            golden_medium(work)
        if not only or "large" in only:
            golden_large(work)
        if not only or "bench128" in only:
            golden_bench128(work)
        if not only or "ckpt" in only:
            golden_ckpt_keys(work)
        if not only or "small_bf16w" in only:
            golden_small_bf16w(work)
        if not only or "bench128_bf16w" in only:
            golden_bench128_bf16w(work)
    finally:
        os.chdir(cwd)


if __name__ == "__main__":
    main()
