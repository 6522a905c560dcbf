"""CPU-only: every kernel launch of the product schedules stays inside live allocations (tests/dryrun.py).

Runs the real host code of the train step, the autograd drop-in path, inference, greedy decode and the
CLIP tower with the C-ABI calls recorded instead of launched, then checks each recorded pointer extent."""

from types import SimpleNamespace

import pytest
import torch

import icap.weights
from dryrun import dry_run
from icap import CaptionTrainer, GPT2Config, GPT2LMHeadModel, ImageCaptioningModel, MLPMappingNetwork
from icap import TransformerMappingNetwork
from icap.clip import CLIPVisionConfig, CLIPVisionTower

CPU = torch.device("cpu")


def tiny_model(mapper="transformer", freeze=True, dtype=torch.float32, task_prompt=None):
    cfg = GPT2Config(vocab_size=512, n_positions=128, n_embd=128, n_layer=2, n_head=2, eos_token_id=511)
    gpt = GPT2LMHeadModel(cfg)
    if mapper == "transformer":
        m = TransformerMappingNetwork(64, 128, 5, 4, 2)
    else:
        m = MLPMappingNetwork(5, 64, 128)
    tok = SimpleNamespace(eos_token_id=511, encode=lambda s, return_tensors=None: torch.tensor([[1, 2, 3]]))
    return ImageCaptioningModel(m, prefix_task_prompt=task_prompt, tokenizer=tok, gpt=gpt, freeze_gpt_weights=freeze,
                                compute_dtype=dtype)


def batch(B, L, vocab=512, E=64):
    ids = torch.randint(0, vocab - 1, (B, L))
    mask = torch.ones((B, L), dtype=torch.int64)
    mask[:, L // 2:] = 0
    labels = ids.clone()
    labels[mask == 0] = -100
    return ids, mask, labels, torch.randn(B, E)


def _assert_clean(rec):
    assert rec.calls, "nothing recorded"
    bad = rec.check()
    assert not bad, "\n".join(bad[:20])


@pytest.mark.parametrize("mapper", ["transformer", "mlp"])
@pytest.mark.parametrize("dropout", [False, True])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_trainer_step_in_bounds(mapper, dropout, dtype):
    with dry_run() as rec:
        icap.weights.ops.call = rec
        model = tiny_model(mapper, dtype=dtype)
        t = CaptionTrainer(model, 3, 12, num_training_steps=3, dropout=dropout)
        t.load_batch(*batch(3, 12))
        t.micro_step()
        _assert_clean(rec)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("dropout", [False, True])
def test_trainer_unfrozen_step_in_bounds(dtype, dropout):
    """freeze_gpt_weights=False in the fused trainer: dW / LN / tied-wte / wpe grads, the optimizer step and the
    in-place refresh of the GPT-2 copies stay in bounds; the GPT-2 grads land in the flat gradient buffer."""
    with dry_run() as rec:
        icap.weights.ops.call = rec
        model = tiny_model(freeze=False, dtype=dtype)
        t = CaptionTrainer(model, 3, 12, num_training_steps=3, dropout=dropout)
        assert t.gpt_trainable and not t.gws.compact
        t.load_batch(*batch(3, 12))
        t.micro_step()
        _assert_clean(rec)
        names = [c[0] for c in rec.calls]
        assert "icap_embedding_scatter_add" in names and names.count("icap_transpose") >= 4 * 2 + 1


def test_trainer_task_prefix_in_bounds():
    with dry_run() as rec:
        icap.weights.ops.call = rec
        model = tiny_model(task_prompt="A picture of")
        t = CaptionTrainer(model, 4, 10, num_training_steps=3)
        t.load_batch(*batch(4, 10))
        t.micro_step()
        _assert_clean(rec)


@pytest.mark.parametrize("freeze", [True, False])
def test_autograd_dropin_in_bounds(freeze):
    with dry_run() as rec:
        icap.weights.ops.call = rec
        model = tiny_model(freeze=freeze)
        ids, mask, labels, emb = batch(3, 12)
        out = model(ids, emb, mask, labels)
        out.loss.backward()
        _assert_clean(rec)


def test_inference_and_greedy_in_bounds():
    with dry_run() as rec:
        icap.weights.ops.call = rec
        model = tiny_model()
        ids, mask, labels, emb = batch(3, 12)
        with torch.no_grad():
            model(ids, emb, mask, labels)
        model.generate(emb, max_length=9, temperature=0.0)
        model.generate(emb, max_length=9, temperature=0.8, top_p=0.9)
        model.gpt(inputs_embeds=torch.randn(2, 7, 128), attention_mask=torch.ones(2, 7, dtype=torch.int64))
        _assert_clean(rec)


def test_negative_temperature_samples_full_softmax():
    """src/models.py:401-407: temperature < 0 divides the logits by 1.0 and skips the top-p filter (a draw from
    the full softmax): the decode calls icap_topp_sample with temperature 1.0 and top_p 1.0."""
    with dry_run() as rec:
        icap.weights.ops.call = rec
        model = tiny_model()
        _, _, _, emb = batch(3, 12)
        model.generate(emb, max_length=4, temperature=-0.5, top_p=0.3)
        _assert_clean(rec)
        topp = [c[1] for c in rec.calls if c[0] == "icap_topp_sample"]
    assert topp, "no sampling call"
    for args in topp:  # (dtype, B, V, logits, ld, temperature, top_p, ...)
        assert args[5] == 1.0 and args[6] == 1.0, args[:8]


def test_train_grad_accum_short_last_batch_steps_like_reference(tmp_path):
    """src/train.py:128-159 with grad_accum_steps=4 over 6 batches (11 samples, batch 2: the last batch has 1
    sample and runs on its own trainer): optimizer steps after batches 4 and 6 only — 2 AdamW calls per epoch —
    and the short batch accumulates into the same cycle (its gradients are not cleared first)."""
    import icap
    from icap.dataset import SyntheticCaptionDataset

    ds = SyntheticCaptionDataset(11, max_length=12, real=5, vocab_size=512, eos=511, embed_dim=64)
    with dry_run() as rec:
        icap.weights.ops.call = rec
        model = tiny_model()
        flags = []
        orig = icap.CaptionTrainer.micro_step

        def micro_step(self, use_graph=False, zero=None, step=None):
            flags.append((self.B, zero, step))
            return orig(self, use_graph=use_graph, zero=zero, step=step)

        icap.CaptionTrainer.micro_step = micro_step
        try:
            icap.train(ds, model, batch_size=2, num_epochs=2, num_workers=0, device=CPU, grad_accum_steps=4,
                       outputs_dir=str(tmp_path), save_every_epoch=10, use_graph=False)
        finally:
            icap.CaptionTrainer.micro_step = orig
        _assert_clean(rec)
    n_adamw = sum(1 for c in rec.calls if c[0] == "icap_adamw_step")
    assert n_adamw == 4, n_adamw  # 2 per epoch
    epoch = flags[:6]
    assert [f[0] for f in epoch] == [2, 2, 2, 2, 2, 1]
    assert [f[1] for f in epoch] == [True, False, False, False, True, False]
    assert [f[2] for f in epoch] == [False, False, False, True, False, True]


def test_train_takes_short_only_attention_for_short_captions(tmp_path):
    """train() hands the loader's host batch to the trainer, which reads the packed attention's short-sequence flag
    from the host labels: with COCO-length captions (every packed sequence <= 32 tokens) every attention launch of
    the GPT-2 blocks is the short-only form, as in bench.py (the labels were moved to the device first,
    which kept the flag off for every batch)."""
    import icap
    from icap.dataset import SyntheticCaptionDataset

    ds = SyntheticCaptionDataset(6, max_length=12, real=5, vocab_size=512, eos=511, embed_dim=64)
    seen = []
    orig = icap.CaptionTrainer.load_batch

    def load_batch(self, ids, mask, labels, emb=None, pixels=None):
        seen.append(labels.device.type)
        orig(self, ids, mask, labels, emb=emb, pixels=pixels)
        seen.append(bool(self.gws.short_only))

    with dry_run() as rec:
        icap.weights.ops.call = rec
        model = tiny_model()
        icap.CaptionTrainer.load_batch = load_batch
        try:
            icap.train(ds, model, batch_size=3, num_epochs=1, num_workers=0, device=CPU, outputs_dir=str(tmp_path),
                       save_every_epoch=10, use_graph=False)
        finally:
            icap.CaptionTrainer.load_batch = orig
        _assert_clean(rec)
    assert seen == ["cpu", True] * 2, seen
    attn = [c[1][0]._obj for c in rec.calls if c[0] in ("icap_attention_fwd", "icap_attention_bwd")]
    gpt = [a for a in attn if a.seq_off]  # the GPT-2 blocks' packed launches (the mapper's are not packed)
    assert gpt and all(a.short_only == 1 for a in gpt), [a.short_only for a in gpt]


def test_serial_mapper_schedule_shares_gradient_buffers():
    """The default (serial) mapper backward shares one set of gradient buffers across layers (two alternating for
    the residual stream); the side / grouped schedules keep one per layer."""
    from icap.mapper import TransformerMapperCore

    with dry_run() as rec:
        icap.weights.ops.call = rec
        model = tiny_model()
        t = CaptionTrainer(model, 3, 12, num_training_steps=3, dropout=True, mapper_dw="serial")
        assert isinstance(t.mcore, TransformerMapperCore)
        ws = t.mws
        nl = len(ws.g_dz)
        assert len({b.data_ptr() for b in ws.g_dz}) == 1 and len({b.data_ptr() for b in ws.g_dqkv}) == 1
        assert len({b.data_ptr() for b in ws.g_r}) == min(2, nl) and len({b.data_ptr() for b in ws.g_m}) == min(2, nl)
        t.load_batch(*batch(3, 12))
        t.micro_step()
        _assert_clean(rec)
        side = CaptionTrainer(model, 3, 12, num_training_steps=3, dropout=True, mapper_dw="side")
        assert len({b.data_ptr() for b in side.mws.g_dz}) == nl


def test_fused_mapper_dw_schedule_in_bounds():
    """mapper_dw="fused" (round 6): each mapper layer's four weight-gradient products and four bias gradients as one
    icap_gemm_group call at the end of the layer's step, on the shared gradient buffers of the serial schedule (nothing the group reads is
    rewritten before the layer ends): every product's operands and fp32 output in bounds, one group call per layer."""
    with dry_run() as rec:
        icap.weights.ops.call = rec
        gpt = GPT2LMHeadModel(GPT2Config(n_layer=2))
        model = ImageCaptioningModel(TransformerMappingNetwork(512, 768, 15, 10, num_layers=2), tokenizer=SimpleNamespace(
            eos_token_id=50256), gpt=gpt, compute_dtype=torch.bfloat16)
        t = CaptionTrainer(model, 4, 20, num_training_steps=3, mapper_dw="fused")
        assert t._group == "fused" and len({b.data_ptr() for b in t.mws.g_dz}) == 1
        ids, mask, labels, emb = batch(4, 20, vocab=50257, E=512)
        t.load_batch(ids, mask, labels, emb=emb)
        t.micro_step()
        _assert_clean(rec)
        groups = [c for c in rec.calls if c[0] == "icap_gemm_group"]
        # four weight products + the four bias gradients (ones-column products) per layer
        assert len(groups) == 2 and all(c[1][1] == 8 for c in groups), [c[1][1] for c in groups]
        assert not [c for c in rec.calls if c[0] == "icap_colsum_batch"], "bias gradients outside the group"


def test_gpt2_small_bench_shape_with_clip_in_bounds():
    """The benchmarked configuration (GPT-2 small + ViT-B/32 + transformer mapper, bf16) at B=8."""
    with dry_run() as rec:
        icap.weights.ops.call = rec
        gpt = GPT2LMHeadModel(GPT2Config())
        model = ImageCaptioningModel(TransformerMappingNetwork(512, 768, 15, 10), tokenizer=SimpleNamespace(
            eos_token_id=50256), gpt=gpt, compute_dtype=torch.bfloat16)
        tower = CLIPVisionTower(CLIPVisionConfig())
        t = CaptionTrainer(model, 8, 50, num_training_steps=10, clip_model=tower)
        ids, mask, labels, _ = batch(8, 50, vocab=50257, E=512)
        t.load_batch(ids, mask, labels, pixels=torch.randn(8, 3, 224, 224))
        t.micro_step()
        model.generate(torch.randn(4, 512), max_length=3, temperature=0.0)
        _assert_clean(rec)


def test_fp8_gpt_schedule_in_bounds():
    """BASELINE configs[4]'s fp8 path (gpt_fp8=True): every MX quantise / GEMM of the train step and the forward
    stays inside live allocations (operands, scales, device row counts of the compact head)."""
    with dry_run() as rec:
        icap.weights.ops.call = rec
        cfg = GPT2Config(vocab_size=512, n_positions=128, n_embd=128, n_layer=2, n_head=2, eos_token_id=511)
        gpt = GPT2LMHeadModel(cfg)
        tok = SimpleNamespace(eos_token_id=511)
        model = ImageCaptioningModel(TransformerMappingNetwork(64, 128, 5, 4, 2), tokenizer=tok, gpt=gpt,
                                     compute_dtype=torch.bfloat16, gpt_fp8=True)
        t = CaptionTrainer(model, 3, 12, num_training_steps=3, dropout=True)
        t.load_batch(*batch(3, 12))
        t.micro_step()
        with torch.no_grad():
            model.eval()(*[x for x in batch(3, 12)][:1], batch(3, 12)[3], None, None)
            model.generate(torch.randn(30, 64), max_length=3, temperature=0.0)  # prefill 150 rows: MX products
            model.generate(torch.randn(40, 64), max_length=3, num_beams=4)  # beam rows 160: MX steps + head
        _assert_clean(rec)
        names = [c[0] for c in rec.calls]
        gemms = [c[1][0]._obj for c in rec.calls if c[0] == "icap_gemm"]
    assert names.count("icap_quantize_mx") >= 2 * 8 + 2  # 4 fwd + 4 bwd products per layer, LM head fwd + dX
    assert sum(g.in_dtype == 2 for g in gemms) >= 2 * 8 + 2
