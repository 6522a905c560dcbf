"""ImageCaptioningModel on the icap HIP path — drop-in for src/models.py:177-547.

Same constructor signature, attributes (`mapping_network`, `gpt`, `tokenizer`,
`image_prefix_length`, `task_prefix_embeds`), methods (`forward`, `generate`,
`generate_captions`, `save_parameters`, `load_saved_parameters`) and checkpoint key
names. `forward` is differentiable through a custom autograd Function whose
forward/backward are the explicit kernel schedules of GPT2Core/MapperCore, so a
reference-style loop (`outputs.loss.backward(); clip_grad_norm_; optimizer.step()`)
works unchanged; icap.train.train() uses the fused CaptionTrainer instead.
"""

from __future__ import annotations

import os
from types import SimpleNamespace
from typing import List, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import ops
from .gpt2 import GPT2Config, GPT2LMHeadModel
from .mapper import DWHelper, MLPMapperCore, MLPMappingNetwork, TransformerMapperCore, TransformerMappingNetwork
from .weights import FlatParams, named_trainable

Tensor = torch.Tensor


def load_gpt2_tokenizer(path: Optional[str] = None):
    """src/utils.py:94-104: GPT2Tokenizer with pad = eos. Needs a local vocab (no network here)."""
    from transformers import GPT2Tokenizer

    tok = GPT2Tokenizer.from_pretrained(path or "gpt2")
    tok.pad_token = tok.eos_token
    return tok


class ImageCaptioningModel(nn.Module):
    def __init__(self, mapping_network: nn.Module, image_prefix_length: Optional[int] = None,
                 prefix_task_prompt: Optional[str] = None, tokenizer=None, gpt: Optional[GPT2LMHeadModel] = None,
                 freeze_gpt_weights: bool = True, compute_dtype: torch.dtype = torch.bfloat16,
                 gpt_fp8: bool = False) -> None:
        super().__init__()
        self.image_prefix_length = image_prefix_length or mapping_network.prefix_length
        self.mapping_network = mapping_network
        self.gpt = gpt if gpt is not None else GPT2LMHeadModel.from_pretrained("gpt2")  # src/models.py:211
        self.gpt_embedding_size = self.gpt.transformer.wte.weight.shape[1]
        if tokenizer is None:
            try:
                tokenizer = load_gpt2_tokenizer()
            except Exception:  # offline: only eos_token_id is needed by generate (src/models.py:348)
                tokenizer = SimpleNamespace(eos_token_id=self.gpt.config.eos_token_id, eos_token="<|endoftext|>")
        self.tokenizer = tokenizer
        self.freeze_gpt_weights = freeze_gpt_weights
        for p in self.gpt.parameters():  # src/models.py:216-217
            p.requires_grad = not freeze_gpt_weights
        self.task_prefix_embeds: Optional[nn.Parameter] = None
        if prefix_task_prompt:  # src/models.py:221-235
            ids = self.tokenizer.encode(prefix_task_prompt, return_tensors="pt")
            with torch.no_grad():
                emb = self.gpt.transformer.wte.weight[ids.reshape(-1)].clone()
            self.task_prefix_embeds = nn.Parameter(emb, requires_grad=True)
        self.compute_dtype = compute_dtype
        # BASELINE configs[4]: the frozen GPT-2's training / forward products as MX fp8 GEMMs (icap.gpt2.GPT2Core)
        if gpt_fp8 and (not freeze_gpt_weights or compute_dtype != torch.bfloat16):
            raise ValueError("gpt_fp8 needs freeze_gpt_weights=True and compute_dtype=torch.bfloat16")
        self.gpt.fp8_mx = bool(gpt_fp8)
        self._flat: Optional[FlatParams] = None
        self._synced_version = None
        self._fwd_cache = {}

    # -- storage ------------------------------------------------------------------------------------------------
    @property
    def device(self) -> torch.device:
        return self.gpt.transformer.wte.weight.device

    @property
    def total_prefix_length(self) -> int:
        n = self.mapping_network.prefix_length
        return n + (self.task_prefix_embeds.shape[0] if self.task_prefix_embeds is not None else 0)

    def flat(self) -> FlatParams:
        """Flatten the trainable parameters into one fp32 buffer on the model's device (first use)."""
        if self._flat is None or self._flat.flat.device != self.device:
            named = named_trainable(self)
            self._flat = FlatParams(named, self.device, self.compute_dtype)
            self._flat.sync_compute_copy()
            self._synced_version = self._flat.flat._version
            self.mapping_network._core = None
        return self._flat

    @torch.no_grad()
    def sync_compute_copies(self) -> None:
        """Refresh compute copies after an external in-place update of the fp32 masters (torch optimizer,
        load_state_dict). The fused AdamW writes them itself, so this is a no-op in icap.train."""
        f = self.flat()
        if f.flat._version != self._synced_version:
            f.sync_compute_copy()
            self.mapping_network.core(self.compute_dtype, f).refresh_transposes()
            if not self.freeze_gpt_weights:
                self.gpt.invalidate_core()
            self._synced_version = f.flat._version

    def _mcore(self):
        return self.mapping_network.core(self.compute_dtype, self.flat())

    def _gcore(self):
        if not self.freeze_gpt_weights:
            self.gpt.invalidate_core()
        return self.gpt.core(self.compute_dtype)

    def _prefix(self, mcore, mws, B: int):
        """(prefix tensor, batch stride) incl. the optional task prefix (src/models.py:269-283)."""
        pre, pbs = mcore.prefix_view(mws)
        if self.task_prefix_embeds is None:
            return pre, pbs
        D, Pm, P = self.gpt_embedding_size, mcore.P, self.total_prefix_length
        out = torch.empty((B, P, D), dtype=self.compute_dtype, device=self.device)
        ops.convert(pre.as_strided((B, Pm * D), (pbs, 1)), out.view(B, P * D)[:, : Pm * D])
        ops.broadcast_rows(self.task_prefix_embeds.data, out.view(-1)[Pm * D:], B, P * D)
        return out, P * D

    # -- forward ------------------------------------------------------------------------------------------------
    def forward(self, caption_token_ids: Tensor, image_embeddings: Tensor, attention_mask: Optional[Tensor] = None,
                labels: Optional[Tensor] = None):
        """src/models.py:237-325 — returns an object with .loss (if labels) and .logits [B, P+L, V] (fp32)."""
        self.sync_compute_copies()
        flat = self.flat()
        if torch.is_grad_enabled() and labels is not None and flat.n > 16:
            loss, logits = _CaptionFn.apply(self, caption_token_ids, image_embeddings, attention_mask, labels,
                                            *flat.params)
            return SimpleNamespace(loss=loss, logits=logits)
        return self._forward_nograd(caption_token_ids, image_embeddings, attention_mask, labels)

    @torch.no_grad()
    def _forward_nograd(self, ids, emb, mask, labels):
        st = self._run_forward(ids, emb, mask, labels, train=False, keep=False)
        return SimpleNamespace(loss=st.loss, logits=st.logits)

    def _run_forward(self, ids, emb, mask, labels, train: bool, keep: bool):
        B, Lc = ids.shape
        mc, gc = self._mcore(), self._gcore()
        st = SimpleNamespace(B=B, Lc=Lc, mc=mc, gc=gc)
        st.ids = ids.to(self.device, torch.int64).contiguous()
        st.mask = mask.to(self.device, torch.int64).contiguous() if mask is not None else None
        st.labels = labels.to(self.device, torch.int64).contiguous() if labels is not None else None
        st.emb_c = emb.to(self.device).to(self.compute_dtype).contiguous()
        st.mws = mc.alloc(B, train=keep)
        P = self.total_prefix_length
        st.gws = gc.alloc_train(B, P, Lc, keep_for_dw=keep and not self.freeze_gpt_weights)
        seed = int(torch.randint(0, 2 ** 62, (1,)).item()) if train else 0
        p_map = 0.1 if (train and isinstance(mc, TransformerMapperCore)) else 0.0
        st.mdr = mc.drops(train, p_map, seed, None, B)
        st.gdr = gc.drops(train, seed, None, st.gws.M, B, st.gws.S)
        mc.forward(st.mws, st.emb_c, st.mdr, train=keep)
        pre, pbs = self._prefix(mc, st.mws, B)
        gc.forward_train(st.gws, pre, pbs, st.ids, st.mask, st.labels, st.gdr, fuse_dlogits=False)
        st.loss = st.gws.loss[0].clone() if labels is not None else None
        S = st.gws.S
        st.logits = st.gws.logits[:, : gc.V].float().reshape(B, S, gc.V)
        return st

    def _backward(self, st, grad_scale: float) -> List[Tensor]:
        flat = self.flat()
        flat.flat_grad.zero_()
        mc, gc, B = st.mc, st.gc, st.B
        D, P = self.gpt_embedding_size, self.total_prefix_length
        gws = st.gws
        dlog = torch.empty_like(gws.logits)
        ops.cross_entropy(gws.logits, gc.V, gws.labels_shift, gws.n_valid, gws.loss, dlog, gws.ce_ws, grad_scale)
        S = gws.S
        max_rows = max(st.mws.M, B, gws.M if not self.freeze_gpt_weights else 0)
        cols = max(4 * D, 3 * D, mc.E, mc.dw_cols(), (gc.V if not self.freeze_gpt_weights else 0))
        dwh = DWHelper(self.compute_dtype, self.device, max_rows, cols, max(st.mws.M, gws.M), D,
                       colsum_cols=S * D)
        ggrads = self._gpt_grads(flat) if not self.freeze_gpt_weights else None
        d_emb = gc.backward(gws, st.gdr, gws.key_mask if st.mask is not None else None, dlog, grads=ggrads,
                            dw=dwh if ggrads is not None else None)
        if ggrads is not None:
            _embedding_grads(d_emb, st.ids, B, P, st.Lc, D, ggrads, dwh)
        d_pre = d_emb.view(B, S * D)[:, : P * D]
        Pm = mc.P
        if self.task_prefix_embeds is not None:
            ops.colsum(d_emb.view(B, S * D)[:, Pm * D: P * D], flat.grad(self.task_prefix_embeds).view(-1),
                       dwh.cs_ws, accumulate=True, M=B, N=(P - Pm) * D)
        mg = mc.grads(flat)
        if isinstance(mc, TransformerMapperCore):
            ws = st.mws
            ops.convert(d_pre[:, : Pm * D], ws.dout.view(B, mc.S * D)[:, mc.Hl * D:])
            mc.backward(ws, st.emb_c, st.mdr, mg, dwh)
        else:
            mc.backward_from(d_pre[:, : Pm * D], S * D, st.mws, st.emb_c, mg, dwh)
        return [g.clone() for g in flat.grad_views]

    def _gpt_grads(self, flat):
        t = self.gpt.transformer
        g = SimpleNamespace(wte=flat.grad(t.wte.weight), wpe=flat.grad(t.wpe.weight),
                            lnf_g=flat.grad(t.ln_f.weight), lnf_b=flat.grad(t.ln_f.bias), layers=[])
        for blk in t.h:
            g.layers.append(SimpleNamespace(
                w_attn=flat.grad(blk.attn.c_attn.weight), b_attn=flat.grad(blk.attn.c_attn.bias),
                w_proj=flat.grad(blk.attn.c_proj.weight), b_proj=flat.grad(blk.attn.c_proj.bias),
                w_fc=flat.grad(blk.mlp.c_fc.weight), b_fc=flat.grad(blk.mlp.c_fc.bias),
                w_mp=flat.grad(blk.mlp.c_proj.weight), b_mp=flat.grad(blk.mlp.c_proj.bias),
                ln1_g=flat.grad(blk.ln_1.weight), ln1_b=flat.grad(blk.ln_1.bias),
                ln2_g=flat.grad(blk.ln_2.weight), ln2_b=flat.grad(blk.ln_2.bias)))
        return g

    # -- decode -------------------------------------------------------------------------------------------------
    @torch.no_grad()
    def generate(self, image_embeddings: Tensor, max_length: int = 50, temperature: float = 1.0,
                 top_p: float = 0.9, early_exit: bool = True, num_beams: int = 1,
                 length_penalty: float = 1.0) -> Tensor:
        """src/models.py:327-477: greedy (temperature == 0) or top-p sampling, KV-cached. early_exit=False keeps
        decoding all max_length steps on the device (output identical; used to time fixed-length captions).
        num_beams > 1 (an extension; the reference has no beam search): transformers' beam search over the
        caption prefix (GPT2LMHeadModel.generate(num_beams=..., do_sample=False), HF/generation/utils.py:
        3208-3540; temperature / top_p are ignored), SURVEY.md §8f row f4."""
        self.eval()
        self.sync_compute_copies()
        B = image_embeddings.shape[0]
        mc, gc = self._mcore(), self._gcore()
        emb_c = image_embeddings.to(self.device).to(self.compute_dtype).contiguous()
        mws = mc.alloc(B, train=False)
        mc.forward(mws, emb_c, mc.drops(False, 0.0, 0, None, B), train=False)
        pre, pbs = self._prefix(mc, mws, B)
        P, D = self.total_prefix_length, self.gpt_embedding_size
        prefix = pre.as_strided((B, P, D), (pbs, D, 1))
        if num_beams > 1:
            return gc.beam_decode(prefix, max_length, num_beams=num_beams, length_penalty=length_penalty,
                                  early_exit=early_exit)
        if temperature == 0:
            return gc.greedy_decode(prefix, max_length, early_exit=early_exit)
        if temperature < 0:  # src/models.py:401-407: divide by 1.0 and skip the top-p filter (full softmax draw)
            temperature, top_p = 1.0, 1.0
        return gc.sample_decode(prefix, max_length, temperature, top_p)

    def generate_captions(self, image_embeddings: Tensor, **kwargs) -> List[str]:
        ids = self.generate(image_embeddings, **kwargs)
        return self.tokenizer.batch_decode(ids, skip_special_tokens=True)

    # -- checkpoints (src/models.py:489-547) ---------------------------------------------------------------------
    def save_parameters(self, output_path: str) -> None:
        trainable = {n for n, p in self.named_parameters() if p.requires_grad}
        keys = {}
        for name, t in self.state_dict().items():
            if name in trainable or not name.startswith("gpt."):
                keys[name] = t.detach().clone()
        print(f"Saving {len(keys)} trainable parameters and buffers to {output_path}.")
        torch.save(keys, output_path)

    def load_saved_parameters(self, checkpoint_path: str, device: Optional[torch.device] = None) -> None:
        state = torch.load(checkpoint_path, map_location=device or self.device, weights_only=True)
        keys = self.load_state_dict(state, strict=False)
        if keys.unexpected_keys:
            raise ValueError(f"Unexpected keys found in the checkpoint: {keys.unexpected_keys}")
        non_gpt = [k for k in keys.missing_keys if not k.startswith("gpt.")]
        if non_gpt:
            raise ValueError(f"Missing keys found in the checkpoint that are not from frozen GPT weights: {non_gpt}")
        if not self.freeze_gpt_weights:
            self.gpt.invalidate_core()


def _embedding_grads(d_emb: Tensor, ids: Tensor, B: int, P: int, Lc: int, D: int, g, dwh: DWHelper) -> None:
    """Unfrozen GPT-2: d(wpe)[t] += sum_b dX[b,t]; d(wte)[ids] += dX caption rows (modeling_gpt2.py:571-577,
    src/models.py:261)."""
    S = P + Lc
    ops.colsum(d_emb.view(B, S * D), g.wpe[:S].reshape(-1), dwh.cs_ws, accumulate=True, M=B, N=S * D)
    ops.embedding_scatter_add(d_emb, ids, g.wte, B=B, P=P, L_=Lc, D=D)


class _CaptionFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, model: ImageCaptioningModel, ids, emb, mask, labels, *params):
        st = model._run_forward(ids, emb, mask, labels, train=model.training, keep=True)
        ctx.model = model
        ctx.st = st
        ctx.mark_non_differentiable(st.logits)
        return st.loss, st.logits

    @staticmethod
    def backward(ctx, g_loss, g_logits):
        scale = float(g_loss.item()) if g_loss is not None else 0.0
        grads = ctx.model._backward(ctx.st, scale)
        ctx.st = None
        return (None, None, None, None, None, *grads)
