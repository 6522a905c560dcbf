"""GPT-2 LM (HF GPT2LMHeadModel surface) on the icap HIP kernels.

Reference: the reference wraps HF GPT2LMHeadModel (src/models.py:211) and reaches
its arithmetic through `gpt.forward(inputs_embeds=, labels=, attention_mask=)`
(src/models.py:321-325, :395) and `gpt.transformer.wte` (src/models.py:212,261,466).
This module keeps that surface. `GPT2Core` holds the weights in the two GEMM
orientations the kernels want (forward: [out,in]; backward dX: HF Conv1D [in,out])
and implements the forward, the dX(/dW) backward and the KV-cached decode step as
explicit kernel schedules (no autograd, no torch compute).
"""

from __future__ import annotations

import math
import os
from dataclasses import dataclass
from types import SimpleNamespace
from typing import List, Optional

import torch
import torch.nn as nn

from . import _lib as L
from . import ops
from .ops import Dropout
from .weights import det_tensor

# decode steps (M <= 128) of a frozen GPT-2: ln_1 / ln_2 folded into the QKV / c_fc weights (GPT2Core._fold_ln);
# False keeps the LayerNorm-fused GEMMs (module constant, not process environment: A/B tools and tests set it)
LN_FOLD = True
# training / inference forward of a frozen bf16 GPT-2 (and the CLIP tower, clip.ClipCore): ln_1 (layers >= 1) and
# ln_2 folded into the QKV / c_fc tile GEMMs, their row statistics handed over from the producing GEMMs' epilogues
# (icap_gemm_args.ln_stats_out / ln_stats_in); False keeps the standalone LayerNorm launches
TRAIN_LN_FOLD = True

Tensor = torch.Tensor


_CUS = {}


def _device_cus(dev) -> int:
    """Compute units of the device (the split rule of the LM head dX)."""
    if dev.type != "cuda" or not torch.cuda.is_available():
        return 256  # (the CPU dry run of the schedules: MI355X's count)
    i = dev.index if dev.index is not None else torch.cuda.current_device()
    if i not in _CUS:
        _CUS[i] = int(torch.cuda.get_device_properties(i).multi_processor_count)
    return _CUS[i]


@dataclass
class GPT2Config:  # HF/models/gpt2/configuration_gpt2.py:84-103
    vocab_size: int = 50257
    n_positions: int = 1024
    n_embd: int = 768
    n_layer: int = 12
    n_head: int = 12
    layer_norm_epsilon: float = 1e-5
    resid_pdrop: float = 0.1
    embd_pdrop: float = 0.1
    attn_pdrop: float = 0.1
    eos_token_id: int = 50256

    @classmethod
    def medium(cls):  # BASELINE configs[3]
        return cls(n_embd=1024, n_layer=24, n_head=16)

    @classmethod
    def large(cls):  # BASELINE configs[4]
        return cls(n_embd=1280, n_layer=36, n_head=20)


def pad_vocab(v: int) -> int:
    return (v + 127) // 128 * 128


def fold_layernorm(wt: Tensor, gamma: Tensor, beta: Tensor, bias: Tensor, dtype: torch.dtype):
    """LayerNorm(x) . W^T + b = rstd (x . (W*gamma)^T - mean * wsum) + (b + W . beta) for an fp32 weight wt [out,in]
    (nn.Linear layout): returns (W*gamma [out,in] in the compute dtype, wsum [out] = row sums of those stored values,
    b + W . beta [out]), all fp32 arithmetic on the MFMA GEMM (W*gamma = W . diag(gamma): one nonzero product per
    output, exact before the rounding to the compute dtype). Used once per frozen model (the decode / training-forward
    ln_1 / ln_2 folds of GPT-2, CLIP's layer_norm1 / layer_norm2)."""
    nout, nin = wt.shape
    dev = wt.device
    dg = torch.zeros((nin, nin), dtype=torch.float32, device=dev)
    dg.view(-1)[:: nin + 1].copy_(gamma)
    wg = torch.empty((nout, nin), dtype=torch.float32, device=dev)
    ops.gemm(wt.contiguous(), dg, wg, split_k=1)
    if dtype == torch.float32:
        wf = wg
    else:
        wf = torch.empty((nout, nin), dtype=dtype, device=dev)
        ops.convert(wg, wf)
    ones = torch.ones((1, nin), dtype=dtype, device=dev)
    wsum = torch.empty((1, nout), dtype=torch.float32, device=dev)
    ops.gemm(ones, wf, wsum, split_k=1)
    bf = torch.empty((1, nout), dtype=torch.float32, device=dev)
    ops.gemm(beta.reshape(1, nin).contiguous(), wt.contiguous(), bf, bias=bias, split_k=1)
    return wf, wsum.view(nout), bf.view(nout)


# --------------------------------------------------------------------------- parameter containers (HF names)


class Conv1D(nn.Module):
    """HF/pytorch_utils.py:95-121 storage: weight [in, out], bias [out]."""

    def __init__(self, nx: int, nf: int):
        super().__init__()
        self.weight = nn.Parameter(torch.zeros(nx, nf))
        self.bias = nn.Parameter(torch.zeros(nf))


class _Attn(nn.Module):
    def __init__(self, d):
        super().__init__()
        self.c_attn = Conv1D(d, 3 * d)
        self.c_proj = Conv1D(d, d)


class _MLP(nn.Module):
    def __init__(self, d):
        super().__init__()
        self.c_fc = Conv1D(d, 4 * d)
        self.c_proj = Conv1D(4 * d, d)


class _Block(nn.Module):
    def __init__(self, d, eps):
        super().__init__()
        self.ln_1 = nn.LayerNorm(d, eps=eps)
        self.attn = _Attn(d)
        self.ln_2 = nn.LayerNorm(d, eps=eps)
        self.mlp = _MLP(d)


class _Transformer(nn.Module):
    def __init__(self, cfg: GPT2Config):
        super().__init__()
        d = cfg.n_embd
        self.wte = nn.Embedding(cfg.vocab_size, d)
        self.wpe = nn.Embedding(cfg.n_positions, d)
        self.h = nn.ModuleList([_Block(d, cfg.layer_norm_epsilon) for _ in range(cfg.n_layer)])
        self.ln_f = nn.LayerNorm(d, eps=cfg.layer_norm_epsilon)


class GPT2LMHeadModel(nn.Module):
    """Drop-in for the `gpt=` argument of ImageCaptioningModel (src/models.py:189,211).

    `.forward(inputs_embeds=, labels=, attention_mask=)` runs the HIP forward (inference) and returns an object
    with `.loss` and `.logits` like HF's CausalLMOutputWithCrossAttentions."""

    def __init__(self, config: Optional[GPT2Config] = None):
        super().__init__()
        self.config = config or GPT2Config()
        self.transformer = _Transformer(self.config)
        self.lm_head = nn.Linear(self.config.n_embd, self.config.vocab_size, bias=False)
        self.lm_head.weight = self.transformer.wte.weight  # tied (modeling_gpt2.py:638)
        # BASELINE configs[4]'s fp8 path: the frozen model's training / prefill-forward and dX products run as MX
        # block-scaled e4m3 GEMMs (weights quantised once, activations before each product); bf16 compute only
        self.fp8_mx = False
        self._core: Optional["GPT2Core"] = None
        self._core_key = None

    @classmethod
    def random_init(cls, config: Optional[GPT2Config] = None, seed: int = 0) -> "GPT2LMHeadModel":
        """Deterministic random weights of the GPT-2 architecture (no pretrained checkpoint is available offline)."""
        m = cls(config)
        cfg = m.config
        d, nl = cfg.n_embd, cfg.n_layer
        proj_std = 0.02 / math.sqrt(2 * nl)
        with torch.no_grad():
            t = m.transformer
            t.wte.weight.copy_(det_tensor(seed, "wte", (cfg.vocab_size, d), 0.02))
            t.wpe.weight.copy_(det_tensor(seed, "wpe", (cfg.n_positions, d), 0.01))
            t.ln_f.weight.copy_(det_tensor(seed, "ln_f.w", (d,), 0.05, 1.0))
            t.ln_f.bias.copy_(det_tensor(seed, "ln_f.b", (d,), 0.02))
            for i, blk in enumerate(t.h):
                p = f"transformer.h.{i}."
                blk.ln_1.weight.copy_(det_tensor(seed, p + "ln_1.w", (d,), 0.05, 1.0))
                blk.ln_1.bias.copy_(det_tensor(seed, p + "ln_1.b", (d,), 0.02))
                blk.attn.c_attn.weight.copy_(det_tensor(seed, p + "c_attn.w", (d, 3 * d), 0.02))
                blk.attn.c_attn.bias.copy_(det_tensor(seed, p + "c_attn.b", (3 * d,), 0.02))
                blk.attn.c_proj.weight.copy_(det_tensor(seed, p + "attn.c_proj.w", (d, d), proj_std))
                blk.attn.c_proj.bias.copy_(det_tensor(seed, p + "attn.c_proj.b", (d,), 0.02))
                blk.ln_2.weight.copy_(det_tensor(seed, p + "ln_2.w", (d,), 0.05, 1.0))
                blk.ln_2.bias.copy_(det_tensor(seed, p + "ln_2.b", (d,), 0.02))
                blk.mlp.c_fc.weight.copy_(det_tensor(seed, p + "c_fc.w", (d, 4 * d), 0.02))
                blk.mlp.c_fc.bias.copy_(det_tensor(seed, p + "c_fc.b", (4 * d,), 0.02))
                blk.mlp.c_proj.weight.copy_(det_tensor(seed, p + "mlp.c_proj.w", (4 * d, d), proj_std))
                blk.mlp.c_proj.bias.copy_(det_tensor(seed, p + "mlp.c_proj.b", (d,), 0.02))
        return m

    @classmethod
    def from_pretrained(cls, path: str) -> "GPT2LMHeadModel":
        """Load an HF GPT-2 checkpoint from a LOCAL directory or file (model.safetensors / pytorch_model.bin +
        config.json). There is no network access: hub names only resolve through a local HF cache."""
        import json
        import os

        cand = path
        if not os.path.exists(cand):
            try:
                from huggingface_hub import snapshot_download

                cand = snapshot_download(path, local_files_only=True)
            except Exception as e:  # noqa: BLE001
                raise FileNotFoundError(
                    f"GPT-2 checkpoint '{path}' is not available locally (offline); pass gpt= explicitly, e.g. "
                    "icap.GPT2LMHeadModel.random_init()") from e
        cfg = GPT2Config()
        if os.path.isdir(cand):
            cj = os.path.join(cand, "config.json")
            if os.path.exists(cj):
                with open(cj) as f:
                    j = json.load(f)
                for k in ("vocab_size", "n_positions", "n_embd", "n_layer", "n_head", "layer_norm_epsilon",
                          "resid_pdrop", "embd_pdrop", "attn_pdrop", "eos_token_id"):
                    if k in j:
                        setattr(cfg, k, j[k])
            st = os.path.join(cand, "model.safetensors")
            cand = st if os.path.exists(st) else os.path.join(cand, "pytorch_model.bin")
        if cand.endswith(".safetensors"):
            from safetensors.torch import load_file

            sd = load_file(cand)
        else:
            sd = torch.load(cand, map_location="cpu", weights_only=True)
        sd = {(k if k.startswith(("transformer.", "lm_head.")) else "transformer." + k): v for k, v in sd.items()
              if not k.endswith((".attn.bias", ".attn.masked_bias"))}
        m = cls(cfg)
        m.load_state_dict(sd, strict=False)
        return m

    def core(self, dtype: torch.dtype) -> "GPT2Core":
        dev = self.transformer.wte.weight.device
        key = (dtype, dev, bool(self.fp8_mx))
        if self._core is None or self._core_key != key:
            self._core = GPT2Core(self, dtype)
            self._core_key = key
        return self._core

    def invalidate_core(self):
        self._core = None

    def forward(self, inputs_embeds: Tensor, labels: Optional[Tensor] = None, attention_mask: Optional[Tensor] = None,
                compute_dtype: Optional[torch.dtype] = None, **_):
        """Inference forward on the HIP path (modeling_gpt2.py:650-725 semantics, dropout off)."""
        dt = compute_dtype or (inputs_embeds.dtype if inputs_embeds.dtype in (torch.float32, torch.bfloat16)
                               else torch.float32)
        core = self.core(dt)
        return core.forward_infer(inputs_embeds, attention_mask, labels)


# --------------------------------------------------------------------------- compute core


class _LayerW(SimpleNamespace):
    pass


class GPT2Core:
    """GEMM-layout weights + kernel schedules for one GPT2LMHeadModel in one compute dtype."""

    def __init__(self, model: GPT2LMHeadModel, dtype: torch.dtype):
        self.model = model
        self.cfg = model.config
        self.dtype = dtype
        self.dev = model.transformer.wte.weight.device
        from ._lib import require_device

        require_device(self.dev)
        c = self.cfg
        self.D, self.H = c.n_embd, c.n_head
        self.hd = self.D // self.H
        self.V = c.vocab_size
        self.Vp = pad_vocab(self.V)
        self.fp8 = bool(getattr(model, "fp8_mx", False))
        if self.fp8 and (dtype != torch.bfloat16 or self.D % 128):
            raise L.IcapError("fp8_mx needs the bf16 compute dtype and n_embd % 128 == 0")
        self.layers: List[_LayerW] = []
        self.refresh()

    # -- weights ---------------------------------------------------------------------------------------
    def _both(self, w: Tensor):
        """HF Conv1D master [in,out] fp32 -> (fwd [out,in], bwd [in,out]) in the compute dtype."""
        nin, nout = w.shape
        fwd = torch.empty((nout, nin), dtype=self.dtype, device=self.dev)
        if self.dtype == torch.float32:
            bwd = w.data
            ops.transpose(bwd, fwd)
        else:
            bwd = torch.empty((nin, nout), dtype=self.dtype, device=self.dev)
            ops.convert(w.data, bwd)
            ops.transpose(bwd, fwd)
        return fwd, bwd

    @torch.no_grad()
    def refresh(self) -> None:
        """(Re)build the compute copies from the fp32 masters (once when frozen; after each step when trained)."""
        t = self.model.transformer
        self.layers = []
        for blk in t.h:
            lw = _LayerW()
            lw.w_attn_t, lw.w_attn = self._both(blk.attn.c_attn.weight)
            lw.w_proj_t, lw.w_proj = self._both(blk.attn.c_proj.weight)
            lw.w_fc_t, lw.w_fc = self._both(blk.mlp.c_fc.weight)
            lw.w_mp_t, lw.w_mp = self._both(blk.mlp.c_proj.weight)
            lw.b_attn, lw.b_proj = blk.attn.c_attn.bias.data, blk.attn.c_proj.bias.data
            lw.b_fc, lw.b_mp = blk.mlp.c_fc.bias.data, blk.mlp.c_proj.bias.data
            lw.ln1_g, lw.ln1_b = blk.ln_1.weight.data, blk.ln_1.bias.data
            lw.ln2_g, lw.ln2_b = blk.ln_2.weight.data, blk.ln_2.bias.data
            self.layers.append(lw)
        self.lnf_g, self.lnf_b = t.ln_f.weight.data, t.ln_f.bias.data
        D, V, Vp = self.D, self.V, self.Vp
        self.wte = torch.zeros((Vp, D), dtype=self.dtype, device=self.dev)  # LM-head B operand + embedding table
        ops.convert(t.wte.weight.data, self.wte[:V])
        self.wte_t = torch.empty((D, Vp), dtype=self.dtype, device=self.dev)  # LM-head dX B operand
        ops.transpose(self.wte, self.wte_t)
        if self.dtype == torch.float32:
            self.wpe = t.wpe.weight.data
        else:
            self.wpe = torch.empty_like(t.wpe.weight.data, dtype=self.dtype)
            ops.convert(t.wpe.weight.data, self.wpe)
        self.eps = self.cfg.layer_norm_epsilon
        if LN_FOLD:  # decode: ln_1 / ln_2 folded into the QKV / c_fc weights (frozen weights: once)
            for blk, lw in zip(t.h, self.layers):
                lw.wf_attn_t, lw.ws_attn, lw.bf_attn = self._fold_ln(blk.attn.c_attn.weight.data, lw.ln1_g,
                                                                     lw.ln1_b, lw.b_attn)
                lw.wf_fc_t, lw.ws_fc, lw.bf_fc = self._fold_ln(blk.mlp.c_fc.weight.data, lw.ln2_g, lw.ln2_b,
                                                               lw.b_fc)
        if self.fp8:  # MX e4m3 copies of every frozen product's weight operand, both orientations
            for lw in self.layers:
                for nm in ("w_attn", "w_proj", "w_fc", "w_mp"):
                    setattr(lw, "q" + nm + "_t", ops.quantize_mx(getattr(lw, nm + "_t")))
                    setattr(lw, "q" + nm, ops.quantize_mx(getattr(lw, nm)))
            self.qwte = ops.quantize_mx(self.wte)
            self.qwte_t = ops.quantize_mx(self.wte_t)

    def _fold_ln(self, w: Tensor, gamma: Tensor, beta: Tensor, bias: Tensor):
        """fold_layernorm of a Conv1D master w [in,out] (fp32): its [out,in] transpose folded."""
        nin, nout = w.shape
        wt = torch.empty((nout, nin), dtype=torch.float32, device=self.dev)
        ops.transpose(w, wt)
        return fold_layernorm(wt, gamma, beta, bias, self.dtype)

    @torch.no_grad()
    def bind_flat(self, flat) -> None:
        """Trainable GPT-2 in the fused trainer: read every weight from the flat parameter storage (fp32 masters
        and the compute-dtype copy the AdamW kernel writes), so an optimizer step updates this core in place.
        The [in,out] (dX) orientation, wpe and the fp32 biases / LayerNorm parameters are views of that storage;
        the [out,in] (forward) transposes and the padded LM-head table are copies that refresh_from_flat()
        rewrites in place (HIP-graph capturable) after each step."""
        if self.fp8:
            raise L.IcapError("fp8_mx is the frozen-GPT-2 path (weights quantised once); train GPT-2 in bf16")
        t = self.model.transformer
        for blk, lw in zip(t.h, self.layers):
            lw.wf_attn_t = lw.wf_fc_t = None  # trained weights: decode keeps ln_1 / ln_2 in the GEMMs (no fold)
            lw.w_attn, lw.w_proj = flat.view_c(blk.attn.c_attn.weight), flat.view_c(blk.attn.c_proj.weight)
            lw.w_fc, lw.w_mp = flat.view_c(blk.mlp.c_fc.weight), flat.view_c(blk.mlp.c_proj.weight)
            lw.b_attn, lw.b_proj = blk.attn.c_attn.bias.data, blk.attn.c_proj.bias.data
            lw.b_fc, lw.b_mp = blk.mlp.c_fc.bias.data, blk.mlp.c_proj.bias.data
            lw.ln1_g, lw.ln1_b = blk.ln_1.weight.data, blk.ln_1.bias.data
            lw.ln2_g, lw.ln2_b = blk.ln_2.weight.data, blk.ln_2.bias.data
        self.lnf_g, self.lnf_b = t.ln_f.weight.data, t.ln_f.bias.data
        self.wpe = flat.view_c(t.wpe.weight)
        self._wte_c = flat.view_c(t.wte.weight)
        self.refresh_from_flat()

    @torch.no_grad()
    def refresh_from_flat(self) -> None:
        """Rewrite the forward-orientation transposes and the padded LM-head table from the bound storage."""
        for lw in self.layers:
            ops.transpose(lw.w_attn, lw.w_attn_t)
            ops.transpose(lw.w_proj, lw.w_proj_t)
            ops.transpose(lw.w_fc, lw.w_fc_t)
            ops.transpose(lw.w_mp, lw.w_mp_t)
        ops.convert(self._wte_c, self.wte[: self.V])
        ops.transpose(self.wte, self.wte_t)

    # -- workspaces --------------------------------------------------------------------------------------
    def alloc_train(self, B: int, P: int, Lc: int, keep_for_dw: bool = False,
                    compact_head: bool = False, pack: bool = False) -> SimpleNamespace:
        """compact_head: the LM head and CE run on the rows whose shifted label is not -100 only (at most B*Lc;
        the count lives on the device). The loss ignores every other row (HF/loss/loss_utils.py:32-46,
        ignore_index=-100), so their logits feed nothing and their dlogits are exactly 0: loss and gradients are
        those of the full-width head. Needs labels; not with a trainable (tied) wte.
        pack (with compact_head): the blocks run on packed token rows — each sequence's prefix and caption
        positions up to its last loss target (icap_caption_pack), the rest of the [B, P + Lc] grid is dead under
        the causal mask — so every block GEMM, LayerNorm and attention launch covers the live rows only (row
        count on the device; launches sized for the padded grid, so one captured graph serves every batch)."""
        S = P + Lc
        M = B * S
        D, H, dt, dev = self.D, self.H, self.dtype, self.dev
        nl = self.cfg.n_layer
        e = lambda *shape, dtype=dt: torch.empty(shape, dtype=dtype, device=dev)  # noqa: E731
        ws = SimpleNamespace(B=B, P=P, Lc=Lc, S=S, M=M)
        ws.compact = bool(compact_head and Lc > 0 and not keep_for_dw)
        ws.Mh = B * Lc if ws.compact else M  # rows of the LM head / CE buffers
        ws.head_rows_hint = None  # host-known number of target rows (roofline bookkeeping only)
        ws.pack = bool(pack and ws.compact)
        ws.live_rows_hint = None  # host-known number of packed rows (roofline bookkeeping only)
        ws.seq_sq_hint = None  # host-known sum of squared packed sequence lengths (attention FLOPs, bookkeeping only)
        ws.short_only = False  # every packed sequence of the loaded batch <= 32 tokens (set per batch by the trainer)
        ws.seqs = ws.m_live = None
        if ws.pack:
            ws.seq_off = e(B, dtype=torch.int32)
            ws.seq_len = e(B, dtype=torch.int32)
            ws.m_live = e(1, dtype=torch.int32)
            ws.seqs = (ws.seq_off, ws.seq_len)
            ws.d_emb = e(M, D)  # the prefix rows' gradient back in the padded [B, S, D] layout
        ws.x = [e(M, D) for _ in range(nl + 1)]
        ws.h1 = [e(M, D) for _ in range(nl)]
        ws.qkv = [e(M, 3 * D) for _ in range(nl)]
        ws.z = [e(M, 4 * D) for _ in range(nl)]
        ws.mean1 = [e(M, dtype=torch.float32) for _ in range(nl)]
        ws.rstd1 = [e(M, dtype=torch.float32) for _ in range(nl)]
        ws.mean2 = [e(M, dtype=torch.float32) for _ in range(nl)]
        ws.rstd2 = [e(M, dtype=torch.float32) for _ in range(nl)]
        ws.lse = [e(B * H * S, dtype=torch.float32) for _ in range(nl)]
        ws.meanf, ws.rstdf = e(M, dtype=torch.float32), e(M, dtype=torch.float32)
        # LayerNorm statistics hand-off of the folded forward (GPT2Core._blocks_fwd_): per row and 32-column group
        # (mean, M2) of x (produced by the MLP c_proj, consumed by the next QKV) and of h1 (attention c_proj -> c_fc)
        ws.st_x = ws.st_h = None
        if self._fold_train(keep_for_dw):
            ws.st_x = e(M, D // 32, 2, dtype=torch.float32)
            ws.st_h = e(M, D // 32, 2, dtype=torch.float32)
        if keep_for_dw:
            ws.a1 = [e(M, D) for _ in range(nl)]
            ws.o = [e(M, D) for _ in range(nl)]
            ws.a2 = [e(M, D) for _ in range(nl)]
            ws.f = [e(M, 4 * D) for _ in range(nl)]
        else:
            a, o, a2, f = e(M, D), e(M, D), e(M, D), e(M, 4 * D)
            ws.a1, ws.o, ws.a2, ws.f = [a] * nl, [o] * nl, [a2] * nl, [f] * nl
        Mh = ws.Mh
        ws.hf = e(Mh, D)
        ws.logits = e(Mh, self.Vp)
        ws.key_mask = e(M, dtype=torch.int32)
        ws.labels_shift = e(M, dtype=torch.int32)
        ws.row_slot = e(M, dtype=torch.int32) if ws.compact else None
        ws.labels_c = e(Mh, dtype=torch.int32) if ws.compact else None
        ws.n_valid = e(1, dtype=torch.int32)
        ws.loss = e(1, dtype=torch.float32)
        ws.ce_ws = e(ops.cross_entropy_workspace(Mh), dtype=torch.uint8)
        # backward scratch
        ws.dx, ws.dx2, ws.dxd = e(M, D), e(M, D), e(M, D)
        ws.dff = e(M, 4 * D)
        ws.dqkv = e(M, 3 * D)
        ws.do, ws.da = e(M, D), e(M, D)
        ws.dhf = e(Mh, D)
        ws.qD = ws.q3D = ws.q4D = ws.qhf = ws.qdl = None
        if self.fp8:  # MX operand buffers (each product quantises its activation operand into one of these)
            mx = lambda R, K: ops.MXTensor.empty(R, K, dev)  # noqa: E731
            ws.qD, ws.q3D, ws.q4D = mx(M, D), mx(M, 3 * D), mx(M, 4 * D)
            ws.qhf, ws.qdl = mx(Mh, D), mx(Mh, self.Vp)
        return ws

    def _fold_train(self, keep_for_dw: bool) -> bool:
        """Whether the forward folds ln_1 / ln_2 into the tile GEMMs: a frozen bf16 model (the folded weights exist),
        not the fp8 path (its MX products have no LayerNorm epilogue), a width the hand-off supports (ops.ln_fold_ok)."""
        return (TRAIN_LN_FOLD and not keep_for_dw and self.dtype == torch.bfloat16 and not self.fp8
                and ops.ln_fold_ok(self.D) and bool(self.layers) and getattr(self.layers[0], "wf_attn_t", None) is not None)

    def _bmm(self, ws, A: Tensor, qA, W: Tensor, qW, out: Tensor, **kw) -> Tensor:
        """A block GEMM over the token rows: with packed rows only rows < m_live are computed (m_dev)."""
        if not ws.pack:
            return self._mm(A, qA, W, qW, out, **kw)
        if ws.live_rows_hint is not None:
            if "alg_flops" not in kw:
                kw["alg_flops"] = 2.0 * ws.live_rows_hint * W.shape[0] * A.shape[1]
            kw["m_hint"] = ws.live_rows_hint  # kernel choice for the expected live rows
        return self._mm(A, qA, W, qW, out, rows_dev=ws.m_live, m_dev=ws.m_live, **kw)

    def _mm(self, A: Tensor, qA, W: Tensor, qW, out: Tensor, rows_dev: Optional[Tensor] = None, **kw) -> Tensor:
        """out = epi(A . W^T): the bf16 / f32 GEMM, or (fp8_mx) quantise A into qA and run the MX product with
        the weight's MX copy qW (same epilogue arguments)."""
        if qA is None:
            return ops.gemm(A, W, out, **kw)
        ops.quantize_mx(A, qA, rows=qA.R, rows_dev=rows_dev)
        return ops.gemm(qA, qW, out, **kw)

    # -- dropout sites (distinct offsets so masks never coincide) -------------------------------------------
    def drops(self, train: bool, seed: int, counter: Optional[Tensor], M: int, B: int, S: int):
        c = self.cfg
        if not train:
            z = Dropout()
            return SimpleNamespace(embd=z, attn=lambda l: z, ra=lambda l: z, rm=lambda l: z)
        D, H = self.D, self.H
        blk = 4 * M * D + B * H * S * S

        def mk(p, off):
            return Dropout(p, seed, off, counter)

        return SimpleNamespace(
            embd=mk(c.embd_pdrop, 0),
            attn=lambda l: mk(c.attn_pdrop, M * D + l * blk),
            ra=lambda l: mk(c.resid_pdrop, M * D + l * blk + B * H * S * S),
            rm=lambda l: mk(c.resid_pdrop, M * D + l * blk + B * H * S * S + M * D),
        )

    # -- training forward ------------------------------------------------------------------------------------
    def forward_train(self, ws, prefix: Tensor, prefix_bstride: int, ids: Tensor, mask: Optional[Tensor],
                      labels: Optional[Tensor], dr, fuse_dlogits: bool, grad_scale: float = 1.0,
                      dlogits: Optional[Tensor] = None) -> None:
        """Embeddings -> 12 blocks -> ln_f -> LM head -> CE (modeling_gpt2.py:514-725 + loss_utils.py:49-71).
        With fuse_dlogits the CE kernel also writes dlogits (in place over the logits, or into `dlogits`)."""
        B, P, Lc, S, M = ws.B, ws.P, ws.Lc, ws.S, ws.M
        D, H, hd = self.D, self.H, self.hd
        cp = ws.compact
        if cp and labels is None:
            raise L.IcapError("compact LM head needs labels")
        if ws.pack:
            ops.caption_pack(B, P, Lc, mask, labels, ws.seq_off, ws.seq_len, ws.m_live, ws.key_mask, ws.labels_shift,
                             ws.n_valid, ws.row_slot, ws.labels_c)
        else:
            ops.caption_prep(B, P, Lc, mask, labels, ws.key_mask, ws.labels_shift, ws.n_valid,
                             ws.row_slot if cp else None, ws.labels_c if cp else None)
        ops.gpt2_embed(prefix, prefix_bstride, self.wte, self.wpe, ids, ws.x[0], B=B, P=P, L_=Lc, D=D, drop=dr.embd,
                       seqs=ws.seqs)
        self._blocks_fwd(ws, dr, B, S, M, causal_mask=ws.key_mask if mask is not None else None)
        ops.layernorm_fwd(ws.x[-1], self.lnf_g, self.lnf_b, self.eps, ws.hf, ws.meanf, ws.rstdf,
                          y_rowmap=ws.row_slot if cp else None, rows_dev=ws.m_live)
        rows = ws.head_rows_hint if (cp and ws.head_rows_hint is not None) else ws.Mh
        self._mm(ws.hf, ws.qhf, self.wte, getattr(self, "qwte", None), ws.logits, rows_dev=ws.n_valid if cp else None,
                 M=ws.Mh, m_dev=ws.n_valid if cp else None, alg_flops=2.0 * rows * self.V * self.D)
        if labels is not None:
            dl = (dlogits if dlogits is not None else ws.logits) if fuse_dlogits else None
            ops.cross_entropy(ws.logits, self.V, ws.labels_c if cp else ws.labels_shift, ws.n_valid, ws.loss, dl,
                              ws.ce_ws, grad_scale, rows=ws.Mh, rows_dev=ws.n_valid if cp else None)

    def _attn_flops(self, ws, B, S, bwd: bool = False) -> Optional[float]:
        """Algorithmic FLOPs of one attention launch (bench timing only): QK^T and PV over each sequence's live
        tokens, dense S x S as the reference's SDPA computes them (4 S^2 hd per head forward; the backward's five
        products 10 S^2 hd); None when no host-side count of the packed lengths is known."""
        sq = getattr(ws, "seq_sq_hint", None)
        if sq is None:
            sq = None if getattr(ws, "pack", False) else B * S * S
        if sq is None:
            return None
        return (10.0 if bwd else 4.0) * sq * self.hd * self.H

    def _blocks_fwd(self, ws, dr, B, S, M, causal_mask):
        with ops.timer_tag("gpt2_block"):
            self._blocks_fwd_(ws, dr, B, S, M, causal_mask)

    def _blocks_fwd_(self, ws, dr, B, S, M, causal_mask):
        D, H, hd = self.D, self.H, self.hd
        scale = 1.0 / math.sqrt(hd)
        rd = getattr(ws, "m_live", None)  # packed rows: device row count (None: every row)
        seqs = getattr(ws, "seqs", None)
        so = bool(getattr(ws, "short_only", False))  # every packed sequence <= 32 tokens (engine.load_batch)
        afl = self._attn_flops(ws, B, S)
        fold = getattr(ws, "st_x", None) is not None  # ln_1 (l >= 1) / ln_2 folded into the QKV / c_fc GEMMs
        nl = len(self.layers)
        for l, lw in enumerate(self.layers):
            x = ws.x[l]
            q = lw if self.fp8 else SimpleNamespace(qw_attn_t=None, qw_proj_t=None, qw_fc_t=None, qw_mp_t=None)
            if fold and l > 0:  # rstd (x . (W gamma)^T - mean wsum) + b + W.beta, x's statistics from the producer
                self._bmm(ws, x, None, lw.wf_attn_t, None, ws.qkv[l], bias=lw.bf_attn, ln_fold=(lw.ws_attn, self.eps),
                          ln_stats_in=ws.st_x, ln_rows_out=(ws.mean1[l], ws.rstd1[l]))
            else:
                ops.layernorm_fwd(x, lw.ln1_g, lw.ln1_b, self.eps, ws.a1[l], ws.mean1[l], ws.rstd1[l], rows_dev=rd)
                self._bmm(ws, ws.a1[l], ws.qD, lw.w_attn_t, q.qw_attn_t, ws.qkv[l], bias=lw.b_attn)
            ops.attention_fwd(ws.qkv[l], ws.o[l], B=B, S=S, H=H, hd=hd, scale=scale, causal=True, key_mask=causal_mask,
                              lse=ws.lse[l], drop=dr.attn(l), seqs=seqs, alg_flops=afl, short_only=so)
            self._bmm(ws, ws.o[l], ws.qD, lw.w_proj_t, q.qw_proj_t, ws.h1[l], bias=lw.b_proj, resid=x, drop=dr.ra(l),
                      **({"ln_stats_out": ws.st_h} if fold else {}))
            if fold:
                self._bmm(ws, ws.h1[l], None, lw.wf_fc_t, None, ws.f[l], bias=lw.bf_fc, act=L.ACT_GELU_NEW,
                          aux=ws.z[l], ln_fold=(lw.ws_fc, self.eps), ln_stats_in=ws.st_h,
                          ln_rows_out=(ws.mean2[l], ws.rstd2[l]))
            else:
                ops.layernorm_fwd(ws.h1[l], lw.ln2_g, lw.ln2_b, self.eps, ws.a2[l], ws.mean2[l], ws.rstd2[l],
                                  rows_dev=rd)
                self._bmm(ws, ws.a2[l], ws.qD, lw.w_fc_t, q.qw_fc_t, ws.f[l], bias=lw.b_fc, act=L.ACT_GELU_NEW,
                          aux=ws.z[l])
            self._bmm(ws, ws.f[l], ws.q4D, lw.w_mp_t, q.qw_mp_t, ws.x[l + 1], bias=lw.b_mp, resid=ws.h1[l],
                      drop=dr.rm(l), **({"ln_stats_out": ws.st_x} if (fold and l + 1 < nl) else {}))

    # -- backward (dX through the frozen GPT-2; + dW when trainable) ---------------------------------------------
    def backward(self, ws, dr, causal_mask, dlogits: Tensor, grads=None, dw=None) -> Tensor:
        """Returns d(inputs_embeds) [M, D] (embedding dropout applied). `grads`: object with per-layer fp32 grad
        views (trainable GPT-2) and `dw`: a DWHelper; both None when GPT-2 is frozen."""
        B, S, M = ws.B, ws.S, ws.M
        D, H, hd = self.D, self.H, self.hd
        scale = 1.0 / math.sqrt(hd)
        nl = len(self.layers)
        cp = ws.compact
        if cp and grads is not None:
            raise L.IcapError("compact LM head: the tied wte gradient needs every row (alloc_train(keep_for_dw))")
        rows = ws.head_rows_hint if (cp and ws.head_rows_hint is not None) else ws.Mh
        # dh_f = dlogits . wte (K padded); compact: target rows only, scattered back by the ln_f backward
        split, rkw = 0, {}
        if cp and rows > 128:  # long K (50304), few output tiles: split K so ~2 blocks/CU work on the live rows
            tiles = -(-rows // 128) * -(-D // 128)
            split = max(1, min(16, round(512 / max(tiles, 1))))
            if dlogits.dtype == torch.bfloat16 and ws.qdl is None:
                # bf16: the 128 x 256 split-role ring, tiles x splits in one round of the CUs (1664 rows: 39 tiles x
                # 6 splits; 127 vs 147 us for the tile kernel at its split, profiles/r06_lmhead_dx_ab.txt)
                t256 = -(-rows // 128) * -(-D // 256)
                split = max(1, min(16, _device_cus(dlogits.device) // max(t256, 1)))
                rkw = dict(roles=256)
        self._mm(dlogits, ws.qdl, self.wte_t, getattr(self, "qwte_t", None), ws.dhf, rows_dev=ws.n_valid if cp else None,
                 M=ws.Mh, m_dev=ws.n_valid if cp else None, alg_flops=2.0 * rows * D * self.V, split_k=split, **rkw)
        if grads is not None:  # d(wte) from the tied LM head: dW[V,D] += dlogits^T . hf
            dw.dW(dlogits, ws.hf, grads.wte, M=M, N=self.V)
        rd, seqs = ws.m_live, ws.seqs  # packed rows (None: every row)
        so = bool(getattr(ws, "short_only", False))
        ops.layernorm_bwd(ws.x[-1], self.lnf_g, ws.meanf, ws.rstdf, ws.dhf, ws.dx, dx_drop=ws.dxd,
                          drop=dr.rm(nl - 1), dgamma=grads.lnf_g if grads else None,
                          dbeta=grads.lnf_b if grads else None, workspace=dw.ln_ws if dw else None,
                          dy_rowmap=ws.row_slot if cp else None, rows_dev=rd)
        dres, dnew = ws.dx, ws.dx2
        afl = self._attn_flops(ws, B, S, bwd=True)
        tag = ops.timer_tag("gpt2_block")
        tag.__enter__()
        for l in reversed(range(nl)):
            lw = self.layers[l]
            g = grads.layers[l] if grads is not None else None
            dy = ws.dxd if dr.rm(l).p > 0 else dres
            if g is not None:
                dw.dW(dy, ws.f[l], g.w_mp, M=M, transpose_out=True)
                dw.db(dy, g.b_mp, M=M)
            q = lw if self.fp8 else SimpleNamespace(qw_attn=None, qw_proj=None, qw_fc=None, qw_mp=None)
            self._bmm(ws, dy, ws.qD, lw.w_mp, q.qw_mp, ws.dff, dact=L.ACT_GELU_NEW, dact_src=ws.z[l])
            if g is not None:
                dw.dW(ws.dff, ws.a2[l], g.w_fc, M=M, transpose_out=True)
                dw.db(ws.dff, g.b_fc, M=M)
            self._bmm(ws, ws.dff, ws.q4D, lw.w_fc, q.qw_fc, ws.da)
            ops.layernorm_bwd(ws.h1[l], lw.ln2_g, ws.mean2[l], ws.rstd2[l], ws.da, dnew, dres=dres, dx_drop=ws.dxd,
                              drop=dr.ra(l), dgamma=g.ln2_g if g else None, dbeta=g.ln2_b if g else None,
                              workspace=dw.ln_ws if dw else None, rows_dev=rd)
            dres, dnew = dnew, dres
            dy = ws.dxd if dr.ra(l).p > 0 else dres
            if g is not None:
                dw.dW(dy, ws.o[l], g.w_proj, M=M, transpose_out=True)
                dw.db(dy, g.b_proj, M=M)
            self._bmm(ws, dy, ws.qD, lw.w_proj, q.qw_proj, ws.do)
            ops.attention_bwd(ws.qkv[l], ws.do, ws.lse[l], ws.dqkv, B=B, S=S, H=H, hd=hd, scale=scale, causal=True,
                              key_mask=causal_mask, drop=dr.attn(l), out=ws.o[l], seqs=seqs, alg_flops=afl,
                              short_only=so)
            if g is not None:
                dw.dW(ws.dqkv, ws.a1[l], g.w_attn, M=M, transpose_out=True)
                dw.db(ws.dqkv, g.b_attn, M=M)
            self._bmm(ws, ws.dqkv, ws.q3D, lw.w_attn, q.qw_attn, ws.da)
            nxt = dr.rm(l - 1) if l > 0 else dr.embd
            ops.layernorm_bwd(ws.x[l], lw.ln1_g, ws.mean1[l], ws.rstd1[l], ws.da, dnew, dres=dres, dx_drop=ws.dxd,
                              drop=nxt, dgamma=g.ln1_g if g else None, dbeta=g.ln1_b if g else None,
                              workspace=dw.ln_ws if dw else None, rows_dev=rd)
            dres, dnew = dnew, dres
        tag.__exit__(None, None, None)
        d_in = ws.dxd if dr.embd.p > 0 else dres
        if ws.pack:  # the prefix rows' gradient, back in the padded layout the mapper backward reads
            ops.rows_unpack(d_in, ws.seq_off, ws.seq_len, ws.d_emb, B=B, P=ws.P, D=D, dst_bstride=S * D)
            return ws.d_emb
        return d_in

    # -- inference ----------------------------------------------------------------------------------------------
    @torch.no_grad()
    def forward_infer(self, inputs_embeds: Tensor, attention_mask: Optional[Tensor], labels: Optional[Tensor]):
        B, S, D = inputs_embeds.shape
        x_in = inputs_embeds
        if x_in.dtype != self.dtype or not x_in.is_contiguous():
            x_in = inputs_embeds.to(self.dtype).contiguous()
        ws = self.alloc_train(B, S, 0)
        dr = self.drops(False, 0, None, ws.M, B, S)
        mask = attention_mask.to(torch.int64) if attention_mask is not None else None
        lab = labels.to(torch.int64) if labels is not None else None
        # all S positions come in as "prefix" rows (ids unused): x = inputs_embeds + wpe
        ops.caption_prep(B, S, 0, None, None, ws.key_mask, None, None)
        if mask is not None:
            ws.key_mask.copy_(mask.reshape(-1).to(torch.int32))
        if lab is not None:
            ops.caption_prep(B, 0, S, None, lab.contiguous(), None, ws.labels_shift, ws.n_valid)
        ops.gpt2_embed(x_in, S * D, self.wte, self.wpe, None, ws.x[0], B=B, P=S, L_=0, D=D, drop=dr.embd)
        self._blocks_fwd(ws, dr, B, S, ws.M, causal_mask=ws.key_mask if mask is not None else None)
        ops.layernorm_fwd(ws.x[-1], self.lnf_g, self.lnf_b, self.eps, ws.hf, ws.meanf, ws.rstdf)
        self._mm(ws.hf, ws.qhf, self.wte, getattr(self, "qwte", None), ws.logits, alg_flops=2.0 * ws.M * self.V * self.D)
        loss = None
        if lab is not None:
            ops.cross_entropy(ws.logits, self.V, ws.labels_shift, ws.n_valid, ws.loss, None, ws.ce_ws)
            loss = ws.loss[0].clone()
        logits = ws.logits[:, : self.V].float().reshape(B, S, self.V)
        return SimpleNamespace(loss=loss, logits=logits)

    # -- KV-cached greedy decode (src/models.py:327-477, temperature 0) ----------------------------------------
    def alloc_decode(self, B: int, P: int, max_length: int) -> SimpleNamespace:
        D, dt, dev = self.D, self.dtype, self.dev
        T = P + max_length
        e = lambda *shape, dtype=dt: torch.empty(shape, dtype=dtype, device=dev)  # noqa: E731
        ds = SimpleNamespace(B=B, P=P, T=T, max_length=max_length)
        ds.cache = [e(T * B, 3 * D) for _ in self.layers]
        ds.x = e(P * B, D)
        ds.h1 = e(P * B, D)
        ds.a = e(P * B, D)
        ds.o = e(P * B, D)
        ds.f = e(P * B, 4 * D)
        ds.logits = e(B, self.Vp)
        ds.finished = torch.zeros(B, dtype=torch.int32, device=dev)
        ds.tokens = torch.full((B, max_length), self.cfg.eos_token_id, dtype=torch.int64, device=dev)
        ds.km = torch.ones(P * B, dtype=torch.int32, device=dev)
        return ds

    def _decode_block(self, ds, rows: int, x: Tensor, pos0: int, npos: int, prefill: bool):
        """One pass of all blocks over `rows` = npos*B position-major rows starting at position pos0."""
        D, H, hd = self.D, self.H, self.hd
        B = ds.B
        scale = 1.0 / math.sqrt(hd)
        a, o, h1, f = ds.a[:rows], ds.o[:rows], ds.h1[:rows], ds.f[:rows]
        # per-token steps (rows = B <= 128): ln_1 / ln_2 run inside the QKV / c_fc GEMMs (one launch each
        # instead of two; the decode step is bound by its ~90 launches, not by bytes)
        fuse_ln = rows <= 128
        # fp8_mx: the tile-kernel products (prefill, beam steps over R = B*W > 128 rows) run as MX GEMMs
        mx = self.fp8 and not fuse_ln
        qD, q4 = (self._dq(ds, rows, D), self._dq(ds, rows, 4 * D)) if mx else (None, None)
        nq = SimpleNamespace(qw_attn_t=None, qw_proj_t=None, qw_fc_t=None, qw_mp_t=None)
        for l, lw in enumerate(self.layers):
            q = lw if mx else nq
            qkv = ds.cache[l][pos0 * B: (pos0 + npos) * B]
            fold = fuse_ln and getattr(lw, "wf_attn_t", None) is not None
            if fold:
                ops.gemm(x, lw.wf_attn_t, qkv, bias=lw.bf_attn, M=rows, ln_fold=(lw.ws_attn, self.eps))
            elif fuse_ln:
                ops.gemm(x, lw.w_attn_t, qkv, bias=lw.b_attn, M=rows, ln=(lw.ln1_g, lw.ln1_b, self.eps))
            else:
                ops.layernorm_fwd(x, lw.ln1_g, lw.ln1_b, self.eps, a, None, None, rows=rows)
                self._mm(a, qD, lw.w_attn_t, q.qw_attn_t, qkv, bias=lw.b_attn, M=rows)
            if prefill:
                ops.attention_fwd(ds.cache[l], o, B=B, S=npos, H=H, hd=hd, scale=scale, causal=True, rsb=1, rss=B)
            else:
                ops.attention_decode(ds.cache[l], o, B=B, H=H, hd=hd, pos=pos0, scale=scale,
                                     anc=getattr(ds, "anc", None))
            self._mm(o, qD, lw.w_proj_t, q.qw_proj_t, h1, bias=lw.b_proj, resid=x, M=rows)
            if fold:
                ops.gemm(h1, lw.wf_fc_t, f, bias=lw.bf_fc, act=L.ACT_GELU_NEW, M=rows, ln_fold=(lw.ws_fc, self.eps))
            elif fuse_ln:
                ops.gemm(h1, lw.w_fc_t, f, bias=lw.b_fc, act=L.ACT_GELU_NEW, M=rows, ln=(lw.ln2_g, lw.ln2_b, self.eps))
            else:
                ops.layernorm_fwd(h1, lw.ln2_g, lw.ln2_b, self.eps, a, None, None, rows=rows)
                self._mm(a, qD, lw.w_fc_t, q.qw_fc_t, f, bias=lw.b_fc, act=L.ACT_GELU_NEW, M=rows)
            self._mm(f, q4, lw.w_mp_t, q.qw_mp_t, x, bias=lw.b_mp, resid=h1, M=rows)

    def _dq(self, ds, rows: int, K: int):
        """MX operand buffer of the decode state for (rows, K) (allocated on first use, outside graph capture:
        the eager warm-up pass of a runner reaches every shape first)."""
        if not hasattr(ds, "mx"):
            ds.mx = {}
        key = (rows, K)
        if key not in ds.mx:
            ds.mx[key] = ops.MXTensor.empty(rows, K, self.dev)
        return ds.mx[key]

    def _head_mm(self, ds, a: Tensor, rows: int) -> None:
        """LM head of `rows` decode rows (bf16 skinny / tile GEMM; fp8_mx: MX when it takes the tile kernel)."""
        mx = self.fp8 and rows > 128
        self._mm(a, self._dq(ds, rows, self.D) if mx else None, self.wte, self.qwte if mx else None, ds.logits,
                 M=rows, alg_flops=2.0 * rows * self.V * self.D)

    def _decode_head(self, ds, x_last: Tensor, step: int, pos_next: int, samp=None):
        """ln_f + LM head on the last position, then the next token: argmax (greedy) or, with samp = (temperature,
        top_p, seed_dev, nxt), the nucleus draw of src/models.py:400-449 (ops.topp_sample); then the EOS latch
        and the next step's input embedding (ops.greedy_next)."""
        D = self.D
        B = ds.B
        a = ds.a[:B]
        # (ln_f stays a launch of its own: folded into the tied LM head's skinny GEMM — W*gamma_f, row sums, W.beta_f
        # — the decode ran 3381 vs 3853 captions/s, profiles/r04_bench_lnf_fold_3381.json: the 50304-column launch
        # re-derives each row's statistics in every one of its workgroups)
        ops.layernorm_fwd(x_last, self.lnf_g, self.lnf_b, self.eps, a, None, None, rows=B)
        self._head_mm(ds, a, B)
        forced = None
        if samp is not None:
            temperature, top_p, seed_dev, forced = samp
            ops.topp_sample(ds.logits, self.V, temperature, top_p, ds.finished, 0, step, self.cfg.eos_token_id,
                            forced, seed_ptr=seed_dev)
        nxt_x = ds.x[:B] if pos_next < ds.T else None
        ops.greedy_next(ds.logits, self.V, self.cfg.eos_token_id, ds.finished, ds.tokens, step,
                        self.wte if nxt_x is not None else None, self.wpe if nxt_x is not None else None,
                        min(pos_next, self.cfg.n_positions - 1), D, nxt_x, forced=forced)

    @torch.no_grad()
    def greedy_decode(self, prefix: Tensor, max_length: int, check_every: int = 8, early_exit: bool = True) -> Tensor:
        """prefix [B,P,D] (compute dtype) -> token ids [B, <=max_length] with the reference's EOS latch and
        early exit (src/models.py:389-391,453-460). Exact to the reference's full-recompute loop: causal
        attention makes cached keys/values of earlier positions identical to recomputed ones."""
        B, P, D = prefix.shape
        if max_length <= 0:
            return torch.empty((B, 0), dtype=torch.long, device=prefix.device)
        if prefix.is_cuda and self.graph_decode:
            return self._runner(B, P, max_length).run(prefix, early_exit, check_every)
        ds = self.alloc_decode(B, P, max_length)
        pre = prefix if (prefix.dtype == self.dtype and prefix.stride(-1) == 1) else prefix.to(self.dtype).contiguous()
        ops.add_position(pre, pre.stride(0), pre.stride(1), self.wpe, ds.x, B=B, npos=P, D=D, pos0=0)
        self._decode_block(ds, P * B, ds.x, 0, P, prefill=True)
        self._decode_head(ds, ds.x[(P - 1) * B: P * B], 0, P)
        steps = 1
        for s in range(1, max_length):
            if early_exit and s % check_every == 0 and bool(ds.finished.bool().all()):
                break
            pos = P + s - 1
            self._decode_block(ds, B, ds.x[:B], pos, 1, prefill=False)
            self._decode_head(ds, ds.x[:B], s, pos + 1)
            steps = s + 1
        toks = ds.tokens[:, :steps]
        # reference loop length: stops before the first step at which every row had already finished
        return self._truncate(toks, steps)

    graph_decode = True  # replay captured HIP graphs of the decode chunks (per batch shape)

    def _runner(self, B: int, P: int, max_length: int, sampling=None) -> "DecodeRunner":
        if not hasattr(self, "_runners"):
            self._runners = {}
        key = (B, P, max_length, sampling)
        if key not in self._runners:
            if len(self._runners) >= 2:
                self._runners.pop(next(iter(self._runners)))
            self._runners[key] = DecodeRunner(self, B, P, max_length, sampling=sampling)
        return self._runners[key]

    def _truncate(self, toks: Tensor, steps: int) -> Tensor:
        B = toks.shape[0]
        is_eos = toks == self.cfg.eos_token_id
        first = torch.where(is_eos.any(1), is_eos.float().argmax(1), torch.full((B,), steps, device=toks.device))
        n = int(min(steps, int(first.max().item()) + 1))
        return toks[:, :n].clone()

    @torch.no_grad()
    def sample_decode(self, prefix: Tensor, max_length: int, temperature: float, top_p: float,
                      seed: Optional[int] = None) -> Tensor:
        """Temperature / nucleus sampling branch of src/models.py:400-449 over the KV-cached decoder. Logits,
        the top-p filter and the draw are HIP kernels (ops.topp_sample), replayed as HIP-graph
        chunks like greedy decode. The draw's seed comes from torch's CPU generator unless given (so
        torch.manual_seed makes a run reproducible); it lives in device memory, so one graph serves every seed."""
        B, P, D = prefix.shape
        if max_length <= 0:
            return torch.empty((B, 0), dtype=torch.long, device=prefix.device)
        if seed is None:
            seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        if prefix.is_cuda and self.graph_decode:
            return self._runner(B, P, max_length, (float(temperature), float(top_p))).run(prefix, seed=seed)
        ds = self.alloc_decode(B, P, max_length)
        samp = (temperature, top_p, torch.full((1,), seed, dtype=torch.int64, device=prefix.device),
                torch.empty(B, dtype=torch.long, device=prefix.device))
        pre = prefix if (prefix.dtype == self.dtype and prefix.stride(-1) == 1) else prefix.to(self.dtype).contiguous()
        ops.add_position(pre, pre.stride(0), pre.stride(1), self.wpe, ds.x, B=B, npos=P, D=D, pos0=0)
        self._decode_block(ds, P * B, ds.x, 0, P, prefill=True)
        self._decode_head(ds, ds.x[(P - 1) * B: P * B], 0, P, samp)
        steps = 1
        for s in range(1, max_length):
            if bool(ds.finished.bool().all()):
                break
            pos = P + s - 1
            self._decode_block(ds, B, ds.x[:B], pos, 1, prefill=False)
            self._decode_head(ds, ds.x[:B], s, pos + 1, samp)
            steps = s + 1
        return self._truncate(ds.tokens[:, :steps], steps)


    # -- beam search (transformers' generate(num_beams=W), HF/generation/utils.py:3208-3540)
    def alloc_beam(self, B: int, W: int, P: int, max_length: int, length_penalty: float = 1.0) -> SimpleNamespace:
        """Decode buffers for R = B*W rows (row b*W + i = beam i of caption b) + the beam state; the KV cache
        is read through the state's ancestry table."""
        ds = self.alloc_decode(B * W, P, max_length)
        ds.beam = ops.BeamState(B, W, self.V, max_length, ds.T, self.cfg.eos_token_id, length_penalty, self.dev)
        ds.beam.set_embedding(self.dtype, self.D, self.cfg.n_positions, self.wte, self.wpe, None)
        ds.anc = ds.beam.anc
        ds.W = W
        return ds

    def _beam_head(self, ds, x_last: Tensor, step: int, pos: int) -> None:
        """ln_f + LM head on every row's last position, then one beam step (icap_beam_rowtop + icap_beam_update:
        candidates, running / finished beams, ancestry, next input rows)."""
        R = ds.B
        a = ds.a[:R]
        ops.layernorm_fwd(x_last, self.lnf_g, self.lnf_b, self.eps, a, None, None, rows=R)
        self._head_mm(ds, a, R)
        nxt_x = ds.x[:R] if pos + 1 < ds.T else None
        ds.beam.step(ds.logits, step, pos, nxt_x)

    def _beam_prefill(self, ds, prefix_rows: Tensor) -> None:
        """prefix_rows [R, P, D]: each caption's prefix once per beam."""
        R, P, D = prefix_rows.shape
        ops.add_position(prefix_rows, prefix_rows.stride(0), prefix_rows.stride(1), self.wpe, ds.x, B=R, npos=P,
                         D=D, pos0=0)
        ds.beam.init(P)
        self._decode_block(ds, P * R, ds.x, 0, P, prefill=True)
        self._beam_head(ds, ds.x[(P - 1) * R: P * R], 0, P - 1)

    def _beam_result(self, ds) -> Tensor:
        out, n = ds.beam.finalize()
        m = int(n.max().item()) if n.numel() else 0
        return out[:, :m].clone()

    @torch.no_grad()
    def beam_decode(self, prefix: Tensor, max_length: int, num_beams: int = 4, length_penalty: float = 1.0,
                    check_every: int = 8, early_exit: bool = True) -> Tensor:
        """prefix [B,P,D] -> ids [B, <= max_length]: each caption's best finished hypothesis (EOS included when it
        ended on one), EOS-padded to the longest (HF/generation/utils.py:3512-3523). Stops early once every
        caption is done (the early-stop heuristic, :3008-3053); early_exit=False runs all max_length steps (finished
        captions stay frozen, so the ids are the same: a fixed-work throughput measurement)."""
        B, P, D = prefix.shape
        if max_length <= 0:
            return torch.empty((B, 0), dtype=torch.long, device=prefix.device)
        if prefix.is_cuda and self.graph_decode:
            return self._beam_runner(B, num_beams, P, max_length, length_penalty).run(prefix, early_exit)
        ds = self.alloc_beam(B, num_beams, P, max_length, length_penalty)
        rows = prefix.to(self.dtype).repeat_interleave(num_beams, dim=0).contiguous()
        self._beam_prefill(ds, rows)
        for s in range(1, max_length):
            if early_exit and s % check_every == 0 and bool(ds.beam.done.bool().all()):
                break
            pos = P + s - 1
            self._decode_block(ds, ds.B, ds.x[:ds.B], pos, 1, prefill=False)
            self._beam_head(ds, ds.x[:ds.B], s, pos)
        return self._beam_result(ds)

    def _beam_runner(self, B: int, W: int, P: int, max_length: int, length_penalty: float) -> "BeamRunner":
        if not hasattr(self, "_beam_runners"):
            self._beam_runners = {}
        key = (B, W, P, max_length, float(length_penalty))
        if key not in self._beam_runners:
            if len(self._beam_runners) >= 2:
                self._beam_runners.pop(next(iter(self._beam_runners)))
            self._beam_runners[key] = BeamRunner(self, B, W, P, max_length, length_penalty)
        return self._beam_runners[key]


class BeamRunner:
    """Beam search of one (B, W, P, max_length) shape as HIP-graph chunks (like DecodeRunner): chunk 0 = state
    init + prefill + step 0, chunk c = steps [c*C, (c+1)*C). Between chunks the host reads the per-caption done
    flags once; finished captions are frozen on the device, so extra steps never change the result."""

    def __init__(self, core: "GPT2Core", B: int, W: int, P: int, max_length: int, length_penalty: float,
                 chunk: int = 8):
        self.core, self.B, self.W, self.P, self.T = core, B, W, P, max_length
        self.ds = core.alloc_beam(B, W, P, max_length, length_penalty)
        self.rows = torch.zeros((B * W, P, core.D), dtype=core.dtype, device=core.dev)
        self.bounds = [(0, min(chunk, max_length))]
        s = chunk
        while s < max_length:
            self.bounds.append((s, min(s + chunk, max_length)))
            s += chunk
        self.graphs = None

    def _chunk(self, c: int) -> None:
        core, ds, P = self.core, self.ds, self.P
        s0, s1 = self.bounds[c]
        if c == 0:
            core._beam_prefill(ds, self.rows)
            s0 = 1
        for s in range(s0, s1):
            pos = P + s - 1
            core._decode_block(ds, ds.B, ds.x[:ds.B], pos, 1, prefill=False)
            core._beam_head(ds, ds.x[:ds.B], s, pos)

    @torch.no_grad()
    def run(self, prefix: Tensor, early_exit: bool = True) -> Tensor:
        self.rows.copy_(prefix.to(self.core.dtype).repeat_interleave(self.W, dim=0))
        if self.graphs is None:
            for c in range(len(self.bounds)):  # eager warm-up pass (initialises every kernel once)
                self._chunk(c)
            torch.cuda.synchronize(self.core.dev)
            self.graphs = []
            for c in range(len(self.bounds)):
                g = torch.cuda.CUDAGraph()
                with ops.graph_capture(g):
                    self._chunk(c)
                self.graphs.append(g)
        for c, g in enumerate(self.graphs):
            g.replay()
            if early_exit and c + 1 < len(self.graphs) and bool(self.ds.beam.done.bool().all()):
                break
        return self.core._beam_result(self.ds)


class DecodeRunner:
    """Greedy (or, with sampling = (temperature, top_p), nucleus-sampled) decode of one batch shape as HIP-graph
    chunks: chunk 0 = prefill + token 0 (+ state reset),
    chunk c = tokens [c*C, (c+1)*C). Between chunks the host reads the EOS latch once (early exit,
    src/models.py:390-391); the returned ids are truncated to the reference loop's length either way."""

    def __init__(self, core: GPT2Core, B: int, P: int, max_length: int, chunk: int = 8, sampling=None):
        self.core, self.B, self.P, self.T = core, B, P, max_length
        self.chunk = chunk
        self.ds = core.alloc_decode(B, P, max_length)
        self.samp = None  # sampling = (temperature, top_p): nucleus draws, seed read from seed_dev at replay
        if sampling is not None:
            self.seed_dev = torch.zeros(1, dtype=torch.int64, device=core.dev)
            self.samp = (sampling[0], sampling[1], self.seed_dev, torch.empty(B, dtype=torch.long, device=core.dev))
        self.prefix = torch.zeros((B, P, core.D), dtype=core.dtype, device=core.dev)
        self.bounds = [(0, min(chunk, max_length))]
        s = chunk
        while s < max_length:
            self.bounds.append((s, min(s + chunk, max_length)))
            s += chunk
        self.graphs = None

    def _chunk(self, c: int) -> None:
        core, ds, B, P, D = self.core, self.ds, self.B, self.P, self.core.D
        s0, s1 = self.bounds[c]
        if c == 0:
            ds.finished.zero_()
            ds.tokens.fill_(core.cfg.eos_token_id)
            ops.add_position(self.prefix, P * D, D, core.wpe, ds.x, B=B, npos=P, D=D, pos0=0)
            core._decode_block(ds, P * B, ds.x, 0, P, prefill=True)
            core._decode_head(ds, ds.x[(P - 1) * B: P * B], 0, P, self.samp)
            s0 = 1
        for s in range(s0, s1):
            pos = P + s - 1
            core._decode_block(ds, B, ds.x[:B], pos, 1, prefill=False)
            core._decode_head(ds, ds.x[:B], s, pos + 1, self.samp)

    @torch.no_grad()
    def run(self, prefix: Tensor, early_exit: bool = True, check_every: int = 8, seed: int = 0) -> Tensor:
        self.prefix.copy_(prefix)
        if self.samp is not None:
            self.seed_dev.fill_(seed)
        if self.graphs is None:
            for c in range(len(self.bounds)):  # eager warm-up pass (initialises every kernel once)
                self._chunk(c)
            torch.cuda.synchronize(self.core.dev)
            self.graphs = []
            for c in range(len(self.bounds)):
                g = torch.cuda.CUDAGraph()
                with ops.graph_capture(g):
                    self._chunk(c)
                self.graphs.append(g)
        steps = 0
        for c, g in enumerate(self.graphs):
            g.replay()
            steps = self.bounds[c][1]
            if early_exit and c + 1 < len(self.graphs) and bool(self.ds.finished.bool().all()):
                break
        return self.core._truncate(self.ds.tokens[:, :steps], steps)
