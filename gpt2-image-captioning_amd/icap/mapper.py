"""Image-prefix mapping networks (src/models.py:14-174) on the icap HIP kernels.

`TransformerMappingNetwork` / `MLPMappingNetwork` keep the reference's constructor
signatures, attributes and state_dict key names; their arithmetic is the
explicit forward/backward kernel schedule of `TransformerMapperCore` /
`MLPMapperCore` (norm_first encoder layer: TORCH/nn/modules/transformer.py:946-982).
"""

from __future__ import annotations

import math
from types import SimpleNamespace
from typing import Optional

import torch
import torch.nn as nn

from . import _lib as L
from . import ops
from .ops import Dropout
from .weights import det_tensor

Tensor = torch.Tensor


def _rup(x: int, m: int) -> int:
    return (x + m - 1) // m * m


# --------------------------------------------------------------------------- dW helper


def _kout_ok(t: Tensor) -> bool:
    """K-outer GEMM operand requirements: 16-byte aligned base, row stride a multiple of 8 elements."""
    return t.data_ptr() % 16 == 0 and t.stride(0) % 8 == 0 and t.stride(-1) == 1


# a mapper layer's two LayerNorm parameter reduces in one launch at the layer's end (ops.ln_param_reduce_batch;
# bitwise the per-call reduces). Read when the backward is built, so a captured graph keeps the setting.
LN_PARAM_BATCH = True

class DWHelper:
    """dW[N,K] += dY[M,N]^T . X[M,K] on the MFMA GEMM. bf16: one K-outer product (trans_ab) straight from dY
    and X; fp32 (parity mode): both operands are transposed into K(=M)-contiguous scratch (M padded to 64 with
    zeros) first, then one C = A.B^T product accumulates into the fp32 grad."""

    def __init__(self, dtype: torch.dtype, device, max_rows: int, max_cols: int, ln_rows: int, ln_D: int,
                 colsum_cols: int = 0):
        self.dtype = dtype
        self.split_k = 0  # icap_gemm split_k for the K-outer products (0 = automatic)
        self.Mp_max = _rup(max(max_rows, 1), 64)
        self.tA = torch.zeros(max_cols * self.Mp_max, dtype=dtype, device=device)
        self.tB = torch.zeros(max_cols * self.Mp_max, dtype=dtype, device=device)
        self.cs_cols = max(max_cols, colsum_cols)
        self.cs_ws = torch.empty(ops.colsum_workspace(max_rows, self.cs_cols), dtype=torch.uint8, device=device)
        # bf16 ones [rows][8]: the B operand of the bias gradients inside a grouped launch (db = dY^T . 1, dW_group)
        self.ones = torch.ones((max(max_rows, 1), 8), dtype=dtype, device=device) if dtype == torch.bfloat16 else None
        self.ln_ws = torch.empty(max(ops.layernorm_bwd_workspace(ln_rows, ln_D), 16), dtype=torch.uint8,
                                 device=device)
        # a second one: a mapper layer's two LayerNorm backwards leave their dgamma / dbeta partials side by side and
        # reduce them in one launch at the layer's end (ops.ln_param_reduce_batch)
        self.ln_ws2 = torch.empty_like(self.ln_ws)
        self.ln_rows, self.ln_D = ln_rows, ln_D

    def _t(self, buf: Tensor, src: Tensor, M: int, N: int, Mp: int) -> Tensor:
        dst = buf[: N * Mp].view(N, Mp)
        ops.transpose(src, dst, rows_pad=Mp, rows=M, cols=N)
        return dst

    def dW(self, dY: Tensor, X: Tensor, out: Tensor, M: int, N: Optional[int] = None, K: Optional[int] = None,
           transpose_out: bool = False, accumulate: bool = True, split_k: Optional[int] = None) -> None:
        """accumulate=False overwrites out (the first micro-batch of a cycle: beta 0, no read of the old value).
        split_k: the K-outer product's split (None: this helper's setting; 1: unsplit, no slabs / reduce pass)."""
        N = dY.shape[1] if N is None else N
        K = X.shape[1] if K is None else K
        beta = 1.0 if accumulate else 0.0
        sk = self.split_k if split_k is None else split_k
        if self.dtype == torch.bfloat16 and _kout_ok(dY) and _kout_ok(X):
            # bf16: one K-outer GEMM reads dY and X in place (icap_gemm_args.trans_ab), no transposes
            if transpose_out:
                ops.gemm(X, dY, out, beta=beta, M=K, N=N, K=M, trans_ab=True, split_k=sk)
            else:
                ops.gemm(dY, X, out, beta=beta, M=N, N=K, K=M, trans_ab=True, split_k=sk)
            return
        Mp = _rup(M, 64)
        a = self._t(self.tA, dY, M, N, Mp)  # [N][Mp]
        b = self._t(self.tB, X, M, K, Mp)   # [K][Mp]
        if transpose_out:  # out[K,N] (HF Conv1D grad layout)
            ops.gemm(b, a, out, beta=beta, M=K, N=N, K=Mp, alg_flops=2.0 * M * N * K)
        else:              # out[N,K] (nn.Linear grad layout)
            ops.gemm(a, b, out, beta=beta, M=N, N=K, K=Mp, alg_flops=2.0 * M * N * K)

    def dW_group(self, items, M: int, accumulate: bool = True, db_items=()) -> bool:
        """dW += dY^T X for every (dY, X, out) of items in one launch (ops.gemm_group: unsplit K-outer products, no
        slabs or reduce pass) where every operand allows the in-place K-outer read; otherwise one dW() each.
        db_items: (dY, db) bias gradients db += dY^T . 1 taken into the same launch as K-outer products against a
        ones column (fp32 MFMA sums over the rows instead of icap_colsum_batch: no launches of their own, and their
        tiles fill the CUs the dW tiles leave idle in the launch's last round). Returns whether db_items were done."""
        beta = 1.0 if accumulate else 0.0
        if self.dtype == torch.bfloat16 and all(_kout_ok(dy) and _kout_ok(x) for dy, x, _ in items):
            group = [(dy, x, out, dy.shape[1], x.shape[1], M, beta) for dy, x, out in items]
            took_db = (self.ones is not None and M <= self.ones.shape[0] and len(group) + len(db_items) <= 8
                       and all(_kout_ok(dy) and out.is_contiguous() for dy, out in db_items))
            if took_db:
                group += [(dy, self.ones, out.view(-1, 1), dy.shape[1], 1, M, beta) for dy, out in db_items]
            ops.gemm_group(group)
            return took_db
        for dy, x, out in items:
            self.dW(dy, x, out, M=M, accumulate=accumulate)
        return False

    def db(self, dY: Tensor, out: Tensor, M: int, N: Optional[int] = None, accumulate: bool = True) -> None:
        ops.colsum(dY, out, self.cs_ws, accumulate=accumulate, M=M, N=N)

    def db_batch(self, items, M: int, accumulate: bool = True) -> None:
        """db += colsum(dY) for every (dY, db) over the same M rows: two launches (icap_colsum_batch) instead of
        two per item; bitwise what db() gives. The workspace holds colsum_cols columns of partials: a call with
        more columns runs in column groups that fit."""
        group, cols = [], 0
        for dy, out in items:
            n = dy.shape[1]
            if group and cols + n > self.cs_cols:
                ops.colsum_batch(group, M, self.cs_ws, accumulate=accumulate)
                group, cols = [], 0
            group.append((dy, out, None))
            cols += n
        if group:
            ops.colsum_batch(group, M, self.cs_ws, accumulate=accumulate)


# --------------------------------------------------------------------------- modules (reference names)


class _MHA(nn.Module):
    """nn.MultiheadAttention storage: in_proj_weight [3D,D], in_proj_bias, out_proj (Linear)."""

    def __init__(self, d: int, nhead: int, dropout: float):
        super().__init__()
        self.num_heads = nhead
        self.dropout = dropout
        self.in_proj_weight = nn.Parameter(torch.empty(3 * d, d))
        self.in_proj_bias = nn.Parameter(torch.zeros(3 * d))
        self.out_proj = nn.Linear(d, d)
        nn.init.xavier_uniform_(self.in_proj_weight)
        nn.init.zeros_(self.out_proj.bias)


class _EncoderLayer(nn.Module):
    """nn.TransformerEncoderLayer(d_model, nhead=8, dim_feedforward=4d, relu, norm_first=True) storage."""

    def __init__(self, d: int, nhead: int, dropout: float = 0.1):
        super().__init__()
        self.self_attn = _MHA(d, nhead, dropout)
        self.linear1 = nn.Linear(d, 4 * d)
        self.linear2 = nn.Linear(4 * d, d)
        self.norm1 = nn.LayerNorm(d, eps=1e-5)
        self.norm2 = nn.LayerNorm(d, eps=1e-5)
        self.dropout_p = dropout


class _Encoder(nn.Module):
    def __init__(self, d: int, nhead: int, num_layers: int):
        super().__init__()
        self.layers = nn.ModuleList([_EncoderLayer(d, nhead) for _ in range(num_layers)])


class TransformerMappingNetwork(nn.Module):
    """src/models.py:77-174 — same constructor, attributes and parameter names."""

    def __init__(self, embed_dim: int, gpt_dim: int, prefix_length: int, hidden_length: int, num_layers: int = 8,
                 nhead: int = 8) -> None:
        super().__init__()
        self.embed_dim = embed_dim
        self.gpt_dim = gpt_dim
        self.hidden_length = hidden_length
        self.prefix_length = prefix_length
        self.nhead = nhead  # models.py:131 hard-codes 8
        self.linear = nn.Linear(embed_dim, hidden_length * gpt_dim)
        self.prefix_const = nn.Parameter(torch.randn(prefix_length, gpt_dim), requires_grad=True)
        self.transformer = _Encoder(gpt_dim, nhead, num_layers)
        self._core = None
        self._core_key = None

    @classmethod
    def random_init(cls, embed_dim=512, gpt_dim=768, prefix_length=15, hidden_length=10, num_layers=8,
                    seed: int = 0) -> "TransformerMappingNetwork":
        m = cls(embed_dim, gpt_dim, prefix_length, hidden_length, num_layers)
        d, ff = gpt_dim, 4 * gpt_dim
        sd = {
            "linear.weight": det_tensor(seed, "m.linear.w", (hidden_length * d, embed_dim), 1 / math.sqrt(3 * embed_dim)),
            "linear.bias": det_tensor(seed, "m.linear.b", (hidden_length * d,), 1 / math.sqrt(3 * embed_dim)),
            "prefix_const": det_tensor(seed, "m.prefix_const", (prefix_length, d), 1.0),
        }
        for i in range(num_layers):
            p = f"transformer.layers.{i}."
            sd[p + "self_attn.in_proj_weight"] = det_tensor(seed, p + "in_w", (3 * d, d), math.sqrt(2.0 / (4 * d)))
            sd[p + "self_attn.in_proj_bias"] = det_tensor(seed, p + "in_b", (3 * d,), 0.02)
            sd[p + "self_attn.out_proj.weight"] = det_tensor(seed, p + "out_w", (d, d), 1 / math.sqrt(3 * d))
            sd[p + "self_attn.out_proj.bias"] = det_tensor(seed, p + "out_b", (d,), 0.02)
            sd[p + "linear1.weight"] = det_tensor(seed, p + "l1_w", (ff, d), 1 / math.sqrt(3 * d))
            sd[p + "linear1.bias"] = det_tensor(seed, p + "l1_b", (ff,), 1 / math.sqrt(3 * d))
            sd[p + "linear2.weight"] = det_tensor(seed, p + "l2_w", (d, ff), 1 / math.sqrt(3 * ff))
            sd[p + "linear2.bias"] = det_tensor(seed, p + "l2_b", (d,), 1 / math.sqrt(3 * ff))
            sd[p + "norm1.weight"] = det_tensor(seed, p + "n1_w", (d,), 0.05, 1.0)
            sd[p + "norm1.bias"] = det_tensor(seed, p + "n1_b", (d,), 0.02)
            sd[p + "norm2.weight"] = det_tensor(seed, p + "n2_w", (d,), 0.05, 1.0)
            sd[p + "norm2.bias"] = det_tensor(seed, p + "n2_b", (d,), 0.02)
        m.load_state_dict(sd)
        return m

    def core(self, dtype: torch.dtype, flat=None) -> "TransformerMapperCore":
        key = (dtype, self.linear.weight.device, id(flat))
        if self._core is None or self._core_key != key:
            self._core = TransformerMapperCore(self, dtype, flat)
            self._core_key = key
        return self._core

    def forward(self, x: Tensor) -> Tensor:
        """(B, embed_dim) -> (B, prefix_length, gpt_dim) on the HIP path (inference; src/models.py:141-174)."""
        dt = x.dtype if x.dtype in (torch.float32, torch.bfloat16) else torch.float32
        return self.core(dt).infer(x)


class MLPMappingNetwork(nn.Module):
    """src/models.py:14-74 — Linear(embed, P*D/2) -> Tanh -> Linear(P*D/2, P*D) -> view."""

    def __init__(self, prefix_length: int = 10, embed_dim: int = 512, gpt_dim: int = 768, bias: bool = True,
                 activation: Optional[nn.Module] = None) -> None:
        super().__init__()
        if activation is not None and not isinstance(activation, nn.Tanh):
            raise NotImplementedError("icap MLPMappingNetwork implements the reference's default Tanh activation")
        if not bias:
            raise NotImplementedError("icap MLPMappingNetwork implements the reference's default bias=True")
        self.prefix_length = prefix_length
        self.embed_dim = embed_dim
        self.gpt_dim = gpt_dim
        out = prefix_length * gpt_dim
        self.model = nn.Sequential(nn.Linear(embed_dim, out // 2, bias=bias), nn.Tanh(), nn.Linear(out // 2, out, bias=bias))
        self._core = None
        self._core_key = None

    @classmethod
    def random_init(cls, prefix_length=15, embed_dim=512, gpt_dim=768, seed: int = 0) -> "MLPMappingNetwork":
        m = cls(prefix_length, embed_dim, gpt_dim)
        out = prefix_length * gpt_dim
        hid = out // 2
        m.load_state_dict({
            "model.0.weight": det_tensor(seed, "mlp.0.w", (hid, embed_dim), 1 / math.sqrt(3 * embed_dim)),
            "model.0.bias": det_tensor(seed, "mlp.0.b", (hid,), 1 / math.sqrt(3 * embed_dim)),
            "model.2.weight": det_tensor(seed, "mlp.2.w", (out, hid), 1 / math.sqrt(3 * hid)),
            "model.2.bias": det_tensor(seed, "mlp.2.b", (out,), 1 / math.sqrt(3 * hid)),
        })
        return m

    def core(self, dtype: torch.dtype, flat=None) -> "MLPMapperCore":
        key = (dtype, self.model[0].weight.device, id(flat))
        if self._core is None or self._core_key != key:
            self._core = MLPMapperCore(self, dtype, flat)
            self._core_key = key
        return self._core

    def forward(self, x: Tensor) -> Tensor:
        dt = x.dtype if x.dtype in (torch.float32, torch.bfloat16) else torch.float32
        return self.core(dt).infer(x)


# --------------------------------------------------------------------------- cores


def _compute_view(flat, p: nn.Parameter, dtype: torch.dtype) -> Tensor:
    if flat is not None:
        return flat.view_c(p)
    if dtype == torch.float32:
        return p.data
    t = torch.empty(p.shape, dtype=dtype, device=p.device)
    ops.convert(p.data.reshape(p.shape[0], -1), t.reshape(p.shape[0], -1))
    return t


class TransformerMapperCore:
    """Kernel schedules for TransformerMappingNetwork: x0 = [linear(emb) ; prefix_const]; 8 pre-LN layers."""

    def __init__(self, m: TransformerMappingNetwork, dtype: torch.dtype, flat=None):
        from ._lib import require_device

        self.m, self.dtype, self.flat = m, dtype, flat
        self.dev = m.linear.weight.device
        require_device(self.dev)
        self.D, self.E = m.gpt_dim, m.embed_dim
        self.H = m.nhead
        self.hd = self.D // self.H
        self.Hl, self.P = m.hidden_length, m.prefix_length
        self.S = self.Hl + self.P
        self.nl = len(m.transformer.layers)
        self.refresh()

    @torch.no_grad()
    def refresh(self) -> None:
        """Compute-dtype weights (forward [out,in]) + transposed copies ([in,out], backward dX operands)."""
        m, dt = self.m, self.dtype
        cv = lambda p: _compute_view(self.flat, p, dt)  # noqa: E731
        self.w_lin, self.b_lin = cv(m.linear.weight), m.linear.bias.data
        self.prefix_const = m.prefix_const.data
        self.layers = []
        for lay in m.transformer.layers:
            w = SimpleNamespace()
            w.in_w, w.in_b = cv(lay.self_attn.in_proj_weight), lay.self_attn.in_proj_bias.data
            w.out_w, w.out_b = cv(lay.self_attn.out_proj.weight), lay.self_attn.out_proj.bias.data
            w.l1_w, w.l1_b = cv(lay.linear1.weight), lay.linear1.bias.data
            w.l2_w, w.l2_b = cv(lay.linear2.weight), lay.linear2.bias.data
            w.n1_g, w.n1_b = lay.norm1.weight.data, lay.norm1.bias.data
            w.n2_g, w.n2_b = lay.norm2.weight.data, lay.norm2.bias.data
            w.in_wt = torch.empty((w.in_w.shape[1], w.in_w.shape[0]), dtype=dt, device=self.dev)
            w.out_wt = torch.empty((w.out_w.shape[1], w.out_w.shape[0]), dtype=dt, device=self.dev)
            w.l1_wt = torch.empty((w.l1_w.shape[1], w.l1_w.shape[0]), dtype=dt, device=self.dev)
            w.l2_wt = torch.empty((w.l2_w.shape[1], w.l2_w.shape[0]), dtype=dt, device=self.dev)
            self.layers.append(w)
        self.refresh_transposes()

    def dw_cols(self) -> int:
        """Widest dW operand (transposed into DWHelper scratch): linear out Hl*D, qkv 3D, ff 4D."""
        return max(self.Hl * self.D, 4 * self.D, self.E)

    def refresh_transposes(self) -> None:
        pairs = [(a, b) for w in self.layers
                 for a, b in ((w.in_w, w.in_wt), (w.out_w, w.out_wt), (w.l1_w, w.l1_wt), (w.l2_w, w.l2_wt))]
        if pairs and pairs[0][0].dtype == torch.bfloat16:
            ops.transpose_batch(pairs)  # one launch for every layer's copies (was 4 per layer)
        else:
            for a, b in pairs:
                ops.transpose(a, b)

    def grads(self, flat) -> SimpleNamespace:
        m = self.m
        g = SimpleNamespace(lin_w=flat.grad(m.linear.weight), lin_b=flat.grad(m.linear.bias),
                            prefix_const=flat.grad(m.prefix_const), layers=[])
        for lay in m.transformer.layers:
            g.layers.append(SimpleNamespace(
                in_w=flat.grad(lay.self_attn.in_proj_weight), in_b=flat.grad(lay.self_attn.in_proj_bias),
                out_w=flat.grad(lay.self_attn.out_proj.weight), out_b=flat.grad(lay.self_attn.out_proj.bias),
                l1_w=flat.grad(lay.linear1.weight), l1_b=flat.grad(lay.linear1.bias),
                l2_w=flat.grad(lay.linear2.weight), l2_b=flat.grad(lay.linear2.bias),
                n1_g=flat.grad(lay.norm1.weight), n1_b=flat.grad(lay.norm1.bias),
                n2_g=flat.grad(lay.norm2.weight), n2_b=flat.grad(lay.norm2.bias)))
        return g

    # -- workspaces ------------------------------------------------------------------------------------------
    def alloc(self, B: int, train: bool, per_layer_grads: bool = False) -> SimpleNamespace:
        """per_layer_grads: one set of backward gradient buffers per layer (the side / grouped weight-gradient
        schedules, whose dW products trail the dX chain); the serial schedule shares two alternating sets."""
        S, D, dt, dev, nl = self.S, self.D, self.dtype, self.dev, self.nl
        M = B * S
        e = lambda *shape, dtype=dt: torch.empty(shape, dtype=dtype, device=dev)  # noqa: E731
        ws = SimpleNamespace(B=B, M=M, S=S)
        n_keep = nl if train else 1
        ws.x = [e(M, D) for _ in range(nl + 1)] if train else [e(M, D), e(M, D)]
        ws.a1 = [e(M, D) for _ in range(n_keep)]
        ws.qkv = [e(M, 3 * D) for _ in range(n_keep)]
        ws.o = [e(M, D) for _ in range(n_keep)]
        ws.h1 = [e(M, D) for _ in range(n_keep)]
        ws.a2 = [e(M, D) for _ in range(n_keep)]
        ws.f = [e(M, 4 * D) for _ in range(n_keep)]
        ws.mean1 = [e(M, dtype=torch.float32) for _ in range(n_keep)]
        ws.rstd1 = [e(M, dtype=torch.float32) for _ in range(n_keep)]
        ws.mean2 = [e(M, dtype=torch.float32) for _ in range(n_keep)]
        ws.rstd2 = [e(M, dtype=torch.float32) for _ in range(n_keep)]
        ws.lse = [e(B * self.H * S, dtype=torch.float32) for _ in range(n_keep)]
        if train:
            ws.dout = torch.zeros((M, D), dtype=dt, device=dev)  # rows t < Hl stay zero
            ws.dres = e(M, D)  # d(mapper input rows): the head step reads it
            # gradient buffers of the backward (mapper.backward_steps). per_layer_grads: one set per layer — every
            # buffer a layer's weight-gradient products read is written once per step, so those products can trail
            # the dX chain on side streams with no write-after-read hazard (8 layers x 11 M x D x 2 B: 433 MB at
            # B = 128). The serial schedule runs each layer's dW products before the next layer's backward writes
            # anything, so it shares one set; g_r / g_m alternate by layer parity (layer l reads g_r[l], g_m[l] and
            # writes g_r[l-1], g_m[l-1]): 2 x 2 + 9 = 13 M x D buffers instead of 88 (round-6 VERDICT item 7)
            n_set = nl if per_layer_grads else 1
            n_alt = nl if per_layer_grads else min(2, nl)

            def bufs(n, cols):
                b = [e(M, cols) for _ in range(n)]
                return [b[l % n] for l in range(nl)]

            ws.g_r = bufs(n_alt, D)        # residual grad entering layer l (LN#2 output of layer l+1)
            ws.g_rm = bufs(n_set, D)       # residual grad after layer l's MLP (its LN#1 output)
            ws.g_m = bufs(n_alt, D)        # g_r[l] through the layer's output dropout (dy of linear2)
            ws.g_mm = bufs(n_set, D)       # g_rm[l] through the attention-output dropout (dy of out_proj)
            ws.g_dz = bufs(n_set, 4 * D)   # d(relu pre-activation) (dy of linear1)
            ws.g_dqkv = bufs(n_set, 3 * D)  # d(in_proj output) (dy of in_proj)
            ws.dz = e(M, 4 * D)
            ws.dqkv = e(M, 3 * D)
            ws.do, ws.da = e(M, D), e(M, D)
        return ws

    def drops(self, train: bool, p: float, seed: int, counter: Optional[Tensor], B: int):
        M, D, S, H = B * self.S, self.D, self.S, self.H
        if not train or p <= 0:
            z = Dropout()
            return SimpleNamespace(attn=lambda l: z, d1=lambda l: z, dff=lambda l: z, d2=lambda l: z)
        base = 1 << 40  # distinct from the GPT-2 sites
        blk = 3 * M * D + 4 * M * D + B * H * S * S

        def mk(off):
            return Dropout(p, seed, base + off, counter)

        return SimpleNamespace(attn=lambda l: mk(l * blk), d1=lambda l: mk(l * blk + B * H * S * S),
                               dff=lambda l: mk(l * blk + B * H * S * S + M * D),
                               d2=lambda l: mk(l * blk + B * H * S * S + M * D + 4 * M * D))

    # -- forward ---------------------------------------------------------------------------------------------
    def forward(self, ws, emb_c: Tensor, dr, train: bool) -> None:
        B, S, D, Hl = ws.B, self.S, self.D, self.Hl
        x0 = ws.x[0]
        flat0 = x0.view(B, S * D)
        ops.gemm(emb_c, self.w_lin, flat0[:, : Hl * D], bias=self.b_lin)  # src/models.py:154-159
        ops.broadcast_rows(self.prefix_const, x0.view(-1)[Hl * D:], B, S * D)  # :163-168
        scale = 1.0 / math.sqrt(self.hd)
        for l, w in enumerate(self.layers):
            k = l if train else 0
            x, xn = (ws.x[l], ws.x[l + 1]) if train else (ws.x[l % 2], ws.x[(l + 1) % 2])
            ops.layernorm_fwd(x, w.n1_g, w.n1_b, 1e-5, ws.a1[k], ws.mean1[k], ws.rstd1[k])
            ops.gemm(ws.a1[k], w.in_w, ws.qkv[k], bias=w.in_b)
            ops.attention_fwd(ws.qkv[k], ws.o[k], B=B, S=S, H=self.H, hd=self.hd, scale=scale, causal=False,
                              lse=ws.lse[k], drop=dr.attn(l))
            ops.gemm(ws.o[k], w.out_w, ws.h1[k], bias=w.out_b, resid=x, drop=dr.d1(l))
            ops.layernorm_fwd(ws.h1[k], w.n2_g, w.n2_b, 1e-5, ws.a2[k], ws.mean2[k], ws.rstd2[k])
            ops.gemm(ws.a2[k], w.l1_w, ws.f[k], bias=w.l1_b, act=L.ACT_RELU, drop=dr.dff(l))
            ops.gemm(ws.f[k], w.l2_w, xn, bias=w.l2_b, resid=ws.h1[k], drop=dr.d2(l))
        ws.out = ws.x[self.nl] if train else ws.x[self.nl % 2]

    def prefix_view(self, ws):
        """(tensor whose data_ptr is the first prefix row, batch stride) of the forward output."""
        return ws.out.view(-1)[self.Hl * self.D:], self.S * self.D

    # -- backward --------------------------------------------------------------------------------------------
    def backward(self, ws, emb_c: Tensor, dr, g, dwh: DWHelper, side=None, overwrite: bool = False) -> None:
        """Consumes ws.dout (d of the forward output, rows t<Hl zero); accumulates every parameter grad (writes
        it, with overwrite)."""
        for _, _, fn in self.backward_steps(ws, emb_c, dr, g, dwh, side=side, join_each=False, overwrite=overwrite):
            fn()

    def backward_steps(self, ws, emb_c: Tensor, dr, g, dwh: DWHelper, side=None, join_each: bool = True,
                       overwrite: bool = False, group=None):
        """The backward as [(name, module, fn)]: one step per layer (the top layer first), then the input
        projection ("head": linear + prefix_const). Run in order they are backward(); each step finalises the
        grads of its module's parameters, which is what engine.CaptionTrainer's data-parallel all-reduce buckets
        key on.
        side: a CUDA stream (ops.register_side_stream) for the weight-gradient work — the four K-outer dW products
        and bias column sums per layer, which feed only the optimizer — so it runs beside the dX chain (the dX
        GEMMs, attention and LayerNorm backward). Every gradient buffer those products read is a per-layer buffer
        written once per step (ws.g_*), so a product only has to be ordered after its producer (the fork); the
        main stream joins the side stream at the end of each layer step (join_each: the data-parallel buckets are
        final when their step ends) or only before the head step. Each gradient is the same kernel on the same
        operands as the serial schedule: bitwise the same result.
        overwrite: every parameter gradient is produced exactly once by these steps, so the first micro-batch of an
        accumulation cycle WRITES them (dW beta 0, column sums and LayerNorm parameter sums stored, not added) and
        the trainer skips zeroing the flat gradient buffer first; the stored values equal 0 + the sum bitwise.
        group: side streams (ops.register_side_stream) for the grouped weight gradients: a layer's four K-outer dW
        products are queued at the end of its step, unsplit (no slabs, no reduce pass), one on the main stream and
        the others on these streams, and joined before the next layer's step starts — so they only ever run beside
        each other (432 tiles at the mapper's shape instead of four split launches + reduces in series), never beside
        the dX chain. Each product is one kernel on its own operands and output: deterministic."""
        B, M, S, D, Hl, P = ws.B, ws.M, self.S, self.D, self.Hl, self.P
        acc = not overwrite
        scale = 1.0 / math.sqrt(self.hd)
        st = SimpleNamespace()

        def order(waiter, signaller):
            """waiter runs its later work after everything queued on signaller so far. The event object is kept
            alive (ops.keep_event) until the work behind it has run."""
            ev = torch.cuda.Event()
            ev.record(signaller)
            waiter.wait_event(ev)
            ops.keep_event(ev)

        st.db = []
        st.dw = []

        def wgrad(dy, x, w_out, b_out):
            """dW += dy^T x now; db += colsum(dy) is queued for the layer's one batched column sum (flush_db: every
            dy is a per-layer buffer, alive until the step ends). With a side stream the dW runs there, behind
            everything queued on the main stream."""
            if side is None and group:
                st.dw.append((dy, x, w_out))
                st.db.append((dy, b_out))
                return
            if side is None:
                dwh.dW(dy, x, w_out, M=M, accumulate=acc)
                st.db.append((dy, b_out))
                return
            main = torch.cuda.current_stream()
            order(side, main)
            with torch.cuda.stream(side):
                dwh.dW(dy, x, w_out, M=M, accumulate=acc)
            st.db.append((dy, b_out))

        def flush_dw():
            """The layer's queued dW products, unsplit and side by side (group streams forked from the main stream
            first, so none of them waits for another), then joined back into the main stream — or, group = "fused",
            in one grouped launch on the main stream (icap_gemm_group)."""
            if not st.dw:
                return
            if group == "fused":
                if dwh.dW_group(st.dw, M, accumulate=acc, db_items=st.db):
                    st.db = []  # (the bias gradients went into the same launch)
                st.dw = []
                return
            main = torch.cuda.current_stream()
            sides = list(group[: len(st.dw) - 1])
            for sd in sides:
                order(sd, main)
            for i, (dy, x, w_out) in enumerate(st.dw):
                with torch.cuda.stream(main if i == 0 else sides[i - 1]):
                    dwh.dW(dy, x, w_out, M=M, accumulate=acc, split_k=1)
            for sd in sides:
                order(main, sd)
            st.dw = []

        def flush_db():
            """The layer's bias gradients in one icap_colsum_batch (2 launches instead of 2 per bias)."""
            if not st.db:
                return
            if side is None:
                dwh.db_batch(st.db, M, accumulate=acc)
            else:
                order(side, torch.cuda.current_stream())
                with torch.cuda.stream(side):
                    dwh.db_batch(st.db, M, accumulate=acc)
            st.db = []

        def layer(l):
            if l == self.nl - 1:  # start of the backward: d(output) enters the top layer
                st.r = ws.dout
            w, gl = self.layers[l], g.layers[l]
            r = st.r
            top = dr.d2(l)  # the layer's output dropout (x = h1 + drop(linear2(...)))
            dy = r
            if top.p > 0:
                if l == self.nl - 1:
                    ops.dropout_apply(r, ws.g_m[l], top)
                dy = ws.g_m[l]  # (below the top layer: written by the LN backward above, as its dx_drop)
            wgrad(dy, ws.f[l], gl.l2_w, gl.l2_b)
            ops.gemm(dy, w.l2_wt, ws.g_dz[l], dact=L.ACT_RELU, dact_src=ws.f[l], drop=dr.dff(l))
            wgrad(ws.g_dz[l], ws.a2[l], gl.l1_w, gl.l1_b)
            ops.gemm(ws.g_dz[l], w.l1_wt, ws.da)
            d1 = dr.d1(l)
            ops.layernorm_bwd(ws.h1[l], w.n2_g, ws.mean2[l], ws.rstd2[l], ws.da, ws.g_rm[l], dres=r,
                              dx_drop=ws.g_mm[l] if d1.p > 0 else None, drop=d1, dgamma=gl.n2_g, dbeta=gl.n2_b,
                              workspace=dwh.ln_ws2, param_accumulate=acc, defer_params=LN_PARAM_BATCH)
            dy2 = ws.g_mm[l] if d1.p > 0 else ws.g_rm[l]
            wgrad(dy2, ws.o[l], gl.out_w, gl.out_b)
            ops.gemm(dy2, w.out_wt, ws.do)
            ops.attention_bwd(ws.qkv[l], ws.do, ws.lse[l], ws.g_dqkv[l], B=B, S=S, H=self.H, hd=self.hd,
                              scale=scale, causal=False, drop=dr.attn(l), out=ws.o[l])
            wgrad(ws.g_dqkv[l], ws.a1[l], gl.in_w, gl.in_b)
            ops.gemm(ws.g_dqkv[l], w.in_wt, ws.da)
            nxt = dr.d2(l - 1) if l > 0 else Dropout()
            out = ws.g_r[l - 1] if l > 0 else ws.dres  # d(layer input): the next layer's residual grad / the head's
            ops.layernorm_bwd(ws.x[l], w.n1_g, ws.mean1[l], ws.rstd1[l], ws.da, out, dres=ws.g_rm[l],
                              dx_drop=ws.g_m[l - 1] if (l > 0 and nxt.p > 0) else None, drop=nxt, dgamma=gl.n1_g,
                              dbeta=gl.n1_b, workspace=dwh.ln_ws, param_accumulate=acc, defer_params=LN_PARAM_BATCH)
            if LN_PARAM_BATCH:
                ops.ln_param_reduce_batch([(dwh.ln_ws2, M, D, gl.n2_g, gl.n2_b, acc),
                                           (dwh.ln_ws, M, D, gl.n1_g, gl.n1_b, acc)])
            st.r = out
            flush_dw()
            flush_db()
            if side is not None and (join_each or l == 0):  # the layer's grads are final when its step ends
                order(torch.cuda.current_stream(), side)

        def head():
            # x0 = [linear(emb) ; prefix_const]
            dres = st.r
            d_lin = dres.view(B, S * D)[:, : Hl * D]
            dwh.dW(d_lin, emb_c, g.lin_w, M=B, accumulate=acc)
            dwh.db(d_lin, g.lin_b, M=B, accumulate=acc)
            d_pc = dres.view(B, S * D)[:, Hl * D:]
            ops.colsum(d_pc, g.prefix_const.view(-1), dwh.cs_ws, accumulate=acc, M=B, N=P * D)

        m = self.m
        steps = [(f"layer{l}", m.transformer.layers[l], (lambda l=l: layer(l))) for l in reversed(range(self.nl))]
        steps.append(("head", None, head))
        return steps

    # -- inference -------------------------------------------------------------------------------------------
    @torch.no_grad()
    def infer(self, x: Tensor) -> Tensor:
        B = x.shape[0]
        emb_c = x.to(self.dtype).contiguous()
        ws = self.alloc(B, train=False)
        self.forward(ws, emb_c, self.drops(False, 0.0, 0, None, B), train=False)
        return ws.out.view(B, self.S, self.D)[:, self.Hl:, :]


class MLPMapperCore:
    """Kernel schedule for MLPMappingNetwork (tanh epilogue fused into the first GEMM)."""

    def __init__(self, m: MLPMappingNetwork, dtype: torch.dtype, flat=None):
        from ._lib import require_device

        self.m, self.dtype, self.flat = m, dtype, flat
        self.dev = m.model[0].weight.device
        require_device(self.dev)
        self.P, self.D, self.E = m.prefix_length, m.gpt_dim, m.embed_dim
        self.hid = self.P * self.D // 2
        self.refresh()

    @torch.no_grad()
    def refresh(self) -> None:
        m, dt = self.m, self.dtype
        self.w0, self.b0 = _compute_view(self.flat, m.model[0].weight, dt), m.model[0].bias.data
        self.w2, self.b2 = _compute_view(self.flat, m.model[2].weight, dt), m.model[2].bias.data
        self.w2t = torch.empty((self.w2.shape[1], self.w2.shape[0]), dtype=dt, device=self.dev)
        self.refresh_transposes()

    def dw_cols(self) -> int:
        return max(self.P * self.D, self.hid, self.E)

    def refresh_transposes(self) -> None:
        ops.transpose(self.w2, self.w2t)

    def grads(self, flat) -> SimpleNamespace:
        m = self.m
        return SimpleNamespace(w0=flat.grad(m.model[0].weight), b0=flat.grad(m.model[0].bias),
                               w2=flat.grad(m.model[2].weight), b2=flat.grad(m.model[2].bias))

    def alloc(self, B: int, train: bool) -> SimpleNamespace:
        e = lambda *shape: torch.empty(shape, dtype=self.dtype, device=self.dev)  # noqa: E731
        ws = SimpleNamespace(B=B, M=B)
        ws.h = e(B, self.hid)
        ws.out = e(B, self.P * self.D)
        if train:
            ws.dh = e(B, self.hid)
        return ws

    def drops(self, *a, **k):
        return None

    def forward(self, ws, emb_c: Tensor, dr, train: bool) -> None:
        ops.gemm(emb_c, self.w0, ws.h, bias=self.b0, act=L.ACT_TANH)  # models.py:52-56,71
        ops.gemm(ws.h, self.w2, ws.out, bias=self.b2)

    def prefix_view(self, ws):
        return ws.out, self.P * self.D

    def backward_from(self, dprefix: Tensor, dprefix_ld_rows: int, ws, emb_c: Tensor, g, dwh: DWHelper) -> None:
        """dprefix: [B, P*D] view (row stride dprefix_ld_rows elements) of d(inputs_embeds) prefix rows."""
        B = ws.B
        dwh.dW(dprefix, ws.h, g.w2, M=B)
        dwh.db(dprefix, g.b2, M=B)
        ops.gemm(dprefix, self.w2t, ws.dh, dact=L.ACT_TANH, dact_src=ws.h)
        dwh.dW(ws.dh, emb_c, g.w0, M=B)
        dwh.db(ws.dh, g.b0, M=B)

    @torch.no_grad()
    def infer(self, x: Tensor) -> Tensor:
        B = x.shape[0]
        emb_c = x.to(self.dtype).contiguous()
        ws = self.alloc(B, False)
        self.forward(ws, emb_c, None, False)
        return ws.out.view(B, self.P, self.D)
