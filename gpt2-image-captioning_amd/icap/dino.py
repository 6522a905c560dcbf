"""DINOv3 ViT-L/16 image tower (src/embeddings/dino.py, BASELINE configs[4]) on the icap HIP kernels.

Mirrors the reference's extraction API (`load_dinov3_models`, `get_dinov3_preprocessor`, `extract_dino_embeddings`,
dino.py:19-185) over the DINOv3 backbone as HF's DINOv3ViTModel states it (transformers 5.15,
HF/models/dinov3_vit/modeling_dinov3_vit.py): patch Conv2d (bias) -> [CLS || 4 register tokens || patches] (no
absolute positions) -> 24 pre-LN layers (norm1, fused q/k/v MFMA GEMM with a zero key bias, rotary embedding of
the patch rows' q and k (icap_rope_patches), softmax attention over 201 tokens, o_proj, LayerScale, +res; norm2,
up_proj + exact erf-GELU in the GEMM epilogue, down_proj, LayerScale, +res) -> final norm of the CLS row ->
L2 normalise (dino.py:177-179). LayerScale is folded into o_proj / down_proj (lambda * (W x + b) = (lambda W) x +
lambda b) when the GEMM weights are laid out, so it costs nothing per image.

Offline limits: the reference loads the dino.txt model from torch.hub with gated weights; its
`encode_image` adds a vision head on top of this backbone that neither the hub code nor its weights exist for
here. The tower therefore returns the backbone's pooled CLS (1024-d, pinned to HF DINOv3ViTModel goldens).
"""

from __future__ import annotations

import math
import os
from dataclasses import dataclass
from types import SimpleNamespace
from typing import Dict, Optional, Tuple

import torch
import torch.nn as nn

from . import _lib as L
from . import ops
from .weights import det_tensor

Tensor = torch.Tensor

WEIGHTS_FILE = "dinov3_vitl16_dinotxt_vision_head_and_text_encoder-a442d8f5.pth"  # dino.py:11-12
BACKBONE_WEIGHTS_FILE = "dinov3_vitl16_pretrain_lvd1689m-8aa4cbdd.pth"
# what extract_dino_embeddings stores: the backbone's L2-normalised pooled CLS, NOT the dino.txt head's output
# (the reference's encode_image); written as the .pt file's "feature" field so the two cannot be mixed silently
FEATURE_NAME = "dinov3_vitl16_backbone_pooled_cls"
RESIZE_DEFAULT_SIZE = 256  # dino.py:13-16
CROP_DEFAULT_SIZE = 224
IMAGENET_DEFAULT_MEAN = (0.485, 0.456, 0.406)
IMAGENET_DEFAULT_STD = (0.229, 0.224, 0.225)


@dataclass
class DinoConfig:  # DINOv3 ViT-L/16 (dinov3_vitl16, 4 registers, RoPE theta 100, LayerScale, key without bias)
    hidden_size: int = 1024
    num_hidden_layers: int = 24
    num_attention_heads: int = 16
    intermediate_size: int = 4096
    patch_size: int = 16
    image_size: int = 224
    num_channels: int = 3
    num_register_tokens: int = 4
    layer_norm_eps: float = 1e-5
    rope_theta: float = 100.0

    @property
    def embedding_dim(self) -> int:
        return self.hidden_size


class _Emb(nn.Module):
    def __init__(self, c: DinoConfig):
        super().__init__()
        d = c.hidden_size
        self.cls_token = nn.Parameter(torch.zeros(1, 1, d))
        self.mask_token = nn.Parameter(torch.zeros(1, 1, d))
        self.register_tokens = nn.Parameter(torch.zeros(1, c.num_register_tokens, d))
        self.patch_embeddings = nn.Conv2d(c.num_channels, d, c.patch_size, c.patch_size, bias=True)


class _Attn(nn.Module):
    def __init__(self, d):
        super().__init__()
        self.q_proj, self.k_proj = nn.Linear(d, d), nn.Linear(d, d, bias=False)
        self.v_proj, self.o_proj = nn.Linear(d, d), nn.Linear(d, d)


class _Scale(nn.Module):
    def __init__(self, d):
        super().__init__()
        self.lambda1 = nn.Parameter(torch.ones(d))


class _MLP(nn.Module):
    def __init__(self, d, f):
        super().__init__()
        self.up_proj, self.down_proj = nn.Linear(d, f), nn.Linear(f, d)


class _Layer(nn.Module):
    def __init__(self, c: DinoConfig):
        super().__init__()
        d = c.hidden_size
        self.norm1 = nn.LayerNorm(d, eps=c.layer_norm_eps)
        self.attention = _Attn(d)
        self.layer_scale1 = _Scale(d)
        self.norm2 = nn.LayerNorm(d, eps=c.layer_norm_eps)
        self.mlp = _MLP(d, c.intermediate_size)
        self.layer_scale2 = _Scale(d)


class _Encoder(nn.Module):
    def __init__(self, c: DinoConfig):
        super().__init__()
        self.layer = nn.ModuleList([_Layer(c) for _ in range(c.num_hidden_layers)])


def rope_tables(c: DinoConfig, h_patches: int, w_patches: int) -> Tuple[Tensor, Tensor]:
    """Patch-token cos / sin [h*w, hd] fp32 (modeling_dinov3_vit.py:96-121,153-200 in eval mode): patch-centre
    coordinates in [-1, 1], inv_freq = 1 / theta^(arange(0, 1, 4/hd)), angles = 2 pi coord inv_freq per axis,
    flattened (y, x) and tiled twice. A per-geometry constant like a position table, built once on the host."""
    hd = c.hidden_size // c.num_attention_heads
    inv_freq = 1 / c.rope_theta ** torch.arange(0, 1, 4 / hd, dtype=torch.float32)
    ch = torch.arange(0.5, h_patches, dtype=torch.float32) / h_patches
    cw = torch.arange(0.5, w_patches, dtype=torch.float32) / w_patches
    coords = 2.0 * torch.stack(torch.meshgrid(ch, cw, indexing="ij"), dim=-1).flatten(0, 1) - 1.0
    angles = (2 * math.pi * coords[:, :, None] * inv_freq[None, None, :]).flatten(1, 2).tile(2)
    return torch.cos(angles).contiguous(), torch.sin(angles).contiguous()


class DINOv3ImageTower(nn.Module):
    """DINOv3 ViT backbone with HF DINOv3ViTModel key names. Frozen (dino.py:80 eval mode, never trained)."""

    def __init__(self, config: Optional[DinoConfig] = None):
        super().__init__()
        self.config = config or DinoConfig()
        c = self.config
        self.embeddings = _Emb(c)
        self.model = _Encoder(c)
        self.norm = nn.LayerNorm(c.hidden_size, eps=c.layer_norm_eps)
        for p in self.parameters():
            p.requires_grad = False
        self._core = None
        self._core_key = None

    @classmethod
    def random_init(cls, config: Optional[DinoConfig] = None, seed: int = 0) -> "DINOv3ImageTower":
        """Deterministic random weights of the architecture (the gated checkpoint is not available offline)."""
        m = cls(config)
        c = m.config
        d, r = c.hidden_size, c.num_register_tokens
        sd = {
            "embeddings.cls_token": det_tensor(seed, "d.cls", (1, 1, d), 0.5),
            "embeddings.mask_token": torch.zeros(1, 1, d),
            "embeddings.register_tokens": det_tensor(seed, "d.reg", (1, r, d), 0.5),
            "embeddings.patch_embeddings.weight": det_tensor(
                seed, "d.patch.w", (d, c.num_channels, c.patch_size, c.patch_size), 0.02),
            "embeddings.patch_embeddings.bias": det_tensor(seed, "d.patch.b", (d,), 0.02),
            "norm.weight": det_tensor(seed, "d.ln.w", (d,), 0.05, 1.0),
            "norm.bias": det_tensor(seed, "d.ln.b", (d,), 0.02),
        }
        for i in range(c.num_hidden_layers):
            p = f"model.layer.{i}."
            for nm in ("q", "k", "v", "o"):
                sd[p + f"attention.{nm}_proj.weight"] = det_tensor(seed, p + nm + ".w", (d, d), 0.02)
                if nm != "k":
                    sd[p + f"attention.{nm}_proj.bias"] = det_tensor(seed, p + nm + ".b", (d,), 0.02)
            sd[p + "mlp.up_proj.weight"] = det_tensor(seed, p + "up.w", (c.intermediate_size, d), 0.02)
            sd[p + "mlp.up_proj.bias"] = det_tensor(seed, p + "up.b", (c.intermediate_size,), 0.02)
            sd[p + "mlp.down_proj.weight"] = det_tensor(seed, p + "down.w", (d, c.intermediate_size), 0.02)
            sd[p + "mlp.down_proj.bias"] = det_tensor(seed, p + "down.b", (d,), 0.02)
            for nm in ("norm1", "norm2"):
                sd[p + nm + ".weight"] = det_tensor(seed, p + nm + ".w", (d,), 0.05, 1.0)
                sd[p + nm + ".bias"] = det_tensor(seed, p + nm + ".b", (d,), 0.02)
            sd[p + "layer_scale1.lambda1"] = det_tensor(seed, p + "ls1", (d,), 0.1, 0.5)
            sd[p + "layer_scale2.lambda1"] = det_tensor(seed, p + "ls2", (d,), 0.1, 0.5)
        m.load_state_dict(sd, strict=True)
        return m

    def load_backbone_state_dict(self, sd: Dict[str, Tensor]):
        """An HF DINOv3ViTModel state dict, or Meta's native DINOv3 checkpoint layout (the file the reference's
        torch.hub loader reads, BACKBONE_WEIGHTS_FILE), converted by meta_to_hf_state_dict. A 'dinov3.' /
        'backbone.' prefix is dropped."""
        out = {}
        for k, v in sd.items():
            for pre in ("dinov3.", "backbone."):
                if k.startswith(pre):
                    k = k[len(pre):]
            out[k] = v
        if is_meta_layout(out):
            out = meta_to_hf_state_dict(out, self.config)
        self._core = None
        return self.load_state_dict(out, strict=True)

    @property
    def device(self):
        return self.norm.weight.device

    def core(self, dtype: torch.dtype = torch.bfloat16) -> "DinoCore":
        key = (dtype, self.device)
        if self._core is None or self._core_key != key:
            self._core = DinoCore(self, dtype)
            self._core_key = key
        return self._core

    @torch.no_grad()
    def pooler_output(self, pixel_values: Tensor, compute_dtype: torch.dtype = torch.bfloat16) -> Tensor:
        """`DINOv3ViTModel(pixel_values).pooler_output` (the normed CLS row) [B, hidden] fp32."""
        return self.core(compute_dtype).features(pixel_values, normalize=False)

    @torch.no_grad()
    def embed(self, pixel_values: Tensor, compute_dtype: torch.dtype = torch.bfloat16) -> Tensor:
        """L2-normalised pooled CLS (dino.py:177-179)."""
        return self.core(compute_dtype).features(pixel_values, normalize=True)

    @torch.no_grad()
    def encode_image(self, pixel_values: Tensor, compute_dtype: torch.dtype = torch.bfloat16) -> Tensor:
        """dino.py:175 `encode_image` stand-in: the backbone's pooled CLS (un-normalised) [B, 1024]."""
        return self.core(compute_dtype).features(pixel_values, normalize=False)


def is_meta_layout(sd: Dict[str, Tensor]) -> bool:
    return any(k.startswith("blocks.") or k in ("storage_tokens", "patch_embed.proj.weight") for k in sd)


def meta_to_hf_state_dict(sd: Dict[str, Tensor], c: Optional[DinoConfig] = None) -> Dict[str, Tensor]:
    """Meta's DINOv3 ViT checkpoint keys -> HF DINOv3ViTModel keys (the layout DINOv3ImageTower holds).

    cls_token / mask_token / storage_tokens -> embeddings.{cls_token, mask_token, register_tokens} (reshaped to
    [1, n, D]); patch_embed.proj -> embeddings.patch_embeddings; blocks.N.attn.qkv [3D, D] (+ bias [3D]) split into
    q / k / v, the key bias dropped (Meta zeroes it through attn.qkv.bias_mask; HF's k_proj has no bias);
    attn.proj -> attention.o_proj; ls{1,2}.gamma -> layer_scale{1,2}.lambda1; mlp.fc1 / fc2 -> mlp.up_proj /
    down_proj; norm -> norm. rope_embed.periods is a derived constant: it is checked against this tower's RoPE
    frequencies (rope_tables) and dropped. Any other key is passed through, so a strict load names it."""
    c = c or DinoConfig()
    D = c.hidden_size
    out: Dict[str, Tensor] = {}
    for k, v in sd.items():
        if k in ("cls_token", "mask_token", "storage_tokens"):
            name = {"cls_token": "cls_token", "mask_token": "mask_token", "storage_tokens": "register_tokens"}[k]
            out["embeddings." + name] = v.reshape(1, -1, D)
        elif k.startswith("patch_embed.proj."):
            out["embeddings.patch_embeddings." + k.split(".")[-1]] = v
        elif k == "rope_embed.periods":
            hd = D // c.num_attention_heads
            inv = 1 / c.rope_theta ** torch.arange(0, 1, 4 / hd, dtype=torch.float64)
            if v.numel() != inv.numel() or float((1.0 / v.double() - inv).abs().max()) > 1e-6 * float(inv.max()):
                raise ValueError("rope_embed.periods does not match the RoPE frequencies of this configuration")
        elif k.startswith("blocks."):
            _, i, rest = k.split(".", 2)
            p = f"model.layer.{i}."
            if rest in ("attn.qkv.weight", "attn.qkv.bias"):
                kind = rest.split(".")[-1]
                q, kk, vv = v.chunk(3, 0)
                out[p + f"attention.q_proj.{kind}"] = q
                out[p + f"attention.v_proj.{kind}"] = vv
                if kind == "weight":
                    out[p + "attention.k_proj.weight"] = kk
            elif rest == "attn.qkv.bias_mask":
                continue
            elif rest.startswith("attn.proj."):
                out[p + "attention.o_proj." + rest.split(".")[-1]] = v
            elif rest in ("ls1.gamma", "ls2.gamma"):
                out[p + f"layer_scale{rest[2]}.lambda1"] = v
            elif rest.startswith("mlp.fc1."):
                out[p + "mlp.up_proj." + rest.split(".")[-1]] = v
            elif rest.startswith("mlp.fc2."):
                out[p + "mlp.down_proj." + rest.split(".")[-1]] = v
            else:  # norm1 / norm2 keep their names
                out[p + rest] = v
        else:
            out[k] = v
    return out


class DinoCore:
    """Kernel schedule of one DINOv3ImageTower in one compute dtype (GEMM-layout weights, per-batch workspaces)."""

    def __init__(self, m: DINOv3ImageTower, dtype: torch.dtype):
        from ._lib import require_device

        self.m, self.dtype = m, dtype
        self.dev = m.device
        require_device(self.dev)
        c = m.config
        self.c = c
        self.D, self.H = c.hidden_size, c.num_attention_heads
        self.hd = self.D // self.H
        self.G = c.image_size // c.patch_size
        self.NP = 1 + c.num_register_tokens
        self.S = self.G * self.G + self.NP
        self._ws = {}
        self.refresh()

    def _cvt(self, t: Tensor) -> Tensor:
        t2 = t.reshape(t.shape[0], -1)
        if self.dtype == torch.float32:
            return t2.contiguous()
        out = torch.empty(t2.shape, dtype=self.dtype, device=self.dev)
        ops.convert(t2.contiguous(), out)
        return out

    @torch.no_grad()
    def refresh(self):
        m, D = self.m, self.D
        e = m.embeddings
        wp = e.patch_embeddings.weight.data.reshape(D, -1)  # [D, C*p*p] in (c, ky, kx) order = im2col's
        self.Kp = (wp.shape[1] + 7) // 8 * 8
        if self.Kp != wp.shape[1]:
            wp = torch.nn.functional.pad(wp, (0, self.Kp - wp.shape[1]))
        self.w_patch = self._cvt(wp)
        self.b_patch = e.patch_embeddings.bias.data.contiguous()
        self.prefix = torch.cat([e.cls_token.data.reshape(1, D), e.register_tokens.data.reshape(-1, D)], 0).contiguous()
        self.lnf = (m.norm.weight.data, m.norm.bias.data)
        cos, sin = rope_tables(self.c, self.G, self.G)
        self.cos, self.sin = cos.to(self.dev), sin.to(self.dev)
        self.layers = []
        for lay in m.model.layer:
            a = lay.attention
            w = SimpleNamespace()
            w.qkv_w = self._cvt(torch.cat([a.q_proj.weight.data, a.k_proj.weight.data, a.v_proj.weight.data], 0))
            w.qkv_b = torch.cat([a.q_proj.bias.data, torch.zeros_like(a.q_proj.bias.data), a.v_proj.bias.data],
                                0).contiguous()
            l1, l2 = lay.layer_scale1.lambda1.data, lay.layer_scale2.lambda1.data
            w.o_w = self._cvt(a.o_proj.weight.data * l1[:, None])  # LayerScale folded into the output rows
            w.o_b = (a.o_proj.bias.data * l1).contiguous()
            w.up_w, w.up_b = self._cvt(lay.mlp.up_proj.weight.data), lay.mlp.up_proj.bias.data.contiguous()
            w.down_w = self._cvt(lay.mlp.down_proj.weight.data * l2[:, None])
            w.down_b = (lay.mlp.down_proj.bias.data * l2).contiguous()
            w.ln1 = (lay.norm1.weight.data, lay.norm1.bias.data)
            w.ln2 = (lay.norm2.weight.data, lay.norm2.bias.data)
            self.layers.append(w)

    def alloc(self, B: int) -> SimpleNamespace:
        if B in self._ws:
            return self._ws[B]
        c, D, dt, dev = self.c, self.D, self.dtype, self.dev
        M = B * self.S
        e = lambda *shape, dtype=dt: torch.empty(shape, dtype=dtype, device=dev)  # noqa: E731
        ws = SimpleNamespace(B=B, M=M)
        if dt != torch.bfloat16:  # (bf16: icap_patch_embed reads the pixels itself — no patch matrix)
            ws.patches = e(B * self.G * self.G, self.Kp)
            ws.pe = e(B * self.G * self.G, D)
        ws.x, ws.h1, ws.a, ws.o = e(M, D), e(M, D), e(M, D), e(M, D)
        ws.qkv = e(M, 3 * D)
        ws.f = e(M, c.intermediate_size)
        ws.cls = e(B, D)
        ws.xc = e(B, D)  # the last layer's CLS rows (see run)
        ws.pool = e(B, D, dtype=torch.float32)
        ws.emb = e(B, D, dtype=torch.float32)
        self._ws = {B: ws}  # keep only the latest batch size
        return ws

    def run(self, ws, pixels: Tensor) -> Tensor:
        """Kernel schedule; fills ws.pool (pooler_output, fp32) and ws.emb (L2-normalised) — graph-capturable."""
        c, D, B, S = self.c, self.D, ws.B, self.S
        eps = c.layer_norm_eps
        if self.dtype == torch.bfloat16:  # patch Conv2d + [CLS || registers || patches], pixels read by the GEMM
            ops.patch_embed(pixels, self.w_patch, ws.x, patch=c.patch_size, prefix=self.prefix, bias=self.b_patch)
        else:
            ops.im2col_patches(pixels, ws.patches, c.patch_size)
            ops.gemm(ws.patches, self.w_patch, ws.pe, bias=self.b_patch)  # Conv2d(stride=patch, bias) as a GEMM
            ops.prefix_embed(ws.pe, self.prefix, ws.x, B, self.G * self.G, D)  # [CLS || registers || patches]
        scale = self.hd ** -0.5
        nl = len(self.layers)
        for i, w in enumerate(self.layers):
            ops.layernorm_fwd(ws.x, w.ln1[0], w.ln1[1], eps, ws.a, None, None)
            ops.gemm(ws.a, w.qkv_w, ws.qkv, bias=w.qkv_b)
            ops.rope_patches(ws.qkv, self.cos, self.sin, B=B, S=S, NP=self.NP, H=self.H, hd=self.hd)
            ops.attention_fwd(ws.qkv, ws.o, B=B, S=S, H=self.H, hd=self.hd, scale=scale, causal=False)
            if i == nl - 1:
                # last layer: pooler_output is the normed CLS row (modeling_dinov3_vit.py:540-541), so past attention
                # the layer runs on the B CLS rows (strided views, row b at b*S*D); the registers' and patches' keys /
                # values were used above
                o_c, x_c = ws.o.view(B, S * D)[:, :D], ws.x.view(B, S * D)[:, :D]
                h1, a, f = ws.h1[:B], ws.a[:B], ws.f[:B]
                ops.gemm(o_c, w.o_w, h1, bias=w.o_b, resid=x_c)
                ops.layernorm_fwd(h1, w.ln2[0], w.ln2[1], eps, a, None, None)
                ops.gemm(a, w.up_w, f, bias=w.up_b, act=L.ACT_GELU_ERF)
                ops.gemm(f, w.down_w, ws.xc, bias=w.down_b, resid=h1)
                break
            ops.gemm(ws.o, w.o_w, ws.h1, bias=w.o_b, resid=ws.x)
            ops.layernorm_fwd(ws.h1, w.ln2[0], w.ln2[1], eps, ws.a, None, None)
            ops.gemm(ws.a, w.up_w, ws.f, bias=w.up_b, act=L.ACT_GELU_ERF)
            ops.gemm(ws.f, w.down_w, ws.x, bias=w.down_b, resid=ws.h1)
        cls_rows = ws.xc  # CLS token of every image after the last layer
        ops.layernorm_fwd(cls_rows, self.lnf[0], self.lnf[1], eps, ws.cls, None, None, rows=B)
        if ws.cls.dtype == torch.float32:
            ws.pool.copy_(ws.cls)
        else:
            ops.convert(ws.cls, ws.pool)
        ops.l2norm_rows(ws.pool, ws.emb)
        return ws.emb

    @torch.no_grad()
    def features(self, pixels: Tensor, normalize: bool = True) -> Tensor:
        if pixels.dtype != torch.float32 or not pixels.is_contiguous():
            pixels = pixels.float().contiguous()
        ws = self.alloc(pixels.shape[0])
        self.run(ws, pixels)
        return (ws.emb if normalize else ws.pool).clone()


# --------------------------------------------------------------------------- reference-shaped API (dino.py:19-185)


class DinoImageProcessor:
    """get_dinov3_preprocessor() (dino.py:86-137) without torchvision: RGB uint8 -> resize the shorter side to
    `resize_size` (bicubic, antialiased, on the uint8 tensor as torchvision v2 does after ToImage; long side
    int(size * long / short)) -> centre crop `crop_size` (offsets int(round((h - crop) / 2))) -> x 1/255 ->
    (x - mean) / std. torchvision is not installed, so this restatement is unpinned."""

    def __init__(self, resize_size: int = RESIZE_DEFAULT_SIZE, crop_size: int = CROP_DEFAULT_SIZE,
                 mean=IMAGENET_DEFAULT_MEAN, std=IMAGENET_DEFAULT_STD):
        self.resize_size, self.crop_size, self.mean, self.std = resize_size, crop_size, mean, std

    def one(self, im) -> Tensor:
        import numpy as np

        if isinstance(im, torch.Tensor):
            t = im
        else:
            if not isinstance(im, np.ndarray):
                im = np.asarray(im.convert("RGB"))
            t = torch.from_numpy(np.ascontiguousarray(im))
        t = t.permute(2, 0, 1).float()[None]  # [1, 3, h, w]
        h, w = t.shape[-2:]
        s = self.resize_size
        nh, nw = (s, int(s * w / h)) if h <= w else (int(s * h / w), s)
        t = torch.nn.functional.interpolate(t, size=(nh, nw), mode="bicubic", align_corners=False, antialias=True)
        t = t.clamp_(0, 255).round_()
        cs = self.crop_size
        top, left = int(round((nh - cs) / 2.0)), int(round((nw - cs) / 2.0))
        t = t[0, :, top:top + cs, left:left + cs] / 255.0
        m = torch.tensor(self.mean, dtype=torch.float32)[:, None, None]
        sd = torch.tensor(self.std, dtype=torch.float32)[:, None, None]
        return (t - m) / sd

    def __call__(self, images=None, return_tensors: str = "pt"):
        if not isinstance(images, (list, tuple)):
            images = [images]
        return SimpleNamespace(pixel_values=torch.stack([self.one(im) for im in images]))


def get_dinov3_preprocessor(*, resize_size: int = RESIZE_DEFAULT_SIZE, crop_size: int = CROP_DEFAULT_SIZE,
                            mean=IMAGENET_DEFAULT_MEAN, std=IMAGENET_DEFAULT_STD) -> DinoImageProcessor:
    """dino.py:121-137."""
    return DinoImageProcessor(resize_size, crop_size, mean, std)


def load_dinov3_models(model_weights_dir: Optional[str] = None, repo_or_dir: str = "facebookresearch/dinov3",
                       source: str = "github", device: Optional[torch.device] = None):
    """dino.py:19-82: (model, tokenizer). Offline: the backbone weights come from BACKBONE_WEIGHTS_FILE in
    `model_weights_dir` when it holds an HF-layout DINOv3ViTModel state dict, else a deterministic random init of the
    ViT-L/16 architecture; the dino.txt text tokenizer is not part of the image path (None). The reference's
    FileNotFoundError rule for a directory missing either file is kept."""
    device = device or torch.device("cuda")
    print(f"Loading DINOv3 model from '{model_weights_dir}' on device: {device}...")
    model = DINOv3ImageTower(DinoConfig())
    if model_weights_dir is not None:
        names = set(os.listdir(model_weights_dir))
        for f in (WEIGHTS_FILE, BACKBONE_WEIGHTS_FILE):
            if f not in names:
                raise FileNotFoundError(f"Could not find '{f}' in directory '{model_weights_dir}'")
        sd = torch.load(os.path.join(model_weights_dir, BACKBONE_WEIGHTS_FILE), map_location="cpu", weights_only=True)
        model.load_backbone_state_dict(sd)
        import warnings

        warnings.warn(f"icap.dino: '{WEIGHTS_FILE}' (the dino.txt vision head) is present but not applied: "
                      f"embeddings are the backbone's pooled CLS ({FEATURE_NAME}), not the reference's "
                      "encode_image output; extraction files record this in their 'feature' field", stacklevel=2)
    else:
        model = DINOv3ImageTower.random_init(DinoConfig())
    return model.to(device).eval(), None


@torch.no_grad()
def extract_dino_embeddings(image_dir: str, output_path: str, dino_model: DINOv3ImageTower,
                            dino_processor: DinoImageProcessor, batch_size: int = 32, num_workers: int = 4,
                            device: Optional[torch.device] = None) -> None:
    """dino.py:140-185: every image of a directory -> {"filenames", "embeddings"} .pt (L2-normalised features, the
    reference's format and file order; decode in `num_workers` DataLoader processes)."""
    from .images import extract_directory

    n = extract_directory(image_dir, output_path, dino_model.embed, dino_processor, dino_model.config.embedding_dim,
                          batch_size, num_workers, device or dino_model.device, feature=FEATURE_NAME)
    print(f"Saving {n} embeddings to {output_path}...")
