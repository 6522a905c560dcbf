"""CLIP ViT image tower (src/embeddings/clip.py) on the icap HIP kernels.

Mirrors the reference's extraction API (`load_clip_model`, `extract_clip_embedding_from_image`,
`extract_clip_embeddings`, clip.py:10-149) over a CLIP vision tower whose
parameters use HF CLIPModel key names (vision_model.*, visual_projection.weight), so an
HF safetensors checkpoint loads directly. Forward = HF/models/clip/modeling_clip.py:
embeddings :138-219 -> pre_layrnorm :642 -> 12 pre-LN layers :353-384 (q/k/v fused into
one MFMA GEMM, quick_gelu fused into fc1) -> post_layernorm(CLS) :650-651 ->
visual_projection :751 -> L2 normalise (clip.py:135-137).
"""

from __future__ import annotations

import math
import os
from dataclasses import dataclass
from types import SimpleNamespace
from typing import List, Optional, Tuple

import torch
import torch.nn as nn

from . import _lib as L
from . import gpt2 as _gpt2
from . import ops
from .gpt2 import fold_layernorm
from .weights import det_tensor

Tensor = torch.Tensor

CLIP_MEAN = (0.48145466, 0.4578275, 0.40821073)  # CLIPImageProcessor defaults
CLIP_STD = (0.26862954, 0.26130258, 0.27577711)


@dataclass
class CLIPVisionConfig:  # HF/models/clip/configuration_clip.py (ViT-B/32 defaults)
    hidden_size: int = 768
    num_hidden_layers: int = 12
    num_attention_heads: int = 12
    intermediate_size: int = 3072
    patch_size: int = 32
    image_size: int = 224
    num_channels: int = 3
    projection_dim: int = 512
    layer_norm_eps: float = 1e-5

    @classmethod
    def vit_l14(cls):  # openai/clip-vit-large-patch14 (BASELINE configs[3])
        return cls(hidden_size=1024, num_hidden_layers=24, num_attention_heads=16, intermediate_size=4096,
                   patch_size=14, projection_dim=768)


class _Emb(nn.Module):
    def __init__(self, c: CLIPVisionConfig):
        super().__init__()
        g = c.image_size // c.patch_size
        self.class_embedding = nn.Parameter(torch.zeros(c.hidden_size))
        self.patch_embedding = nn.Conv2d(c.num_channels, c.hidden_size, c.patch_size, c.patch_size, bias=False)
        self.position_embedding = nn.Embedding(g * g + 1, c.hidden_size)


class _Attn(nn.Module):
    def __init__(self, d):
        super().__init__()
        self.q_proj, self.k_proj, self.v_proj, self.out_proj = (nn.Linear(d, d) for _ in range(4))


class _MLP(nn.Module):
    def __init__(self, d, i):
        super().__init__()
        self.fc1 = nn.Linear(d, i)
        self.fc2 = nn.Linear(i, d)


class _Layer(nn.Module):
    def __init__(self, c: CLIPVisionConfig):
        super().__init__()
        d = c.hidden_size
        self.self_attn = _Attn(d)
        self.layer_norm1 = nn.LayerNorm(d, eps=c.layer_norm_eps)
        self.mlp = _MLP(d, c.intermediate_size)
        self.layer_norm2 = nn.LayerNorm(d, eps=c.layer_norm_eps)


class _Encoder(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.layers = nn.ModuleList([_Layer(c) for _ in range(c.num_hidden_layers)])


class _VisionModel(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.embeddings = _Emb(c)
        self.pre_layrnorm = nn.LayerNorm(c.hidden_size, eps=c.layer_norm_eps)  # sic (HF name)
        self.encoder = _Encoder(c)
        self.post_layernorm = nn.LayerNorm(c.hidden_size, eps=c.layer_norm_eps)


class CLIPVisionTower(nn.Module):
    """The image half of HF CLIPModel: `get_image_features(pixel_values)` (modeling_clip.py:719-752)."""

    def __init__(self, config: Optional[CLIPVisionConfig] = None):
        super().__init__()
        self.config = config or CLIPVisionConfig()
        self.vision_model = _VisionModel(self.config)
        self.visual_projection = nn.Linear(self.config.hidden_size, self.config.projection_dim, bias=False)
        for p in self.parameters():
            p.requires_grad = False  # frozen encoder (clip.py:30 eval mode, no training)
        self._core = None
        self._core_key = None

    @classmethod
    def random_init(cls, config: Optional[CLIPVisionConfig] = None, seed: int = 0) -> "CLIPVisionTower":
        m = cls(config)
        c = m.config
        d, g = c.hidden_size, c.image_size // c.patch_size
        v = "vision_model."
        sd = {
            v + "embeddings.class_embedding": det_tensor(seed, "c.cls", (d,), 0.5),
            v + "embeddings.patch_embedding.weight": det_tensor(seed, "c.patch", (d, c.num_channels, c.patch_size, c.patch_size), 0.02),
            v + "embeddings.position_embedding.weight": det_tensor(seed, "c.pos", (g * g + 1, d), 0.02),
            v + "pre_layrnorm.weight": det_tensor(seed, "c.pre.w", (d,), 0.05, 1.0),
            v + "pre_layrnorm.bias": det_tensor(seed, "c.pre.b", (d,), 0.02),
            v + "post_layernorm.weight": det_tensor(seed, "c.post.w", (d,), 0.05, 1.0),
            v + "post_layernorm.bias": det_tensor(seed, "c.post.b", (d,), 0.02),
            "visual_projection.weight": det_tensor(seed, "c.proj", (c.projection_dim, d), 0.02),
        }
        for i in range(c.num_hidden_layers):
            p = v + f"encoder.layers.{i}."
            for nm in ("q_proj", "k_proj", "v_proj", "out_proj"):
                sd[p + f"self_attn.{nm}.weight"] = det_tensor(seed, p + nm + ".w", (d, d), 0.02)
                sd[p + f"self_attn.{nm}.bias"] = det_tensor(seed, p + nm + ".b", (d,), 0.02)
            sd[p + "layer_norm1.weight"] = det_tensor(seed, p + "ln1.w", (d,), 0.05, 1.0)
            sd[p + "layer_norm1.bias"] = det_tensor(seed, p + "ln1.b", (d,), 0.02)
            sd[p + "layer_norm2.weight"] = det_tensor(seed, p + "ln2.w", (d,), 0.05, 1.0)
            sd[p + "layer_norm2.bias"] = det_tensor(seed, p + "ln2.b", (d,), 0.02)
            sd[p + "mlp.fc1.weight"] = det_tensor(seed, p + "fc1.w", (c.intermediate_size, d), 0.02)
            sd[p + "mlp.fc1.bias"] = det_tensor(seed, p + "fc1.b", (c.intermediate_size,), 0.02)
            sd[p + "mlp.fc2.weight"] = det_tensor(seed, p + "fc2.w", (d, c.intermediate_size), 0.02)
            sd[p + "mlp.fc2.bias"] = det_tensor(seed, p + "fc2.b", (d,), 0.02)
        m.load_state_dict(sd, strict=True)
        return m

    @property
    def device(self):
        return self.visual_projection.weight.device

    def core(self, dtype: torch.dtype = torch.bfloat16) -> "ClipCore":
        key = (dtype, self.device)
        if self._core is None or self._core_key != key:
            self._core = ClipCore(self, dtype)
            self._core_key = key
        return self._core

    @torch.no_grad()
    def get_image_features(self, pixel_values: Tensor, compute_dtype: torch.dtype = torch.bfloat16) -> Tensor:
        """Projected (un-normalised) image features [B, projection_dim] fp32."""
        return self.core(compute_dtype).features(pixel_values, normalize=False)

    @torch.no_grad()
    def embed(self, pixel_values: Tensor, compute_dtype: torch.dtype = torch.bfloat16) -> Tensor:
        """L2-normalised features (src/embeddings/clip.py:132-137)."""
        return self.core(compute_dtype).features(pixel_values, normalize=True)


class ClipCore:
    def __init__(self, m: CLIPVisionTower, dtype: torch.dtype):
        from ._lib import require_device

        self.m, self.dtype = m, dtype
        self.dev = m.device
        require_device(self.dev)
        c = m.config
        self.c = c
        self.D, self.H = c.hidden_size, c.num_attention_heads
        self.hd = self.D // self.H
        self.G = c.image_size // c.patch_size
        self.S = self.G * self.G + 1
        self.refresh()
        self._ws = {}

    def _cvt(self, t: Tensor) -> Tensor:
        t2 = t.reshape(t.shape[0], -1)
        if self.dtype == torch.float32:
            return t2.contiguous()
        out = torch.empty(t2.shape, dtype=self.dtype, device=self.dev)
        ops.convert(t2.contiguous(), out)
        return out

    @torch.no_grad()
    def refresh(self):
        vm, dt = self.m.vision_model, self.dtype
        # bf16: layer_norm1 (layers >= 1) / layer_norm2 (all but the last) folded into the QKV / fc1 tile GEMMs, the row
        # statistics handed over from the producing GEMMs' epilogues (icap_gemm_args.ln_stats_out / ln_stats_in)
        self.fold = dt == torch.bfloat16 and ops.ln_fold_ok(self.D) and _gpt2.TRAIN_LN_FOLD
        # [D, C*p*p] (c, ky, kx) order, zero-padded to the 8-multiple row of icap_im2col_patches (p = 14: 592)
        wp = vm.embeddings.patch_embedding.weight.data.reshape(self.D, -1)
        self.Kp = (wp.shape[1] + 7) // 8 * 8
        # bf16 towers: the fused gather GEMM (icap_patch_embed) where it is the faster form. Measured round 6
        # (profiles/r06_patch_bench.txt, B = 128): ViT-B/32 fused 101.0 us vs im2col + the split-role GEMM (96 x 128
        # tiles) + vit_embed 85.8 us — the fused kernel's 6 column tiles each re-gather their rows' fp32 pixels;
        # ViT-L/14 fused 200.5 vs 221.5 us (K = 588: the GEMM is short, the im2col pass is not)
        self.fused_patch = self.dtype == torch.bfloat16 and self.c.patch_size != 32
        if self.Kp != wp.shape[1]:
            wp = torch.nn.functional.pad(wp, (0, self.Kp - wp.shape[1]))
        self.w_patch = self._cvt(wp)
        self.cls = vm.embeddings.class_embedding.data
        self.pos = vm.embeddings.position_embedding.weight.data
        self.pre = (vm.pre_layrnorm.weight.data, vm.pre_layrnorm.bias.data)
        self.post = (vm.post_layernorm.weight.data, vm.post_layernorm.bias.data)
        self.w_proj = self._cvt(self.m.visual_projection.weight.data)
        self.layers = []
        for lay in vm.encoder.layers:
            a = lay.self_attn
            w = SimpleNamespace()
            w.qkv_w = self._cvt(torch.cat([a.q_proj.weight.data, a.k_proj.weight.data, a.v_proj.weight.data], 0))
            w.qkv_b = torch.cat([a.q_proj.bias.data, a.k_proj.bias.data, a.v_proj.bias.data], 0).contiguous()
            w.out_w, w.out_b = self._cvt(a.out_proj.weight.data), a.out_proj.bias.data
            w.fc1_w, w.fc1_b = self._cvt(lay.mlp.fc1.weight.data), lay.mlp.fc1.bias.data
            w.fc2_w, w.fc2_b = self._cvt(lay.mlp.fc2.weight.data), lay.mlp.fc2.bias.data
            w.ln1 = (lay.layer_norm1.weight.data, lay.layer_norm1.bias.data)
            w.ln2 = (lay.layer_norm2.weight.data, lay.layer_norm2.bias.data)
            if self.fold:  # layer_norm1 / layer_norm2 folded into the QKV / fc1 weights (frozen tower: once)
                qkv32 = torch.cat([a.q_proj.weight.data, a.k_proj.weight.data, a.v_proj.weight.data], 0)
                w.qkv_wf, w.qkv_ws, w.qkv_bf = fold_layernorm(qkv32, w.ln1[0], w.ln1[1], w.qkv_b, dt)
                w.fc1_wf, w.fc1_ws, w.fc1_bf = fold_layernorm(lay.mlp.fc1.weight.data, w.ln2[0], w.ln2[1], w.fc1_b, dt)
            self.layers.append(w)

    def alloc(self, B: int) -> SimpleNamespace:
        if B in self._ws:
            return self._ws[B]
        c, D, dt, dev = self.c, self.D, self.dtype, self.dev
        M = B * self.S
        e = lambda *shape, dtype=dt: torch.empty(shape, dtype=dtype, device=dev)  # noqa: E731
        ws = SimpleNamespace(B=B, M=M)
        if not self.fused_patch:  # (icap_patch_embed reads the pixels itself — no patch matrix)
            ws.patches = e(B * self.G * self.G, self.Kp)
            ws.pe = e(B * self.G * self.G, D)
        ws.x, ws.h1, ws.a, ws.o = e(M, D), e(M, D), e(M, D), e(M, D)
        ws.qkv = e(M, 3 * D)
        ws.f = e(M, c.intermediate_size)
        ws.pooled = e(B, D)
        ws.xc = e(B, D)  # the last layer's CLS rows (see run)
        ws.feat = e(B, c.projection_dim)
        ws.emb = e(B, c.projection_dim, dtype=torch.float32)
        ws.feat32 = e(B, c.projection_dim, dtype=torch.float32)
        ws.st_x = ws.st_h = None
        if self.fold:  # (mean, M2) per row and 32-column group of x / h1 (the LayerNorm statistics hand-off)
            ws.st_x = e(M, D // 32, 2, dtype=torch.float32)
            ws.st_h = e(M, D // 32, 2, dtype=torch.float32)
        self._ws = {B: ws}  # keep only the latest batch size
        return ws

    def run(self, ws, pixels: Tensor) -> Tensor:
        """Kernel schedule; returns ws.emb (fp32, L2-normalised) — graph-capturable."""
        c, D, B = self.c, self.D, ws.B
        eps = c.layer_norm_eps
        if self.fused_patch:
            # Conv2d(stride=patch, bias=False) + [CLS || patches] + positions in one launch that gathers the pixel runs
            # into its LDS stages (round 5: no im2col patch matrix, no separate embedding pass)
            ops.patch_embed(pixels, self.w_patch, ws.h1, patch=c.patch_size, prefix=self.cls.view(1, D), pos=self.pos)
        else:  # the im2col matrix (bf16 / fp32 parity mode) and the GEMM over it
            ops.im2col_patches(pixels, ws.patches, c.patch_size)
            ops.gemm(ws.patches, self.w_patch, ws.pe)  # Conv2d(stride=patch, bias=False) as a GEMM
            ops.vit_embed(ws.pe, self.cls, self.pos, ws.h1, B, self.G * self.G, D)
        ops.layernorm_fwd(ws.h1, self.pre[0], self.pre[1], eps, ws.x, None, None)
        scale = self.hd ** -0.5
        nl = len(self.layers)
        fold = ws.st_x is not None
        for i, w in enumerate(self.layers):
            if fold and i > 0:  # x's statistics come from the previous layer's fc2 epilogue
                ops.gemm(ws.x, w.qkv_wf, ws.qkv, bias=w.qkv_bf, ln_fold=(w.qkv_ws, eps), ln_stats_in=ws.st_x)
            else:
                ops.layernorm_fwd(ws.x, w.ln1[0], w.ln1[1], eps, ws.a, None, None)
                ops.gemm(ws.a, w.qkv_w, ws.qkv, bias=w.qkv_b)
            ops.attention_fwd(ws.qkv, ws.o, B=B, S=self.S, H=self.H, hd=self.hd, scale=scale, causal=False)
            if i == nl - 1:
                # last layer: only the CLS rows reach the output (pooler_output = post_layernorm(last_hidden[:, 0]),
                # modeling_clip.py:741-752), so the rows past attention — out_proj, LayerNorm 2, the MLP — run on the
                # B CLS rows alone (strided views: row b at b*S*D); every other token's keys / values were used above
                o_c, x_c = ws.o.view(B, self.S * D)[:, :D], ws.x.view(B, self.S * D)[:, :D]
                h1, a, f = ws.h1[:B], ws.a[:B], ws.f[:B]
                ops.gemm(o_c, w.out_w, h1, bias=w.out_b, resid=x_c)
                ops.layernorm_fwd(h1, w.ln2[0], w.ln2[1], eps, a, None, None)
                ops.gemm(a, w.fc1_w, f, bias=w.fc1_b, act=L.ACT_QUICK_GELU)
                ops.gemm(f, w.fc2_w, ws.xc, bias=w.fc2_b, resid=h1)
                break
            if fold:
                ops.gemm(ws.o, w.out_w, ws.h1, bias=w.out_b, resid=ws.x, ln_stats_out=ws.st_h)
                ops.gemm(ws.h1, w.fc1_wf, ws.f, bias=w.fc1_bf, act=L.ACT_QUICK_GELU, ln_fold=(w.fc1_ws, eps),
                         ln_stats_in=ws.st_h)
                ops.gemm(ws.f, w.fc2_w, ws.x, bias=w.fc2_b, resid=ws.h1, ln_stats_out=ws.st_x)
                continue
            ops.gemm(ws.o, w.out_w, ws.h1, bias=w.out_b, resid=ws.x)
            ops.layernorm_fwd(ws.h1, w.ln2[0], w.ln2[1], eps, ws.a, None, None)
            ops.gemm(ws.a, w.fc1_w, ws.f, bias=w.fc1_b, act=L.ACT_QUICK_GELU)
            ops.gemm(ws.f, w.fc2_w, ws.x, bias=w.fc2_b, resid=ws.h1)
        cls_rows = ws.xc  # CLS token of every image after the last layer
        ops.layernorm_fwd(cls_rows, self.post[0], self.post[1], eps, ws.pooled, None, None, rows=B)
        ops.gemm(ws.pooled, self.w_proj, ws.feat32)
        ops.l2norm_rows(ws.feat32, ws.emb)
        return ws.emb

    @torch.no_grad()
    def features(self, pixels: Tensor, normalize: bool = True) -> Tensor:
        if pixels.dtype != torch.float32 or not pixels.is_contiguous():
            pixels = pixels.float().contiguous()
        ws = self.alloc(pixels.shape[0])
        self.run(ws, pixels)
        return (ws.emb if normalize else ws.feat32).clone()


# --------------------------------------------------------------------------- reference-shaped API (clip.py:10-149)


def load_clip_model(model_name: str = "openai/clip-vit-base-patch32", device: Optional[torch.device] = None,
                    checkpoint: Optional[str] = None) -> Tuple[CLIPVisionTower, "CLIPProcessor"]:
    """clip.py:10-35. Offline: weights come from `checkpoint` (HF safetensors/.bin state dict of CLIPModel, vision
    keys used) when given, else a deterministic random init of the named architecture."""
    device = device or torch.device("cuda")
    cfg = CLIPVisionConfig.vit_l14() if "large-patch14" in model_name else CLIPVisionConfig()
    if checkpoint is not None:
        model = CLIPVisionTower(cfg)
        model.load_state_dict(_load_state(checkpoint), strict=False)
    else:
        model = CLIPVisionTower.random_init(cfg)
    model = model.to(device).eval()
    return model, CLIPProcessor(cfg.image_size)


def _load_state(path: str):
    if path.endswith(".safetensors"):
        from safetensors.torch import load_file

        sd = load_file(path)
    else:
        sd = torch.load(path, map_location="cpu", weights_only=True)
    return {k: v for k, v in sd.items() if k.startswith("vision_model.") or k == "visual_projection.weight"}


def resize_shortest_edge(wh, size: int):
    """(width, height) after CLIPImageProcessor's shortest-edge resize: short side -> size, long side ->
    int(size * long / short) (HF image_transforms.get_resize_output_image_size, default_to_square=False)."""
    w, h = wh
    short, long = (w, h) if w <= h else (h, w)
    new_long = int(size * long / short)
    return (size, new_long) if w <= h else (new_long, size)


class CLIPProcessor:
    """Host-side CLIPImageProcessor equivalent: shortest-edge resize (bicubic) to 224, centre crop, /255,
    mean/std normalise -> fp32 [B,3,224,224]. Images: PIL images or RGB uint8 arrays. DeviceCLIPProcessor runs
    the same arithmetic on the GPU."""

    def __init__(self, size: int = 224):
        self.size = size

    def __call__(self, images, return_tensors: str = "pt"):
        import numpy as np
        from PIL import Image

        if not isinstance(images, (list, tuple)):
            images = [images]
        out = []
        for im in images:
            if isinstance(im, torch.Tensor):  # decoded RGB uint8 from the extraction workers
                im = im.numpy()
            im = Image.fromarray(np.asarray(im, dtype=np.uint8)) if isinstance(im, np.ndarray) else im.convert("RGB")
            im = im.resize(resize_shortest_edge(im.size, self.size), Image.BICUBIC)
            w, h = im.size
            left, top = (w - self.size) // 2, (h - self.size) // 2
            im = im.crop((left, top, left + self.size, top + self.size))
            a = np.asarray(im, dtype=np.float32) / 255.0
            a = (a - np.array(CLIP_MEAN, np.float32)) / np.array(CLIP_STD, np.float32)
            out.append(torch.from_numpy(a.transpose(2, 0, 1).copy()))
        return SimpleNamespace(pixel_values=torch.stack(out))


class DeviceCLIPProcessor(CLIPProcessor):
    """CLIPProcessor with the resize / crop / normalise on the GPU (icap_clip_preprocess; Pillow-exact):
    the host only decodes to RGB uint8. pixel_values come back on `device`."""

    def __init__(self, size: int = 224, device=None):
        super().__init__(size)
        self.device = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)

    def __call__(self, images, return_tensors: str = "pt"):
        import numpy as np

        from . import ops

        if not isinstance(images, (list, tuple)):
            images = [images]
        arrs = [np.asarray(im.convert("RGB")) if hasattr(im, "convert") else np.asarray(im) for im in images]
        return SimpleNamespace(pixel_values=ops.clip_preprocess(arrs, self.device, self.size, self.size))

    def preprocess_packed(self, packed: Tensor, sizes) -> Tensor:
        """pixel_values of a batch the loader already packed (icap.images: one host buffer per batch, pinned)."""
        from . import ops

        return ops.clip_preprocess_packed(packed, sizes, self.device, self.size, self.size)


@torch.no_grad()
def extract_clip_embedding_from_image(image, clip_model: CLIPVisionTower, clip_processor: CLIPProcessor,
                                      device: Optional[torch.device] = None) -> Tensor:
    """clip.py:38-76: one image -> normalised (embedding_dim,) embedding."""
    from PIL import Image

    if isinstance(image, str):
        image = Image.open(image)
    px = clip_processor(images=image).pixel_values.to(device or clip_model.device)
    return clip_model.embed(px).squeeze(0)


@torch.no_grad()
def extract_clip_embeddings(image_dir: str, output_path: str, clip_model: CLIPVisionTower,
                            clip_processor: CLIPProcessor, batch_size: int = 32, num_workers: int = 4,
                            device: Optional[torch.device] = None) -> None:
    """clip.py:79-149: every image of a directory -> {"filenames", "embeddings"} .pt file (same format, same file
    order). JPEG decode runs in `num_workers` DataLoader processes as in the reference (icap.images)."""
    from .images import extract_directory

    n = extract_directory(image_dir, output_path, clip_model.embed, clip_processor, clip_model.config.projection_dim,
                          batch_size, num_workers, device or clip_model.device)
    print(f"Saved {n} CLIP embeddings to {output_path}.")
