"""ViT image tower (src/embeddings/vit.py) on the icap HIP kernels.

Mirrors the reference's extraction API (`load_vit_model`, `extract_vit_embedding_from_image`,
`extract_vit_embeddings`, vit.py:10-137) over HF ViTModel's forward (HF/models/vit/modeling_vit.py): patch Conv2d
WITH bias -> [CLS || patches] + position embeddings (no pre-LN, unlike CLIP) -> pre-LN encoder layers
(layernorm_before, MHA with q/k/v fused into one MFMA GEMM, +res; layernorm_after, dense + exact erf-GELU fused into
the GEMM epilogue, dense, +res; LayerNorm eps 1e-12) -> final layernorm (CLS row only: the pooler reads token 0)
-> pooler tanh(dense(CLS)) -> L2 normalise (vit.py:63-72). Parameters use the HF ViTModel key names of
transformers 4.57 (the reference's pin); checkpoints in the 5.x layout load too (`load_hf_state_dict`).
"""

from __future__ import annotations

from dataclasses import dataclass
from types import SimpleNamespace
from typing import Dict, Optional, Tuple

import torch
import torch.nn as nn

from . import _lib as L
from . import ops
from .weights import det_tensor

Tensor = torch.Tensor

VIT_MEAN = (0.5, 0.5, 0.5)  # ViTImageProcessor defaults (google/vit-base-patch16-224)
VIT_STD = (0.5, 0.5, 0.5)


@dataclass
class ViTConfig:  # HF ViTConfig defaults = google/vit-base-patch16-224
    hidden_size: int = 768
    num_hidden_layers: int = 12
    num_attention_heads: int = 12
    intermediate_size: int = 3072
    patch_size: int = 16
    image_size: int = 224
    num_channels: int = 3
    layer_norm_eps: float = 1e-12

    @property
    def embedding_dim(self) -> int:  # pooler_output width (vit.py:69)
        return self.hidden_size


class _PatchEmb(nn.Module):
    def __init__(self, c: ViTConfig):
        super().__init__()
        self.projection = nn.Conv2d(c.num_channels, c.hidden_size, c.patch_size, c.patch_size, bias=True)


class _Emb(nn.Module):
    def __init__(self, c: ViTConfig):
        super().__init__()
        g = c.image_size // c.patch_size
        self.cls_token = nn.Parameter(torch.zeros(1, 1, c.hidden_size))
        self.position_embeddings = nn.Parameter(torch.zeros(1, g * g + 1, c.hidden_size))
        self.patch_embeddings = _PatchEmb(c)


class _SelfAttn(nn.Module):
    def __init__(self, d):
        super().__init__()
        self.query, self.key, self.value = nn.Linear(d, d), nn.Linear(d, d), nn.Linear(d, d)


class _Dense(nn.Module):
    def __init__(self, i, o):
        super().__init__()
        self.dense = nn.Linear(i, o)


class _Attention(nn.Module):
    def __init__(self, d):
        super().__init__()
        self.attention = _SelfAttn(d)
        self.output = _Dense(d, d)


class _Layer(nn.Module):
    def __init__(self, c: ViTConfig):
        super().__init__()
        d = c.hidden_size
        self.attention = _Attention(d)
        self.intermediate = _Dense(d, c.intermediate_size)
        self.output = _Dense(c.intermediate_size, d)
        self.layernorm_before = nn.LayerNorm(d, eps=c.layer_norm_eps)
        self.layernorm_after = nn.LayerNorm(d, eps=c.layer_norm_eps)


class _Encoder(nn.Module):
    def __init__(self, c: ViTConfig):
        super().__init__()
        self.layer = nn.ModuleList([_Layer(c) for _ in range(c.num_hidden_layers)])


class ViTImageTower(nn.Module):
    """HF ViTModel with its pooler (`ViTModel(pixel_values).pooler_output`, vit.py:66-69). Frozen."""

    def __init__(self, config: Optional[ViTConfig] = None):
        super().__init__()
        self.config = config or ViTConfig()
        c = self.config
        self.embeddings = _Emb(c)
        self.encoder = _Encoder(c)
        self.layernorm = nn.LayerNorm(c.hidden_size, eps=c.layer_norm_eps)
        self.pooler = _Dense(c.hidden_size, c.hidden_size)
        for p in self.parameters():
            p.requires_grad = False  # vit.py:31 eval mode, never trained
        self._core = None
        self._core_key = None

    @classmethod
    def random_init(cls, config: Optional[ViTConfig] = None, seed: int = 0) -> "ViTImageTower":
        """Deterministic random weights of the architecture (no pretrained checkpoint offline)."""
        m = cls(config)
        c = m.config
        d, g = c.hidden_size, c.image_size // c.patch_size
        sd = {
            "embeddings.cls_token": det_tensor(seed, "v.cls", (1, 1, d), 0.5),
            "embeddings.position_embeddings": det_tensor(seed, "v.pos", (1, g * g + 1, d), 0.02),
            "embeddings.patch_embeddings.projection.weight": det_tensor(
                seed, "v.patch.w", (d, c.num_channels, c.patch_size, c.patch_size), 0.02),
            "embeddings.patch_embeddings.projection.bias": det_tensor(seed, "v.patch.b", (d,), 0.02),
            "layernorm.weight": det_tensor(seed, "v.ln.w", (d,), 0.05, 1.0),
            "layernorm.bias": det_tensor(seed, "v.ln.b", (d,), 0.02),
            "pooler.dense.weight": det_tensor(seed, "v.pool.w", (d, d), 0.02),
            "pooler.dense.bias": det_tensor(seed, "v.pool.b", (d,), 0.02),
        }
        for i in range(c.num_hidden_layers):
            p = f"encoder.layer.{i}."
            for nm in ("query", "key", "value"):
                sd[p + f"attention.attention.{nm}.weight"] = det_tensor(seed, p + nm + ".w", (d, d), 0.02)
                sd[p + f"attention.attention.{nm}.bias"] = det_tensor(seed, p + nm + ".b", (d,), 0.02)
            sd[p + "attention.output.dense.weight"] = det_tensor(seed, p + "ao.w", (d, d), 0.02)
            sd[p + "attention.output.dense.bias"] = det_tensor(seed, p + "ao.b", (d,), 0.02)
            sd[p + "intermediate.dense.weight"] = det_tensor(seed, p + "fc1.w", (c.intermediate_size, d), 0.02)
            sd[p + "intermediate.dense.bias"] = det_tensor(seed, p + "fc1.b", (c.intermediate_size,), 0.02)
            sd[p + "output.dense.weight"] = det_tensor(seed, p + "fc2.w", (d, c.intermediate_size), 0.02)
            sd[p + "output.dense.bias"] = det_tensor(seed, p + "fc2.b", (d,), 0.02)
            sd[p + "layernorm_before.weight"] = det_tensor(seed, p + "lnb.w", (d,), 0.05, 1.0)
            sd[p + "layernorm_before.bias"] = det_tensor(seed, p + "lnb.b", (d,), 0.02)
            sd[p + "layernorm_after.weight"] = det_tensor(seed, p + "lna.w", (d,), 0.05, 1.0)
            sd[p + "layernorm_after.bias"] = det_tensor(seed, p + "lna.b", (d,), 0.02)
        m.load_state_dict(sd, strict=True)
        return m

    def load_hf_state_dict(self, sd: Dict[str, Tensor]):
        """An HF ViTModel / ViTForImageClassification state dict in either key layout (4.57: encoder.layer.N.attention
        .attention.query ...; 5.x: layers.N.attention.q_proj ...); a 'vit.' prefix and classifier keys are dropped."""
        out = {}
        for k, v in sd.items():
            if k.startswith("vit."):
                k = k[4:]
            if k.startswith("classifier."):
                continue
            if k.startswith("layers."):
                i, rest = k[len("layers."):].split(".", 1)
                rest = (rest.replace("attention.q_proj", "attention.attention.query")
                        .replace("attention.k_proj", "attention.attention.key")
                        .replace("attention.v_proj", "attention.attention.value")
                        .replace("attention.o_proj", "attention.output.dense")
                        .replace("mlp.fc1", "intermediate.dense").replace("mlp.fc2", "output.dense"))
                k = f"encoder.layer.{i}.{rest}"
            out[k] = v
        self._core = None
        return self.load_state_dict(out, strict=True)

    @property
    def device(self):
        return self.pooler.dense.weight.device

    def core(self, dtype: torch.dtype = torch.bfloat16) -> "ViTCore":
        key = (dtype, self.device)
        if self._core is None or self._core_key != key:
            self._core = ViTCore(self, dtype)
            self._core_key = key
        return self._core

    @torch.no_grad()
    def pooler_output(self, pixel_values: Tensor, compute_dtype: torch.dtype = torch.bfloat16) -> Tensor:
        """`ViTModel(pixel_values).pooler_output` [B, hidden] fp32 (un-normalised)."""
        return self.core(compute_dtype).features(pixel_values, normalize=False)

    @torch.no_grad()
    def embed(self, pixel_values: Tensor, compute_dtype: torch.dtype = torch.bfloat16) -> Tensor:
        """L2-normalised pooler output (vit.py:63-72)."""
        return self.core(compute_dtype).features(pixel_values, normalize=True)


class ViTCore:
    """Kernel schedule of one ViTImageTower in one compute dtype (weights in GEMM layout, per-batch workspaces)."""

    def __init__(self, m: ViTImageTower, dtype: torch.dtype):
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
        m = self.m
        e = m.embeddings
        wp = e.patch_embeddings.projection.weight.data.reshape(self.D, -1)  # [D, C*p*p] in (c, ky, kx) order
        self.Kp = (wp.shape[1] + 7) // 8 * 8  # icap_im2col_patches row width (p = 16: 768, no padding)
        if self.Kp != wp.shape[1]:
            wp = torch.nn.functional.pad(wp, (0, self.Kp - wp.shape[1]))
        self.w_patch = self._cvt(wp)
        self.b_patch = e.patch_embeddings.projection.bias.data.contiguous()
        self.cls = e.cls_token.data.reshape(-1).contiguous()
        self.pos = e.position_embeddings.data.reshape(self.S, self.D).contiguous()
        self.lnf = (m.layernorm.weight.data, m.layernorm.bias.data)
        self.w_pool, self.b_pool = self._cvt(m.pooler.dense.weight.data), m.pooler.dense.bias.data
        self.layers = []
        for lay in m.encoder.layer:
            a = lay.attention.attention
            w = SimpleNamespace()
            w.qkv_w = self._cvt(torch.cat([a.query.weight.data, a.key.weight.data, a.value.weight.data], 0))
            w.qkv_b = torch.cat([a.query.bias.data, a.key.bias.data, a.value.bias.data], 0).contiguous()
            w.out_w, w.out_b = self._cvt(lay.attention.output.dense.weight.data), lay.attention.output.dense.bias.data
            w.fc1_w, w.fc1_b = self._cvt(lay.intermediate.dense.weight.data), lay.intermediate.dense.bias.data
            w.fc2_w, w.fc2_b = self._cvt(lay.output.dense.weight.data), lay.output.dense.bias.data
            w.ln1 = (lay.layernorm_before.weight.data, lay.layernorm_before.bias.data)
            w.ln2 = (lay.layernorm_after.weight.data, lay.layernorm_after.bias.data)
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
        """Kernel schedule; fills ws.pool (pooler_output) and ws.emb (L2-normalised) — graph-capturable."""
        c, D, B = self.c, self.D, ws.B
        eps = c.layer_norm_eps
        if self.dtype == torch.bfloat16:  # patch Conv2d + [CLS || patches] + positions, pixels read by the GEMM
            ops.patch_embed(pixels, self.w_patch, ws.x, patch=c.patch_size, prefix=self.cls.view(1, D), pos=self.pos,
                            bias=self.b_patch)
        else:
            ops.im2col_patches(pixels, ws.patches, c.patch_size)
            ops.gemm(ws.patches, self.w_patch, ws.pe, bias=self.b_patch)  # Conv2d(stride=patch, bias) as a GEMM
            ops.vit_embed(ws.pe, self.cls, self.pos, ws.x, B, self.G * self.G, D)  # [CLS || patches] + positions
        scale = self.hd ** -0.5
        nl = len(self.layers)
        for i, w in enumerate(self.layers):
            ops.layernorm_fwd(ws.x, w.ln1[0], w.ln1[1], eps, ws.a, None, None)
            ops.gemm(ws.a, w.qkv_w, ws.qkv, bias=w.qkv_b)
            ops.attention_fwd(ws.qkv, ws.o, B=B, S=self.S, H=self.H, hd=self.hd, scale=scale, causal=False)
            if i == nl - 1:
                # last layer: the pooler reads token 0 only (modeling_vit.py:289-301), so past attention the layer
                # runs on the B CLS rows (strided views, row b at b*S*D); the other tokens' keys / values were used
                o_c, x_c = ws.o.view(B, self.S * D)[:, :D], ws.x.view(B, self.S * D)[:, :D]
                h1, a, f = ws.h1[:B], ws.a[:B], ws.f[:B]
                ops.gemm(o_c, w.out_w, h1, bias=w.out_b, resid=x_c)
                ops.layernorm_fwd(h1, w.ln2[0], w.ln2[1], eps, a, None, None)
                ops.gemm(a, w.fc1_w, f, bias=w.fc1_b, act=L.ACT_GELU_ERF)
                ops.gemm(f, w.fc2_w, ws.xc, bias=w.fc2_b, resid=h1)
                break
            ops.gemm(ws.o, w.out_w, ws.h1, bias=w.out_b, resid=ws.x)
            ops.layernorm_fwd(ws.h1, w.ln2[0], w.ln2[1], eps, ws.a, None, None)
            ops.gemm(ws.a, w.fc1_w, ws.f, bias=w.fc1_b, act=L.ACT_GELU_ERF)
            ops.gemm(ws.f, w.fc2_w, ws.x, bias=w.fc2_b, resid=ws.h1)
        cls_rows = ws.xc  # CLS token of every image after the last layer
        ops.layernorm_fwd(cls_rows, self.lnf[0], self.lnf[1], eps, ws.cls, None, None, rows=B)
        ops.gemm(ws.cls, self.w_pool, ws.pool, bias=self.b_pool, act=L.ACT_TANH)
        ops.l2norm_rows(ws.pool, ws.emb)
        return ws.emb

    @torch.no_grad()
    def features(self, pixels: Tensor, normalize: bool = True) -> Tensor:
        if pixels.dtype != torch.float32 or not pixels.is_contiguous():
            pixels = pixels.float().contiguous()
        ws = self.alloc(pixels.shape[0])
        self.run(ws, pixels)
        return (ws.emb if normalize else ws.pool).clone()


# --------------------------------------------------------------------------- reference-shaped API (vit.py:10-137)


class ViTImageProcessor:
    """Host ViTImageProcessor equivalent (google/vit-base-patch16-224 defaults): resize to 224 x 224 (PIL bilinear),
    x 1/255, (x - 0.5) / 0.5 -> fp32 [B, 3, 224, 224]. Images: PIL images or RGB uint8 arrays."""

    def __init__(self, size: int = 224, mean=VIT_MEAN, std=VIT_STD):
        self.size, self.mean, self.std = size, mean, std

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
            im = im.resize((self.size, self.size), Image.BILINEAR)
            a = np.asarray(im, dtype=np.float32) * np.float32(1 / 255)
            a = (a - np.array(self.mean, np.float32)) / np.array(self.std, np.float32)
            out.append(torch.from_numpy(a.transpose(2, 0, 1).copy()))
        return SimpleNamespace(pixel_values=torch.stack(out))


def load_vit_model(model_name: str = "google/vit-base-patch16-224", device: Optional[torch.device] = None,
                   checkpoint: Optional[str] = None) -> Tuple[ViTImageTower, ViTImageProcessor]:
    """vit.py:10-35. Offline: weights come from `checkpoint` (an HF ViT safetensors / .bin state dict, either key
    layout) when given, else a deterministic random init of the architecture."""
    device = device or torch.device("cuda")
    print(f"Loading ViT model '{model_name}' on device: {device}...")
    model = ViTImageTower(ViTConfig())
    if checkpoint is not None:
        if checkpoint.endswith(".safetensors"):
            from safetensors.torch import load_file

            sd = load_file(checkpoint)
        else:
            sd = torch.load(checkpoint, map_location="cpu", weights_only=True)
        model.load_hf_state_dict(sd)
    else:
        model = ViTImageTower.random_init(ViTConfig())
    return model.to(device).eval(), ViTImageProcessor(model.config.image_size)


@torch.no_grad()
def extract_vit_embedding_from_image(image, vit_model: ViTImageTower, vit_processor: ViTImageProcessor,
                                     device: Optional[torch.device] = None) -> Tensor:
    """vit.py:38-77: one image (path or PIL image) -> L2-normalised (embedding_dim,) pooler embedding."""
    from PIL import Image

    if isinstance(image, str):
        image = Image.open(image)
    px = vit_processor(images=image).pixel_values.to(device or vit_model.device)
    return vit_model.embed(px).squeeze(0)


@torch.no_grad()
def extract_vit_embeddings(image_dir: str, output_path: str, vit_model: ViTImageTower,
                           vit_processor: ViTImageProcessor, batch_size: int = 32, num_workers: int = 4,
                           device: Optional[torch.device] = None) -> None:
    """vit.py:80-137: every image of a directory -> {"filenames", "embeddings"} .pt file (the reference's format and
    file order; decode in `num_workers` DataLoader processes)."""
    from .images import extract_directory

    n = extract_directory(image_dir, output_path, vit_model.embed, vit_processor, vit_model.config.embedding_dim,
                          batch_size, num_workers, device or vit_model.device)
    print(f"Saved {n} ViT embeddings to {output_path}.")
