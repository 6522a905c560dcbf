"""Parameter containers, deterministic initialisation and flat parameter storage.

Parameters live in nn.Modules whose attribute paths reproduce the reference's
state_dict key names (HF GPT2LMHeadModel, src/models.py mapping networks, HF
CLIPModel vision tower), so checkpoints written by the reference's
save_parameters() (src/models.py:489-519) load unchanged. The modules are
storage only: every forward/backward runs in libicap_hip.so.
"""

from __future__ import annotations

import math
import zlib
from typing import Dict, Iterable, List, Optional, Tuple

import numpy as np
import torch
import torch.nn as nn

from . import ops

Tensor = torch.Tensor


# --------------------------------------------------------------------------- deterministic init


def _splitmix_uniform(seed: int, tag: int, n: int) -> np.ndarray:
    """n uniforms in [-1, 1) from splitmix64(seed, tag, index)."""
    with np.errstate(over="ignore"):
        base = np.uint64((seed * 0x9E3779B97F4A7C15 + tag * 0xD1B54A32D192ED03) & 0xFFFFFFFFFFFFFFFF)
        z = base + (np.arange(n, dtype=np.uint64) + np.uint64(1)) * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return (z >> np.uint64(11)).astype(np.float64) * (2.0 / 9007199254740992.0) - 1.0


def det_tensor(seed: int, name: str, shape, std: float, mean: float = 0.0) -> Tensor:
    """Closed-form deterministic fp32 tensor (mean + std*sqrt(3)*U[-1,1)); identical to the test oracle's."""
    n = int(np.prod(shape)) if len(shape) else 1
    u = _splitmix_uniform(seed, zlib.crc32(name.encode()), n)
    return torch.from_numpy((mean + std * math.sqrt(3.0) * u).astype(np.float32).reshape(shape))


# --------------------------------------------------------------------------- flat parameter storage


def _round_up(x: int, m: int) -> int:
    return (x + m - 1) // m * m


class FlatParams:
    """One contiguous fp32 buffer for a set of parameters (+ grads, AdamW moments, compute-dtype copy).

    Each nn.Parameter's .data becomes a view into `flat`, so state_dict()/load_state_dict() read and write the
    flat buffer in place; `grad_views` are the matching views into `flat_grad`. Tensors start on 64-byte
    boundaries (16 fp32) so every segment is float4-aligned for the kernels."""

    def __init__(self, named: List[Tuple[str, nn.Parameter]], device: torch.device, compute_dtype: torch.dtype):
        self.names = [n for n, _ in named]
        self.params = [p for _, p in named]
        offs, o = [], 0
        for p in self.params:
            offs.append(o)
            o = _round_up(o + p.numel(), 16)
        self.n = max(o, 16)
        self.offsets = offs
        self.flat = torch.zeros(self.n, dtype=torch.float32, device=device)
        self.flat_grad = torch.zeros(self.n, dtype=torch.float32, device=device)
        for p, off in zip(self.params, offs):
            self.flat[off:off + p.numel()].copy_(p.data.reshape(-1))
            p.data = self.flat[off:off + p.numel()].view(p.shape)
        self.grad_views = [self.flat_grad[off:off + p.numel()].view(p.shape) for p, off in zip(self.params, offs)]
        self.compute_dtype = compute_dtype
        self.flat_c: Optional[Tensor] = None
        if compute_dtype != torch.float32:
            self.flat_c = torch.empty(self.n, dtype=compute_dtype, device=device)
        self.exp_avg: Optional[Tensor] = None
        self.exp_avg_sq: Optional[Tensor] = None

    def view_c(self, p: nn.Parameter) -> Tensor:
        """Compute-dtype view of parameter p (the master itself in fp32 mode)."""
        if self.flat_c is None:
            return p.data
        i = self._index(p)
        off = self.offsets[i]
        return self.flat_c[off:off + p.numel()].view(p.shape)

    def grad(self, p: nn.Parameter) -> Tensor:
        return self.grad_views[self._index(p)]

    def _index(self, p: nn.Parameter) -> int:
        for i, q in enumerate(self.params):
            if q is p:
                return i
        raise KeyError("parameter not in this FlatParams")

    def sync_compute_copy(self) -> None:
        """flat_c <- flat (after an external write to the masters, e.g. load_state_dict)."""
        if self.flat_c is not None:
            ops.convert(self.flat.view(1, -1), self.flat_c.view(1, -1))

    def zero_grad(self) -> None:
        self.flat_grad.zero_()

    def attach_grads(self) -> None:
        """Expose the flat grad views as .grad (for drop-in code that reads param.grad)."""
        for p, g in zip(self.params, self.grad_views):
            p.grad = g


def named_trainable(module: nn.Module, prefix: str = "") -> List[Tuple[str, nn.Parameter]]:
    seen, out = set(), []
    for n, p in module.named_parameters(prefix=prefix.rstrip(".")):
        if p.requires_grad and id(p) not in seen:
            seen.add(id(p))
            out.append((n, p))
    return out


def load_into(module: nn.Module, sd: Dict[str, Tensor], strict: bool = True):
    with torch.no_grad():
        return module.load_state_dict(sd, strict=strict)
