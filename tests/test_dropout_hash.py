"""The counter-based dropout mask (csrc/common.h hash32 / drop_scale, include/icap.h "Dropout").

A numpy restatement of the device hash checks its statistics on the CPU, and the GPU test checks the device
mask bit-for-bit against it (icap_dropout_apply over a tensor of ones, with and without the device seed
counter). The reference draws its masks from torch's Philox stream, so masks are not comparable with it; what
the path must keep is the Bernoulli(1-p) keep rate, independence across elements / seeds / steps, and forward
and backward regenerating the same mask from (seed, index).
"""

import numpy as np
import pytest
import torch

M32 = np.uint64(0xFFFFFFFF)
GOLDEN64 = 0x9E3779B97F4A7C15


def hash32(seed: int, idx: np.ndarray) -> np.ndarray:
    """numpy restatement of common.h hash32 (uint32 results)."""
    idx = idx.astype(np.uint64)
    s0, s1 = np.uint64(seed & 0xFFFFFFFF), np.uint64((seed >> 32) & 0xFFFFFFFF)
    lo, hi = idx & M32, idx >> np.uint64(32)
    x = ((((lo ^ s0) * np.uint64(0x9E3779B9)) + hi) & M32) ^ s1
    x ^= x >> np.uint64(16)
    x = (x * np.uint64(0x7FEB352D)) & M32
    x ^= x >> np.uint64(15)
    x = (x * np.uint64(0x846CA68B)) & M32
    x ^= x >> np.uint64(16)
    return x.astype(np.uint32)


def eff_seed(seed: int, counter) -> int:
    return seed if counter is None else (seed + counter * GOLDEN64) & (2**64 - 1)


def threshold(p: float) -> int:
    return min(int(p * 4294967296.0), 4294967295)


def keep_mask(seed: int, offset: int, n: int, p: float, counter=None) -> np.ndarray:
    return hash32(eff_seed(seed, counter), offset + np.arange(n, dtype=np.uint64)) >= np.uint32(threshold(p))


def test_keep_rate_and_bijection():
    n = 1 << 20
    h = hash32(1234, np.arange(n, dtype=np.uint64))
    assert len(np.unique(h)) == n  # a bijection on 32-bit indices: no two elements share a draw
    for p in (0.1, 0.5):
        kept = (h >= np.uint32(threshold(p))).mean()
        assert abs(kept - (1 - p)) < 4 * np.sqrt(p * (1 - p) / n)


def test_independence():
    n = 1 << 20
    k = keep_mask(7, 0, n, 0.5).astype(np.float64)
    for lag in (1, 4, 768, 65 * 65):
        c = np.corrcoef(k[:-lag], k[lag:])[0, 1]
        assert abs(c) < 5e-3, (lag, c)
    # successive steps (device counter) and different seeds give unrelated masks
    k1 = keep_mask(7, 0, n, 0.5, counter=1).astype(np.float64)
    k2 = keep_mask(8, 0, n, 0.5).astype(np.float64)
    assert abs(np.corrcoef(k, k1)[0, 1]) < 5e-3
    assert abs(np.corrcoef(k, k2)[0, 1]) < 5e-3
    # bits are uniform
    h = hash32(99, np.arange(n, dtype=np.uint64))
    bits = ((h[:, None] >> np.arange(32, dtype=np.uint32)) & 1).mean(axis=0)
    assert np.abs(bits - 0.5).max() < 4 * 0.5 / np.sqrt(n)


@pytest.mark.gpu
@pytest.mark.parametrize("counter", [None, 3])
def test_device_mask_matches_restatement(dev, counter):
    from icap import ops

    M, N, p, seed, offset = 300, 768, 0.1, 0xDEADBEEF12345678, 5 + (1 << 32)
    x = torch.ones((M, N), device=dev)
    y = torch.empty_like(x)
    ctr = None if counter is None else torch.full((1,), counter, dtype=torch.int64, device=dev)
    ops.dropout_apply(x, y, ops.Dropout(p, seed, offset, ctr))
    got = (y != 0).cpu().numpy().reshape(-1)
    want = keep_mask(seed, offset, M * N, p, counter)
    assert np.array_equal(got, want)
    assert torch.allclose(y[y != 0], torch.full_like(y[y != 0], 1 / (1 - p)))
