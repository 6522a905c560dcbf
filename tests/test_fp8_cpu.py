"""MX fp8 contract on the CPU (BASELINE configs[4]'s fp8 path; no reference counterpart: the reference computes in
fp32). oracle.mx_quantize restates OCP MX (32-element blocks, E8M0 power-of-two scale, e4m3fn elements); here it is
pinned against torch's own float8_e4m3fn conversion (an independent RNE implementation) and its defining
properties; tests/test_fp8_gpu.py then checks the device quantiser against it bit for bit."""

import numpy as np
import torch

from oracle import icap_oracle as O


def test_e4m3_round_matches_torch_float8():
    rng = np.random.default_rng(0)
    x = np.concatenate([rng.standard_normal(20000) * s for s in (1e-3, 0.05, 1.0, 30.0, 200.0)]).astype(np.float32)
    x = np.clip(x, -448, 448)
    # exact ties of the e4m3 grid at several binades (round half to even)
    ties = np.array([(2 * k + 1) / 16 * 2.0 ** e for k in range(8) for e in range(-8, 8)], dtype=np.float32)
    x = np.concatenate([x, ties, -ties, [0.0, 2.0 ** -9, 3 * 2.0 ** -10, 448.0]]).astype(np.float32)
    ref = torch.from_numpy(x).to(torch.float8_e4m3fn).to(torch.float64).numpy()
    got = O.e4m3_round(x)
    assert np.array_equal(got, ref)
    codes = O.e4m3_encode(got)
    assert np.array_equal(O.e4m3_decode(codes), got)
    tcodes = torch.from_numpy(x).to(torch.float8_e4m3fn).view(torch.uint8).numpy()
    nz = got != 0  # (a negative value rounding to zero: -0 in both, but compare codes where the value is nonzero)
    assert np.array_equal(codes[nz], tcodes[nz])


def test_mx_quantize_properties():
    rng = np.random.default_rng(1)
    R, K = 70, 256
    x = (rng.standard_normal((R, K)) * np.exp(rng.uniform(-8, 8, size=(R, K // 32, 1))).repeat(32, -1).reshape(R, K))
    x = x.astype(np.float32)
    x[3, 32:64] = 0.0  # an all-zero block
    q, s = O.mx_quantize(x)
    d = O.mx_dequantize(q, s)
    blk = np.abs(x.astype(np.float64)).reshape(R, K // 32, 32)
    X = s.astype(np.int64) - 127
    assert s[3, 1] == 127 and np.all(d[3, 32:64] == 0)
    # the scale is the smallest power of two that keeps the block's max within 448 (no element saturates)
    amax = blk.max(-1)
    nz = amax > 0
    assert np.all(amax[nz] <= 448.0 * 2.0 ** X[nz]) and np.all(amax[nz] > 448.0 * 2.0 ** (X[nz] - 1))
    # elements: round-to-nearest on the scaled e4m3 grid (half a step of the element's binade)
    scaled = x.reshape(R, K // 32, 32) * 2.0 ** (-X[..., None])
    step = 2.0 ** (np.floor(np.log2(np.maximum(np.abs(scaled), 2.0 ** -6))) - 3)
    err = np.abs(d.reshape(R, K // 32, 32) * 2.0 ** (-X[..., None]) - scaled)
    assert np.all(err <= step / 2 + 1e-12)


def test_mx_scale_layout():
    R, K = 130, 384
    s = np.arange(R * (K // 32), dtype=np.int64).reshape(R, K // 32) % 250
    lay = O.mx_scale_layout(s.astype(np.uint8))
    rg = (R + 63) // 64
    assert lay.size == (K // 32) * rg * 64
    for r in (0, 1, 15, 16, 63, 64, 100, 129):
        for kb in range(K // 32):
            st = kb // 4
            assert lay[((st * rg + r // 64) * 16 + r % 16) * 16 + ((r // 16) % 4) * 4 + kb % 4] == s[r, kb]
    assert np.all(lay[((0 * rg + 2) * 16 + 5) * 16: ((0 * rg + 2) * 16 + 6) * 16][8:] == 127)  # padded rows
