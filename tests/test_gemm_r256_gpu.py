"""The 256 x 128 ring tile kernel (variant 22: gemm_kernel<.., 3, 1, 4, 2, 4, 4, ..>, csrc/gemm_tile.h ring path,
csrc/gemm_tile_r256.hip) against the 128-row tile kernels and fp64.

Both run the same MFMA 16x16x32 chain per output element (64-deep k-steps in order, their two 32-deep halves in
order; the tile path with tile_only=True keeps the natural k order) and the shared epilogue, so the outputs are
bitwise equal for every epilogue form, with a device row count (m_dev: the packed step's rows) and for the
LayerNorm statistics hand-off (producer statistics, consumer fold). Shapes: the packed step's products, partial
row / column tiles, K tails, one and two K-tiles (pipeline prologue / drain), fp32 output."""

import math

import pytest
import torch

from icap import _lib as L
from icap import ops
from gemm_helpers import _assert_same, _run, rnd

pytestmark = pytest.mark.gpu

SHAPES = [
    (3584, 2304, 768),  # GPT-2 QKV at the packed rows
    (3584, 3072, 768),  # c_fc
    (3584, 768, 3072),  # mlp c_proj
    (1000, 520, 200),   # partial tiles both ways, K tail (200 = 3 x 64 + 8)
    (512, 256, 64),     # one K-tile
    (768, 384, 128),    # two K-tiles
]


def _name(bn, tc, act):
    return f"icap::gemm_kernel<unsigned short, {tc}, 3, 1, 4, 2, 4, 4, false, {act}>"


@pytest.mark.parametrize("bn", [128])
@pytest.mark.parametrize("M,N,K", SHAPES)
def test_r256_plain_matches_tile_and_fp64(dev, bn, M, N, K):
    A = rnd((M, K), dev, seed=1)
    B = rnd((N, K), dev, seed=2)
    C = torch.full((M, N), 7.0, device=dev, dtype=torch.bfloat16)
    Ct = torch.empty_like(C)
    names = _run(lambda: ops.gemm(A, B, C, split_k=1, r256=True))
    assert names == [_name(bn, "unsigned short", 0)], names
    ops.gemm(A, B, Ct, split_k=1, tile_only=True)
    torch.cuda.synchronize()
    _assert_same("C", C, Ct)
    ref = A.double() @ B.double().t()
    err = ((C.double() - ref).abs() / (A.double().abs() @ B.double().abs().t())).max().item()
    assert err < 4e-3, err


@pytest.mark.parametrize("bn", [128])
@pytest.mark.parametrize("M,N,K", [(3584, 3072, 768), (1000, 520, 200)])
def test_r256_epilogues_match_tile(dev, bn, M, N, K):
    A = rnd((M, K), dev, scale=0.1, seed=6)
    B = rnd((N, K), dev, scale=0.1, seed=7)
    bias = rnd((N,), dev, torch.float32, 0.5, seed=8)
    resid = rnd((M, N), dev, seed=9)
    drop = ops.Dropout(0.1, seed=1234, offset=77)
    act = L.ACT_GELU_NEW
    out = {}
    for tile in (False, True):
        kw = dict(tile_only=True) if tile else dict(r256=True)
        C = torch.empty((M, N), device=dev, dtype=torch.bfloat16)
        aux, C2, dZ, C3 = torch.empty_like(C), torch.empty_like(C), torch.empty_like(C), torch.empty_like(C)
        names = _run(lambda: (ops.gemm(A, B, C, bias=bias, act=act, aux=aux, split_k=1, **kw),
                              ops.gemm(A, B, C2, bias=bias, resid=resid, drop=drop, alpha=0.75, split_k=1, **kw),
                              ops.gemm(A, B, dZ, dact=act, dact_src=aux, drop=drop, alpha=0.5, split_k=1, **kw),
                              ops.gemm(A, B, C3, bias=bias, act=L.ACT_RELU, split_k=1, **kw)))
        assert all(("4, 2, 4, 4" in n) != tile for n in names), names
        out[tile] = (C, aux, C2, dZ, C3)
    torch.cuda.synchronize()
    for name, a, b in zip(("C", "aux", "C2", "dZ", "relu"), out[False], out[True]):
        _assert_same(name, a, b)
    z = A.double() @ B.double().t() + bias.double()
    y = 0.5 * z * (1 + torch.tanh(math.sqrt(2 / math.pi) * (z + 0.044715 * z ** 3)))
    assert (out[False][0].double() - y).abs().max().item() < 2e-2 * max(1.0, y.abs().max().item())


@pytest.mark.parametrize("bn", [128])
def test_r256_device_row_count(dev, bn):
    """m_dev: rows past the device count are neither computed nor stored; the rest equal the tile path's."""
    M, live, N, K = 8320, 3584, 2304, 768
    A = rnd((M, K), dev, seed=21)
    B = rnd((N, K), dev, seed=22)
    md = torch.tensor([live], dtype=torch.int32, device=dev)
    C = torch.full((M, N), 3.0, device=dev, dtype=torch.bfloat16)
    Ct = torch.full_like(C, 3.0)
    names = _run(lambda: ops.gemm(A, B, C, m_dev=md, m_hint=live, split_k=1, r256=True))
    assert names == [_name(bn, "unsigned short", 0)], names
    ops.gemm(A, B, Ct, m_dev=md, m_hint=live, split_k=1, tile_only=True)
    torch.cuda.synchronize()
    _assert_same("C", C[:live], Ct[:live])
    assert bool((C[live:] == 3.0).all())


@pytest.mark.parametrize("bn", [128])
def test_r256_layernorm_handoff_matches_tile(dev, bn):
    """Producer: C and its (mean, M2) per row and 32-column group equal the tile kernel's. Consumer: the folded
    LayerNorm epilogue (+ gelu_new + aux), and the row statistics it writes, equal the tile kernel's."""
    from icap.gpt2 import fold_layernorm

    M, live, D, F = 8320, 3584, 768, 3072
    md = torch.tensor([live], dtype=torch.int32, device=dev)
    A = rnd((M, F), dev, scale=0.5, seed=31)
    W = rnd((D, F), dev, scale=0.05, seed=32)
    resid = rnd((M, D), dev, scale=2.0, seed=33)
    bias = rnd((D,), dev, torch.float32, 0.1, seed=34)
    Wc = rnd((F, D), dev, torch.float32, 0.05, seed=35)
    gamma = 1 + rnd((D,), dev, torch.float32, 0.2, seed=36)
    beta = rnd((D,), dev, torch.float32, 0.1, seed=37)
    bc = rnd((F,), dev, torch.float32, 0.1, seed=38)
    wf, wsum, bf = fold_layernorm(Wc, gamma, beta, bc, torch.bfloat16)
    out = {}
    for tile in (False, True):
        kw = dict(tile_only=True) if tile else dict(r256=True)
        C = torch.zeros((M, D), device=dev, dtype=torch.bfloat16)
        st = torch.full((M, D // 32, 2), float("nan"), device=dev)
        F2 = torch.zeros((M, F), device=dev, dtype=torch.bfloat16)
        Z = torch.zeros_like(F2)
        mo, ro = torch.zeros(M, device=dev), torch.zeros(M, device=dev)
        names = _run(lambda: (ops.gemm(A, W, C, bias=bias, resid=resid, m_dev=md, m_hint=live, split_k=1,
                                       ln_stats_out=st, **kw),
                              ops.gemm(C, wf, F2, bias=bf, act=L.ACT_GELU_NEW, aux=Z, m_dev=md, m_hint=live, split_k=1,
                                       ln_fold=(wsum, 1e-5), ln_stats_in=st, ln_rows_out=(mo, ro), **kw)))
        assert all(("4, 2, 4, 4" in n) != tile for n in names), names
        out[tile] = (C, st, F2, Z, mo, ro)
    torch.cuda.synchronize()
    for name, a, b in zip(("C", "stats", "F", "Z", "mean", "rstd"), out[False], out[True]):
        a, b = a[:live], b[:live]
        if a.dim() == 3:
            a, b = a.reshape(live, -1), b.reshape(live, -1)
        if a.dim() == 1:
            a, b = a[:, None], b[:, None]
        _assert_same(name, a, b)


def test_r256_f32_output_matches_tile(dev):
    M, N, K = 2048, 1024, 320
    A = rnd((M, K), dev, seed=11)
    B = rnd((N, K), dev, seed=12)
    for bn in (128,):
        C = torch.empty((M, N), device=dev, dtype=torch.float32)
        Ct = torch.empty_like(C)
        names = _run(lambda: ops.gemm(A, B, C, split_k=1, r256=True))
        assert names == [_name(bn, "float", 0)], names
        ops.gemm(A, B, Ct, split_k=1, tile_only=True)
        torch.cuda.synchronize()
        _assert_same("C", C, Ct)
