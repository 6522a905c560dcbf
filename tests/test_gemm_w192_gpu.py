"""The 192 x 64 tile kernel (variant 24: gemm_kernel<.., 2, 2, 4, 1, 3, 4, ..>, 4 waves stacked in M, csrc/
gemm_tile_w192.hip; past 16 k-stages the 4-stage LDS-DMA ring, variant 25: gemm_kernel<.., 4, 1, 4, 1, 3, 4, ..>)
against the 128-row tile kernels and fp64.

Both run the same MFMA 16x16x32 chain per output element (64-deep k-steps in order, their two 32-deep halves in
order; the tile path with tile_only=True keeps the natural k order) and the shared epilogue, so the outputs are
bitwise equal for every epilogue form the variant has (plain, bias / residual / dropout / alpha, dgelu, relu through
the dispatching form), with a device row count (the packed step's rows) and for the LayerNorm statistics producer.
Shapes: the packed step's N = 768 products, partial row / column tiles, K tails, one and two K-tiles, fp32 output."""

import pytest
import torch

from icap import _lib as L
from icap import ops
from gemm_helpers import _assert_same, _run, rnd

pytestmark = pytest.mark.gpu

SHAPES = [
    (3584, 768, 768),   # GPT-2 attn c_proj at the packed rows
    (3584, 768, 2304),  # c_attn dX
    (3584, 768, 3072),  # mlp c_proj
    (3200, 768, 768),   # mapper projections
    (1000, 520, 200),   # partial tiles both ways, K tail (200 = 3 x 64 + 8)
    (384, 256, 64),     # one K-tile
    (600, 128, 128),    # two K-tiles, partial last row tile
]


def _name(tc, act, K=0):
    """variant 24 (double-buffered, 2 blocks / CU) up to 16 k-stages of 64, the 4-stage ring (variant 25) past that"""
    form = "4, 1" if (K + 63) // 64 > 16 else "2, 2"
    return f"icap::gemm_kernel<unsigned short, {tc}, {form}, 4, 1, 3, 4, false, {act}>"


@pytest.mark.parametrize("M,N,K", SHAPES)
def test_w192_plain_matches_tile_and_fp64(dev, M, N, K):
    A = rnd((M, K), dev, seed=1)
    B = rnd((N, K), dev, seed=2)
    C = torch.full((M, N), 7.0, device=dev, dtype=torch.bfloat16)
    Ct = torch.empty_like(C)
    names = _run(lambda: ops.gemm(A, B, C, split_k=1, w192=True))
    assert names == [_name("unsigned short", 0, K)], names
    ops.gemm(A, B, Ct, split_k=1, tile_only=True)
    torch.cuda.synchronize()
    _assert_same("C", C, Ct)
    ref = A.double() @ B.double().t()
    err = ((C.double() - ref).abs() / (A.double().abs() @ B.double().abs().t())).max().item()
    assert err < 4e-3, err


@pytest.mark.parametrize("M,N,K", [(3584, 768, 768), (1000, 520, 200)])
def test_w192_epilogues_match_tile(dev, M, N, K):
    A = rnd((M, K), dev, scale=0.1, seed=6)
    B = rnd((N, K), dev, scale=0.1, seed=7)
    bias = rnd((N,), dev, torch.float32, 0.5, seed=8)
    resid = rnd((M, N), dev, seed=9)
    dsrc = rnd((M, N), dev, seed=10)
    drop = ops.Dropout(0.1, seed=1234, offset=77)
    out = {}
    for tile in (False, True):
        kw = dict(tile_only=True) if tile else dict(w192=True)
        C = torch.empty((M, N), device=dev, dtype=torch.bfloat16)
        C2, dZ = torch.empty_like(C), torch.empty_like(C)
        names = _run(lambda: (ops.gemm(A, B, C, bias=bias, resid=resid, drop=drop, alpha=0.75, split_k=1, **kw),
                              ops.gemm(A, B, dZ, dact=L.ACT_GELU_NEW, dact_src=dsrc, drop=drop, alpha=0.5, split_k=1,
                                       **kw),
                              ops.gemm(A, B, C2, bias=bias, act=L.ACT_RELU, split_k=1, **kw)))
        assert all(("4, 1, 3, 4" in n) != tile for n in names), names
        out[tile] = (C, dZ, C2)
    torch.cuda.synchronize()
    for name, a, b in zip(("C", "dZ", "relu"), out[False], out[True]):
        _assert_same(name, a, b)


def test_w192_device_row_count(dev):
    """m_dev: rows past the device count are neither computed nor stored; the rest equal the tile path's."""
    M, live, N, K = 8320, 3584, 768, 768
    A = rnd((M, K), dev, seed=21)
    B = rnd((N, K), dev, seed=22)
    md = torch.tensor([live], dtype=torch.int32, device=dev)
    C = torch.full((M, N), 3.0, device=dev, dtype=torch.bfloat16)
    Ct = torch.full_like(C, 3.0)
    names = _run(lambda: ops.gemm(A, B, C, m_dev=md, m_hint=live, split_k=1, w192=True))
    assert names == [_name("unsigned short", 0)], names
    ops.gemm(A, B, Ct, m_dev=md, m_hint=live, split_k=1, tile_only=True)
    torch.cuda.synchronize()
    _assert_same("C", C[:live], Ct[:live])
    assert bool((C[live:] == 3.0).all())


def test_w192_layernorm_stats_producer_matches_tile(dev):
    """C and its (mean, M2) per row and 32-column group equal the tile kernel's (the GPT-2 attn c_proj form:
    bias + residual + dropout + statistics, device row count)."""
    M, live, D = 8320, 3584, 768
    md = torch.tensor([live], dtype=torch.int32, device=dev)
    A = rnd((M, D), dev, scale=0.5, seed=31)
    W = rnd((D, D), dev, scale=0.05, seed=32)
    resid = rnd((M, D), dev, scale=2.0, seed=33)
    bias = rnd((D,), dev, torch.float32, 0.1, seed=34)
    drop = ops.Dropout(0.1, seed=99, offset=5)
    out = {}
    for tile in (False, True):
        kw = dict(tile_only=True) if tile else dict(w192=True)
        C = torch.zeros((M, D), device=dev, dtype=torch.bfloat16)
        st = torch.full((M, D // 32, 2), float("nan"), device=dev)
        names = _run(lambda: ops.gemm(A, W, C, bias=bias, resid=resid, drop=drop, m_dev=md, m_hint=live, split_k=1,
                                      ln_stats_out=st, **kw))
        assert all(("4, 1, 3, 4" in n) != tile for n in names), names
        out[tile] = (C, st)
    torch.cuda.synchronize()
    _assert_same("C", out[False][0][:live], out[True][0][:live])
    _assert_same("stats", out[False][1][:live].reshape(live, -1), out[True][1][:live].reshape(live, -1))


def test_w192_f32_output_matches_tile(dev):
    M, N, K = 2048, 1024, 320
    A = rnd((M, K), dev, seed=11)
    B = rnd((N, K), dev, seed=12)
    C = torch.empty((M, N), device=dev, dtype=torch.float32)
    Ct = torch.empty_like(C)
    names = _run(lambda: ops.gemm(A, B, C, split_k=1, w192=True))
    assert names == [_name("float", 0)], names
    ops.gemm(A, B, Ct, split_k=1, tile_only=True)
    torch.cuda.synchronize()
    _assert_same("C", C, Ct)
