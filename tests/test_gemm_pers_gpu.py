"""The persistent split-role GEMM with the overlapped epilogue (round 6: gemm_pers_kernel, csrc/gemm_pers.h; variant 30,
ops.gemm(roles=1)) against the 128-row tile kernels and fp64.

Each block walks several 96 x 128 tiles: 4 MFMA waves run tile j's k-steps while 4 loader waves stream the ring across
tile boundaries and 4 epilogue waves store tile j-1 from an LDS C buffer, a slice of rows per k-step. The MFMA chain per
output element is the tile kernel's (64-deep k-steps in natural order) and the epilogue arithmetic is the shared epiw,
so every output is bitwise the tile path's (tile_only=True, split_k=1): plain, bias / residual / dropout / alpha, gelu_new
+ aux, dgelu, relu fwd / bwd, the device row count, the LayerNorm statistics producer and consumer, fp32 C. The shapes
give blocks one to seven tiles, partial row / column tiles, K tails and fewer k-steps than epilogue row groups; these
are also the race screen of the C-buffer hand-off (a tile stored before its accumulators landed, or overwritten before
its rows were stored, shows up as a bitwise difference)."""

import pytest
import torch

from icap import _lib as L
from icap import ops
from gemm_helpers import _assert_same, _run, rnd

pytestmark = pytest.mark.gpu

SHAPES = [  # (M, N, K)
    (3584, 3072, 768),   # GPT-2 c_fc / mlp c_proj dX: 912 tiles, 3-4 per block
    (6400, 3072, 768),   # CLIP fc1: 1600 tiles
    (6400, 768, 3072),   # CLIP fc2: 400 tiles, long K
    (3584, 768, 768),    # one round
    (1000, 520, 200),    # partial tiles both ways, K tail
    (384, 256, 64),      # one k-step per tile
    (200, 130, 128),
    (8320, 2304, 768),   # many rounds
]


def _name(tc, act):
    return f"icap::gemm_pers_kernel<{tc}, 3, 3, 4, {act}>"


@pytest.mark.parametrize("M,N,K", SHAPES)
def test_pers_plain_matches_tile_and_fp64(dev, M, N, K):
    A = rnd((M, K), dev, seed=1)
    B = rnd((N, K), dev, seed=2)
    C = torch.full((M, N), 7.0, device=dev, dtype=torch.bfloat16)
    Ct = torch.empty_like(C)
    names = _run(lambda: ops.gemm(A, B, C, split_k=1, roles=1))
    assert names == [_name("unsigned short", 0)], names
    ops.gemm(A, B, Ct, split_k=1, tile_only=True)
    torch.cuda.synchronize()
    _assert_same("C", C, Ct)
    ref = A.double() @ B.double().t()
    err = ((C.double() - ref).abs() / (A.double().abs() @ B.double().abs().t())).max().item()
    assert err < 4e-3, err


def test_pers_repeatable(dev):
    """20 launches of a 4-tiles-per-block product are bitwise identical."""
    M, N, K = 3584, 3072, 1536
    A = rnd((M, K), dev, seed=3)
    B = rnd((N, K), dev, seed=4)
    C0 = torch.empty((M, N), device=dev, dtype=torch.bfloat16)
    ops.gemm(A, B, C0, split_k=1, roles=1)
    outs = []
    for _ in range(20):
        C = torch.empty_like(C0)
        ops.gemm(A, B, C, split_k=1, roles=1)
        outs.append(C)
    torch.cuda.synchronize()
    for i, C in enumerate(outs):
        _assert_same(f"launch {i}", C, C0)


@pytest.mark.parametrize("M,N,K", [(3584, 3072, 768), (1000, 520, 200), (384, 256, 64), (6400, 768, 3072)])
def test_pers_epilogues_match_tile(dev, M, N, K):
    A = rnd((M, K), dev, scale=0.1, seed=6)
    B = rnd((N, K), dev, scale=0.1, seed=7)
    bias = rnd((N,), dev, torch.float32, 0.5, seed=8)
    resid = rnd((M, N), dev, seed=9)
    dsrc = rnd((M, N), dev, seed=10)
    drop = ops.Dropout(0.1, seed=1234, offset=77)
    out = {}
    for tile in (False, True):
        kw = dict(tile_only=True) if tile else dict(roles=1)
        C = torch.empty((M, N), device=dev, dtype=torch.bfloat16)
        C2, dZ, G, Ga, R, dR = (torch.empty_like(C) for _ in range(6))
        names = _run(lambda: (ops.gemm(A, B, C, bias=bias, resid=resid, drop=drop, alpha=0.75, split_k=1, **kw),
                              ops.gemm(A, B, dZ, dact=L.ACT_GELU_NEW, dact_src=dsrc, drop=drop, alpha=0.5, split_k=1,
                                       **kw),
                              ops.gemm(A, B, C2, bias=bias, act=L.ACT_QUICK_GELU, split_k=1, **kw),
                              ops.gemm(A, B, G, bias=bias, act=L.ACT_GELU_NEW, aux=Ga, split_k=1, **kw),
                              ops.gemm(A, B, R, bias=bias, act=L.ACT_RELU, drop=drop, split_k=1, **kw),
                              ops.gemm(A, B, dR, dact=L.ACT_RELU, dact_src=dsrc, split_k=1, **kw)))
        assert all(("gemm_pers_kernel" in n) != tile for n in names), names
        out[tile] = (C, dZ, C2, G, Ga, R, dR)
    torch.cuda.synchronize()
    for name, a, b in zip(("C", "dZ", "quick_gelu", "gelu", "gelu aux", "relu", "drelu"), out[False], out[True]):
        _assert_same(name, a, b)


@pytest.mark.parametrize("N", [768, 3072])
def test_pers_device_row_count(dev, N):
    M, live, K = 8320, 3584, 768
    A = rnd((M, K), dev, seed=21)
    B = rnd((N, K), dev, seed=22)
    md = torch.tensor([live], dtype=torch.int32, device=dev)
    C = torch.full((M, N), 3.0, device=dev, dtype=torch.bfloat16)
    Ct = torch.full_like(C, 3.0)
    names = _run(lambda: ops.gemm(A, B, C, m_dev=md, m_hint=live, split_k=1, roles=1))
    assert names == [_name("unsigned short", 0)], names
    ops.gemm(A, B, Ct, m_dev=md, m_hint=live, split_k=1, tile_only=True)
    torch.cuda.synchronize()
    _assert_same("C", C[:live], Ct[:live])
    assert bool((C[live:] == 3.0).all())


def test_pers_layernorm_stats_producer_matches_tile(dev):
    M, live, D, K = 8320, 3584, 768, 3072
    md = torch.tensor([live], dtype=torch.int32, device=dev)
    A = rnd((M, K), dev, scale=0.5, seed=31)
    W = rnd((D, K), dev, scale=0.05, seed=32)
    resid = rnd((M, D), dev, scale=2.0, seed=33)
    bias = rnd((D,), dev, torch.float32, 0.1, seed=34)
    drop = ops.Dropout(0.1, seed=99, offset=5)
    out = {}
    for tile in (False, True):
        kw = dict(tile_only=True) if tile else dict(roles=1)
        C = torch.zeros((M, D), device=dev, dtype=torch.bfloat16)
        st = torch.full((M, D // 32, 2), float("nan"), device=dev)
        names = _run(lambda: ops.gemm(A, W, C, bias=bias, resid=resid, drop=drop, m_dev=md, m_hint=live, split_k=1,
                                      ln_stats_out=st, **kw))
        assert all(("gemm_pers_kernel" in n) != tile for n in names), names
        out[tile] = (C, st)
    torch.cuda.synchronize()
    _assert_same("C", out[False][0][:live], out[True][0][:live])
    _assert_same("stats", out[False][1][:live].reshape(live, -1), out[True][1][:live].reshape(live, -1))


@pytest.mark.parametrize("N,act", [(2304, L.ACT_NONE), (3072, L.ACT_GELU_NEW), (3072, L.ACT_QUICK_GELU)])
def test_pers_layernorm_consumer_matches_tile(dev, N, act):
    from icap.gpt2 import fold_layernorm

    M, live, K = 8320, 3584, 768
    md = torch.tensor([live], dtype=torch.int32, device=dev)
    g = torch.Generator().manual_seed(N + act)
    x = (torch.randn((M, K), generator=g) * 2 + 0.5).to(dev, torch.bfloat16)
    w = (torch.randn((N, K), generator=g) * 0.05).to(dev)
    gamma = (1 + 0.2 * torch.randn(K, generator=g)).to(dev)
    beta = (0.1 * torch.randn(K, generator=g)).to(dev)
    bias = (0.1 * torch.randn(N, generator=g)).to(dev)
    wf, wsum, bf = fold_layernorm(w, gamma, beta, bias, torch.bfloat16)
    xf = x.float()
    grp = xf.view(M, K // 32, 32)
    st = torch.stack((grp.mean(-1), ((grp - grp.mean(-1, keepdim=True)) ** 2).sum(-1)), -1).contiguous()
    out = {}
    for tile in (False, True):
        kw = dict(tile_only=True) if tile else dict(roles=1)
        C = torch.zeros((M, N), device=dev, dtype=torch.bfloat16)
        aux = torch.zeros_like(C) if act == L.ACT_GELU_NEW else None
        mo, ro = torch.zeros(M, device=dev), torch.zeros(M, device=dev)
        names = _run(lambda: ops.gemm(x, wf, C, bias=bf, act=act, aux=aux, ln_fold=(wsum, 1e-5), ln_stats_in=st,
                                      ln_rows_out=(mo, ro), m_dev=md, m_hint=live, split_k=1, **kw))
        assert all(("gemm_pers_kernel" in n) != tile for n in names), names
        out[tile] = (C, mo, ro) + ((aux,) if aux is not None else ())
    torch.cuda.synchronize()
    for name, a, b in zip(("C", "mean", "rstd", "aux"), out[False], out[True]):
        _assert_same(name, a[:live], b[:live])


def test_pers_f32_output_matches_tile(dev):
    M, N, K = 2048, 1024, 320
    A = rnd((M, K), dev, seed=11)
    B = rnd((N, K), dev, seed=12)
    C = torch.empty((M, N), device=dev, dtype=torch.float32)
    Ct = torch.empty_like(C)
    names = _run(lambda: ops.gemm(A, B, C, split_k=1, roles=1))
    assert names == [_name("float", 0)], names
    ops.gemm(A, B, Ct, split_k=1, tile_only=True)
    torch.cuda.synchronize()
    _assert_same("C", C, Ct)
