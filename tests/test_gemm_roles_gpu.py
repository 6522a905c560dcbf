"""The split-role ring kernels (round 6: gemm_kernel<..., ROLES = true>, csrc/gemm_tile.h; variant 26 = 128 x 256 tiles,
csrc/gemm_tile_roles.hip; variant 27 = 96 x 128 tiles, csrc/gemm_tile_roles96.hip; variant 32 = 160 x 128 tiles,
csrc/gemm_tile_roles160.hip) against the 128-row tile kernels
and fp64.

Four MFMA waves read fragments and issue the MFMAs, four loader waves issue the LDS-DMA of the ring; the MFMA chain per
output element is the tile kernel's (64-deep k-steps in natural order, their two 32-deep halves in order) and the
epilogue is the shared one, so the outputs are bitwise equal to the tile path (tile_only=True, split_k=1) for every
epilogue form: plain, bias / residual / dropout / alpha, gelu_new + aux, dgelu, relu through the dispatching form, the
device row count (packed rows), the LayerNorm statistics producer and (variant 26) the LayerNorm consumer. Shapes: the
packed step's products, partial row / column tiles, K tails, fewer k-steps than ring stages, fp32 output. These are
also the race screen of the ring's barrier protocol: a slot read before its DMA landed, or re-filled before every wave
read it, shows up as a bitwise difference."""

import pytest
import torch

from icap import _lib as L
from icap import ops
from gemm_helpers import _assert_same, _run, rnd

pytestmark = pytest.mark.gpu

R256, R96, R192, R160 = "3, 1, 2, 2, 4, 8", "5, 1, 2, 2, 3, 4", "2, 1, 2, 4, 6, 4", "4, 1, 2, 2, 5, 4"

SHAPES = [  # (M, N, K, roles)
    (3584, 2304, 768, 256),  # GPT-2 c_attn at the packed rows
    (3584, 3072, 768, 256),  # c_fc / mlp c_proj dX
    (3584, 768, 768, 96),    # attn c_proj
    (3584, 768, 2304, 96),   # c_attn dX
    (3584, 768, 3072, 96),   # mlp c_proj
    (1000, 520, 200, 256),   # partial tiles both ways, K tail (200 = 3 x 64 + 8)
    (1000, 520, 200, 96),
    (384, 256, 64, 256),     # one k-step (fewer than the ring's stages)
    (200, 130, 128, 96),     # two k-steps, partial tiles
    (6400, 2304, 768, 256),  # CLIP-B/32 qkv
    (3584, 3072, 768, 192),  # c_fc / mlp c_proj dX on 192 x 256 tiles (8 MFMA waves)
    (1000, 520, 200, 192),
    (384, 256, 64, 192),
    (3200, 3072, 768, 192),  # the mapper's linear1
    (6400, 768, 768, 160),   # CLIP-B/32 out_proj on 160 x 128 tiles (variant 32)
    (6400, 768, 3072, 160),  # CLIP-B/32 fc2
    (1000, 520, 200, 160),
    (200, 130, 128, 160),
]


def _name(tc, act, roles):
    form = {256: R256, 96: R96, 192: R192, 160: R160}[roles]
    return f"icap::gemm_kernel<unsigned short, {tc}, {form}, false, {act}, true>"


@pytest.mark.parametrize("M,N,K,roles", SHAPES)
def test_roles_plain_matches_tile_and_fp64(dev, M, N, K, roles):
    A = rnd((M, K), dev, seed=1)
    B = rnd((N, K), dev, seed=2)
    C = torch.full((M, N), 7.0, device=dev, dtype=torch.bfloat16)
    Ct = torch.empty_like(C)
    names = _run(lambda: ops.gemm(A, B, C, split_k=1, roles=roles))
    assert names == [_name("unsigned short", 0, roles)], names
    ops.gemm(A, B, Ct, split_k=1, tile_only=True)
    torch.cuda.synchronize()
    _assert_same("C", C, Ct)
    ref = A.double() @ B.double().t()
    err = ((C.double() - ref).abs() / (A.double().abs() @ B.double().abs().t())).max().item()
    assert err < 4e-3, err


def test_roles_repeatable(dev):
    """20 launches of the same product (the ring's protocol under back-to-back blocks) are bitwise identical."""
    M, N, K = 3584, 2304, 1536
    A = rnd((M, K), dev, seed=3)
    B = rnd((N, K), dev, seed=4)
    C0 = torch.empty((M, N), device=dev, dtype=torch.bfloat16)
    ops.gemm(A, B, C0, split_k=1, roles=256)
    outs = []
    for _ in range(20):
        C = torch.empty_like(C0)
        ops.gemm(A, B, C, split_k=1, roles=256)
        outs.append(C)
    torch.cuda.synchronize()
    for i, C in enumerate(outs):
        _assert_same(f"launch {i}", C, C0)


@pytest.mark.parametrize("M,N,K,roles", [(3584, 2304, 768, 256), (1000, 520, 200, 256), (3584, 768, 768, 96),
                                         (1000, 520, 200, 96), (3584, 3072, 768, 192), (1000, 520, 200, 192),
                                         (6400, 768, 768, 160), (1000, 520, 200, 160)])
def test_roles_epilogues_match_tile(dev, M, N, K, roles):
    A = rnd((M, K), dev, scale=0.1, seed=6)
    B = rnd((N, K), dev, scale=0.1, seed=7)
    bias = rnd((N,), dev, torch.float32, 0.5, seed=8)
    resid = rnd((M, N), dev, seed=9)
    dsrc = rnd((M, N), dev, seed=10)
    drop = ops.Dropout(0.1, seed=1234, offset=77)
    out = {}
    for tile in (False, True):
        kw = dict(tile_only=True) if tile else dict(roles=roles)
        C = torch.empty((M, N), device=dev, dtype=torch.bfloat16)
        C2, dZ, G, Ga = (torch.empty_like(C) for _ in range(4))
        names = _run(lambda: (ops.gemm(A, B, C, bias=bias, resid=resid, drop=drop, alpha=0.75, split_k=1, **kw),
                              ops.gemm(A, B, dZ, dact=L.ACT_GELU_NEW, dact_src=dsrc, drop=drop, alpha=0.5, split_k=1,
                                       **kw),
                              ops.gemm(A, B, C2, bias=bias, act=L.ACT_RELU, split_k=1, **kw),
                              ops.gemm(A, B, G, bias=bias, act=L.ACT_GELU_NEW, aux=Ga, split_k=1, **kw)))
        assert all(n.endswith(", true>") != tile for n in names), names
        out[tile] = (C, dZ, C2, G, Ga)
    torch.cuda.synchronize()
    for name, a, b in zip(("C", "dZ", "relu", "gelu", "gelu aux"), out[False], out[True]):
        _assert_same(name, a, b)


@pytest.mark.parametrize("roles,N", [(256, 2304), (96, 768), (192, 3072), (160, 768)])
def test_roles_device_row_count(dev, roles, N):
    """m_dev: rows past the device count are neither computed nor stored; the rest equal the tile path's."""
    M, live, K = 8320, 3584, 768
    A = rnd((M, K), dev, seed=21)
    B = rnd((N, K), dev, seed=22)
    md = torch.tensor([live], dtype=torch.int32, device=dev)
    C = torch.full((M, N), 3.0, device=dev, dtype=torch.bfloat16)
    Ct = torch.full_like(C, 3.0)
    names = _run(lambda: ops.gemm(A, B, C, m_dev=md, m_hint=live, split_k=1, roles=roles))
    assert names == [_name("unsigned short", 0, roles)], names
    ops.gemm(A, B, Ct, m_dev=md, m_hint=live, split_k=1, tile_only=True)
    torch.cuda.synchronize()
    _assert_same("C", C[:live], Ct[:live])
    assert bool((C[live:] == 3.0).all())


@pytest.mark.parametrize("roles", [256, 96, 192, 160])
def test_roles_layernorm_stats_producer_matches_tile(dev, roles):
    """C and its (mean, M2) per row and 32-column group equal the tile kernel's (the GPT-2 attn c_proj form: bias +
    residual + dropout + statistics, device row count)."""
    M, live, D = 8320, 3584, 768
    md = torch.tensor([live], dtype=torch.int32, device=dev)
    A = rnd((M, D), dev, scale=0.5, seed=31)
    W = rnd((D, D), dev, scale=0.05, seed=32)
    resid = rnd((M, D), dev, scale=2.0, seed=33)
    bias = rnd((D,), dev, torch.float32, 0.1, seed=34)
    drop = ops.Dropout(0.1, seed=99, offset=5)
    out = {}
    for tile in (False, True):
        kw = dict(tile_only=True) if tile else dict(roles=roles)
        C = torch.zeros((M, D), device=dev, dtype=torch.bfloat16)
        st = torch.full((M, D // 32, 2), float("nan"), device=dev)
        names = _run(lambda: ops.gemm(A, W, C, bias=bias, resid=resid, drop=drop, m_dev=md, m_hint=live, split_k=1,
                                      ln_stats_out=st, **kw))
        assert all(n.endswith(", true>") != tile for n in names), names
        out[tile] = (C, st)
    torch.cuda.synchronize()
    _assert_same("C", out[False][0][:live], out[True][0][:live])
    _assert_same("stats", out[False][1][:live].reshape(live, -1), out[True][1][:live].reshape(live, -1))


@pytest.mark.parametrize("N,act,roles", [(2304, L.ACT_NONE, 256), (3072, L.ACT_GELU_NEW, 256),
                                         (3072, L.ACT_GELU_NEW, 192), (3072, L.ACT_QUICK_GELU, 192)])
def test_roles_layernorm_consumer_matches_tile(dev, N, act, roles):
    """The LayerNorm folded into the consumer's epilogue from handed-over statistics (GPT-2's c_attn / c_fc forward,
    device row count): C and the row mean / rstd outputs equal the tile kernel's."""
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
        kw = dict(tile_only=True) if tile else dict(roles=roles)
        C = torch.zeros((M, N), device=dev, dtype=torch.bfloat16)
        aux = torch.zeros_like(C) if act == L.ACT_GELU_NEW else None
        mo, ro = torch.zeros(M, device=dev), torch.zeros(M, device=dev)
        names = _run(lambda: ops.gemm(x, wf, C, bias=bf, act=act, aux=aux, ln_fold=(wsum, 1e-5), ln_stats_in=st,
                                      ln_rows_out=(mo, ro), m_dev=md, m_hint=live, split_k=1, **kw))
        assert all(n.endswith(", true>") != tile for n in names), names
        out[tile] = (C, mo, ro) + ((aux,) if aux is not None else ())
    torch.cuda.synchronize()
    for name, a, b in zip(("C", "mean", "rstd", "aux"), out[False], out[True]):
        _assert_same(name, a[:live], b[:live])


@pytest.mark.parametrize("roles", [256, 96, 192, 160])
def test_roles_f32_output_matches_tile(dev, roles):
    M, N, K = 2048, 1024, 320
    A = rnd((M, K), dev, seed=11)
    B = rnd((N, K), dev, seed=12)
    C = torch.empty((M, N), device=dev, dtype=torch.float32)
    Ct = torch.empty_like(C)
    names = _run(lambda: ops.gemm(A, B, C, split_k=1, roles=roles))
    assert names == [_name("float", 0, roles)], names
    ops.gemm(A, B, Ct, split_k=1, tile_only=True)
    torch.cuda.synchronize()
    _assert_same("C", C, Ct)


@pytest.mark.parametrize("roles,split", [(96, 3), (256, 4), (160, 2)])
def test_roles_split_k_matches_tile(dev, roles, split):
    """A caller's split_k > 1 on the split-role rings (the long-K LM head dX): each split's K range on the ring, fp32
    slabs, the same reduce pass — bitwise the tile kernel at the same split (device row count, K tail, partial tiles)."""
    M, N, K, live = 1000, 776, 8192 + 40, 931
    A = rnd((M, K), dev, scale=0.1, seed=21)
    B = rnd((N, K), dev, scale=0.1, seed=22)
    md = torch.tensor([live], dtype=torch.int32, device=dev)
    ws = torch.empty(split * M * N, device=dev, dtype=torch.float32)
    C = torch.full((M, N), 3.0, device=dev, dtype=torch.bfloat16)
    Ct = C.clone()
    names = _run(lambda: ops.gemm(A, B, C, m_dev=md, m_hint=live, split_k=split, roles=roles, workspace=ws))
    assert names == [_name("unsigned short", 0, roles)], names
    ops.gemm(A, B, Ct, m_dev=md, m_hint=live, split_k=split, tile_only=True, workspace=ws)
    torch.cuda.synchronize()
    _assert_same("C", C[:live], Ct[:live])
    ref = A[:live].double() @ B.double().t()
    err = ((C[:live].double() - ref).abs() / (A[:live].double().abs() @ B.double().abs().t())).max().item()
    assert err < 1e-2, err
