"""The persistent ring GEMM (gemm_ring_kernel, csrc/gemm.hip) against the 128-row tile kernels and an fp64 reference.

Both paths run the same MFMA 16x16x32 chains in the same k order and apply the same epilogue arithmetic, so their
outputs must be bitwise equal for every epilogue form the train step uses (bias / gelu_new + aux store / relu /
quick_gelu / tanh aux / dropout / residual / backward dact, alpha, device row counts); the fp64 reference checks
the shared arithmetic. Shapes cover both tile heights (256 x 128 when the 256-row tiles fill the chip, 128 x 128
otherwise), several output tiles per workgroup (the persistent stream across tile boundaries), K tails (K % 64 !=
0), partial row / column tiles and the step's real shapes."""

import math

import pytest
import torch

from icap import _lib as L
from icap import ops

pytestmark = pytest.mark.gpu


def rnd(shape, dev, dtype=torch.bfloat16, scale=1.0, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.randn(shape, generator=g) * scale).to(device=dev, dtype=dtype)


class _Names:
    """ops.GEMM_TIMER hook that records which kernel instantiation each launch used."""

    def __init__(self):
        self.names = []

    def launch(self, key, flops, fn):
        self.names.append(key[0])
        fn()


def _run(fn):
    rec = _Names()
    ops.GEMM_TIMER = rec
    try:
        fn()
    finally:
        ops.GEMM_TIMER = None
    return rec.names


def _assert_same(name, a, b):
    if torch.equal(a, b):
        return
    bad = (a != b).nonzero()
    d = (a.float() - b.float()).abs().max().item()
    rows = sorted(set(bad[:, 0].tolist()))
    cols = sorted(set(bad[:, 1].tolist()))
    raise AssertionError(f"{name}: {bad.shape[0]} of {a.numel()} differ (max |d| {d:.3g}); rows {rows[:12]}"
                         f"{'...' if len(rows) > 12 else ''} ({len(rows)}), cols {cols[:12]}"
                         f"{'...' if len(cols) > 12 else ''} ({len(cols)})")


SHAPES = [
    (8320, 768, 3072),   # GPT-2 mlp.c_proj / c_fc dX (N = 768, long K): 256 x 128 tiles, one per CU
    (8320, 3072, 768),   # c_fc / dgelu (short K): ~3 tiles per workgroup
    (3200, 768, 3072),   # mapper: 128 x 128 tiles
    (6400, 2304, 768),   # CLIP qkv
    (1000, 136, 200),    # partial row / column tiles, K tail (200 = 3 x 64 + 8)
    (520, 1024, 192),    # three k-steps per tile (the fewest the ring kernel takes)
]


@pytest.mark.parametrize("M,N,K", SHAPES)
def test_ring_plain_matches_tile_and_fp64(dev, M, N, K):
    A = rnd((M, K), dev, seed=1)
    B = rnd((N, K), dev, seed=2)
    C = torch.empty((M, N), device=dev, dtype=torch.bfloat16)
    Ct = torch.empty_like(C)
    names = _run(lambda: ops.gemm(A, B, C, split_k=1, ring=True))
    assert "gemm_ring_kernel" in names[0], names
    ops.gemm(A, B, Ct, split_k=1, tile_only=True)
    torch.cuda.synchronize()
    _assert_same("C", C, Ct)
    ref = A.double() @ B.double().t()
    err = ((C.double() - ref).abs() / (A.double().abs() @ B.double().abs().t())).max().item()
    assert err < 4e-3, err  # bf16 output rounding (2^-8 relative) of an fp32-accumulated exact-product sum


def _act_ref(act, z):
    if act == L.ACT_GELU_NEW:
        return 0.5 * z * (1 + torch.tanh(math.sqrt(2 / math.pi) * (z + 0.044715 * z ** 3)))
    if act == L.ACT_RELU:
        return torch.relu(z)
    if act == L.ACT_QUICK_GELU:
        return z * torch.sigmoid(1.702 * z)
    return torch.tanh(z)


@pytest.mark.parametrize("act", [L.ACT_GELU_NEW, L.ACT_RELU, L.ACT_QUICK_GELU, L.ACT_TANH])
@pytest.mark.parametrize("M,N,K", [(8320, 3072, 768), (3200, 768, 3072), (1000, 136, 200)])
def test_ring_epilogues_match_tile(dev, act, M, N, K):
    A = rnd((M, K), dev, scale=0.1, seed=6)
    B = rnd((N, K), dev, scale=0.1, seed=7)
    bias = rnd((N,), dev, torch.float32, 0.5, seed=8)
    resid = rnd((M, N), dev, seed=9)
    drop = ops.Dropout(0.1, seed=1234, offset=77)
    out = {}
    for tile in (False, True):
        C = torch.empty((M, N), device=dev, dtype=torch.bfloat16)
        aux = torch.empty_like(C)
        C2 = torch.empty_like(C)
        dZ = torch.empty_like(C)
        names = _run(lambda: (ops.gemm(A, B, C, bias=bias, act=act, aux=aux, split_k=1, tile_only=tile,
                                       ring=not tile),
                              ops.gemm(A, B, C2, bias=bias, resid=resid, drop=drop, alpha=0.75, split_k=1,
                                       tile_only=tile, ring=not tile),
                              ops.gemm(A, B, dZ, dact=act, dact_src=aux, drop=drop, alpha=0.5, split_k=1,
                                       tile_only=tile, ring=not tile)))
        assert all(("gemm_ring_kernel" in n) != tile for n in names), names
        out[tile] = (C, aux, C2, dZ)
    torch.cuda.synchronize()
    for name, a, b in zip(("C", "aux", "C2", "dZ"), out[False], out[True]):
        _assert_same(name, a, b)
    C, aux, C2, _ = out[False]
    z = A.double() @ B.double().t() + bias.double()
    y = _act_ref(act, z)
    rel = lambda a, b: ((a.double() - b).abs().max() / b.abs().max()).item()  # noqa: E731
    assert rel(C, y) < 1e-2 and rel(aux, y if act == L.ACT_TANH else z) < 1e-2
    kept = C2 != resid  # dropped positions carry the residual alone
    z2 = 0.75 * (A.double() @ B.double().t()) + bias.double()
    frac = 1.0 - kept.double().mean().item()
    assert 0.08 < frac < 0.12, frac
    assert rel(torch.where(kept, C2.double(), resid.double() + z2 / 0.9), resid.double() + z2 / 0.9) < 1e-2


def test_ring_device_row_count(dev):
    """m_dev: only rows < *m_dev are computed and stored (LM head over the compacted targets)."""
    M, N, K = 6400, 1024, 768
    A = rnd((M, K), dev, seed=11)
    B = rnd((N, K), dev, seed=12)
    for mv in (1792, 1, 256, 6400):
        m_dev = torch.tensor([mv], dtype=torch.int32, device=dev)
        C = torch.full((M, N), 7.0, device=dev, dtype=torch.bfloat16)
        Ct = C.clone()
        names = _run(lambda: ops.gemm(A, B, C, m_dev=m_dev, split_k=1, ring=True))
        assert "gemm_ring_kernel" in names[0]
        ops.gemm(A, B, Ct, m_dev=m_dev, split_k=1, tile_only=True)
        torch.cuda.synchronize()
        assert torch.equal(C, Ct)
        assert (C[mv:] == 7.0).all()


def test_ring_strided_operands(dev):
    """Leading dimensions larger than the logical widths (views into wider buffers), as the fused QKV / cache
    layouts pass them."""
    M, N, K = 2000, 512, 384
    Af = rnd((M, K + 64), dev, seed=13)
    Bf = rnd((N, K + 128), dev, seed=14)
    A, B = Af[:, 64:], Bf[:, :K]
    Cf = torch.zeros((M, N + 256), device=dev, dtype=torch.bfloat16)
    C = Cf[:, 128:128 + N]
    Ct = torch.empty((M, N), device=dev, dtype=torch.bfloat16)
    names = _run(lambda: ops.gemm(A, B, C, split_k=1, ring=True))
    assert "gemm_ring_kernel" in names[0]
    ops.gemm(A, B, Ct, split_k=1, tile_only=True)
    torch.cuda.synchronize()
    assert torch.equal(C, Ct)
    assert (Cf[:, :128] == 0).all() and (Cf[:, 128 + N:] == 0).all()
