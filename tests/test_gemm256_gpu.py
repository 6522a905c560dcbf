"""The 256 x 256 8-phase GEMM (gemm256_kernel, csrc/gemm256.hip) against the 128-row tile kernels and fp64.

Both run the same MFMA 16x16x32 chain per output element (k-steps in order, the two 32-deep halves of each
64-deep step in order) and the shared epilogue (gemm_common.h), so their outputs are bitwise equal for every
epilogue form; fp64 checks the arithmetic. Shapes cover the step's wide products, partial row / column tiles,
K tails (K % 64 != 0), one and two K-tiles (the pipeline's prologue / drain paths) and fp32 output."""

import math

import pytest
import torch

from icap import _lib as L
from icap import ops
from gemm_helpers import _assert_same, _run, rnd

pytestmark = pytest.mark.gpu

SHAPES = [
    (8320, 3072, 768),  # GPT-2 c_fc / activation-gradient product (the dominant launch)
    (8320, 2304, 768),  # GPT-2 QKV
    (6400, 3072, 768),  # CLIP fc1
    (1000, 520, 200),   # partial tiles both ways, K tail (200 = 3 x 64 + 8)
    (512, 256, 64),     # one K-tile
    (768, 768, 128),    # two K-tiles
    (3200, 768, 3072),  # long K
]


@pytest.mark.parametrize("M,N,K", SHAPES)
def test_g256_plain_matches_tile_and_fp64(dev, M, N, K):
    A = rnd((M, K), dev, seed=1)
    B = rnd((N, K), dev, seed=2)
    C = torch.full((M, N), 7.0, device=dev, dtype=torch.bfloat16)
    Ct = torch.empty_like(C)
    names = _run(lambda: ops.gemm(A, B, C, split_k=1, g256=True))
    assert names == ["icap::gemm256_kernel<unsigned short>"], names
    ops.gemm(A, B, Ct, split_k=1, tile_only=True)
    torch.cuda.synchronize()
    _assert_same("C", C, Ct)
    ref = A.double() @ B.double().t()
    err = ((C.double() - ref).abs() / (A.double().abs() @ B.double().abs().t())).max().item()
    assert err < 4e-3, err


@pytest.mark.parametrize("act", [L.ACT_GELU_NEW, L.ACT_QUICK_GELU, L.ACT_RELU])
@pytest.mark.parametrize("M,N,K", [(8320, 3072, 768), (1000, 520, 200)])
def test_g256_epilogues_match_tile(dev, act, M, N, K):
    A = rnd((M, K), dev, scale=0.1, seed=6)
    B = rnd((N, K), dev, scale=0.1, seed=7)
    bias = rnd((N,), dev, torch.float32, 0.5, seed=8)
    resid = rnd((M, N), dev, seed=9)
    drop = ops.Dropout(0.1, seed=1234, offset=77)
    out = {}
    for tile in (False, True):
        C = torch.empty((M, N), device=dev, dtype=torch.bfloat16)
        aux, C2, dZ = torch.empty_like(C), torch.empty_like(C), torch.empty_like(C)
        names = _run(lambda: (ops.gemm(A, B, C, bias=bias, act=act, aux=aux, split_k=1, tile_only=tile, g256=not tile),
                              ops.gemm(A, B, C2, bias=bias, resid=resid, drop=drop, alpha=0.75, split_k=1,
                                       tile_only=tile, g256=not tile),
                              ops.gemm(A, B, dZ, dact=act, dact_src=aux, drop=drop, alpha=0.5, split_k=1,
                                       tile_only=tile, g256=not tile)))
        assert all(("gemm256_kernel" in n) != tile for n in names), names
        out[tile] = (C, aux, C2, dZ)
    torch.cuda.synchronize()
    for name, a, b in zip(("C", "aux", "C2", "dZ"), out[False], out[True]):
        _assert_same(name, a, b)
    z = A.double() @ B.double().t() + bias.double()
    y = {L.ACT_GELU_NEW: lambda v: 0.5 * v * (1 + torch.tanh(math.sqrt(2 / math.pi) * (v + 0.044715 * v ** 3))),
         L.ACT_QUICK_GELU: lambda v: v * torch.sigmoid(1.702 * v), L.ACT_RELU: torch.relu}[act](z)
    assert (out[False][0].double() - y).abs().max().item() < 2e-2 * max(1.0, y.abs().max().item())
    kept = (out[False][2].double() != resid.double()).float().mean().item()
    assert 0.85 < kept <= 1.0


def test_g256_f32_output_matches_tile(dev):
    M, N, K = 2048, 1024, 320
    A = rnd((M, K), dev, seed=11)
    B = rnd((N, K), dev, seed=12)
    C = torch.empty((M, N), device=dev, dtype=torch.float32)
    Ct = torch.empty_like(C)
    names = _run(lambda: ops.gemm(A, B, C, split_k=1, g256=True))
    assert names == ["icap::gemm256_kernel<float>"], names
    ops.gemm(A, B, Ct, split_k=1, tile_only=True)
    torch.cuda.synchronize()
    _assert_same("C", C, Ct)


def test_g256_strided_operands(dev):
    """Leading dimensions larger than K / N (views into wider buffers)."""
    M, N, K = 1536, 768, 512
    Aw = rnd((M, K + 64), dev, seed=13)
    Bw = rnd((N, K + 128), dev, seed=14)
    A, B = Aw[:, :K], Bw[:, :K]
    Cw = torch.zeros((M, N + 32), device=dev, dtype=torch.bfloat16)
    Ct = torch.empty((M, N), device=dev, dtype=torch.bfloat16)
    ops.gemm(A, B, Cw[:, :N], split_k=1, g256=True)
    ops.gemm(A, B, Ct, split_k=1, tile_only=True)
    torch.cuda.synchronize()
    _assert_same("C", Cw[:, :N], Ct)
    assert torch.count_nonzero(Cw[:, N:]) == 0
