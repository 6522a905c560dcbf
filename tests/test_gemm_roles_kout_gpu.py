"""The K-outer split-role GEMM (round 6: gemm_kernel<..., KOUT = true, ..., ROLES = true>, variant 31,
csrc/gemm_tile_roles_kout.hip; ops.gemm(trans_ab=True, roles=1)) — the mapper's weight gradients dW[N, K] += dY[rows, N]^T
X[rows, K] read in place — against the K-outer tile kernels and fp64.

Four MFMA waves read their fragments with ds_read_b64_tr_b16 from the same T10 (b) images the tile kernel uses (same k
order on both operands) while four loader waves stream the 4-stage ring, so an unsplit product is bitwise the tile
kernel's unsplit one, and a product split S ways is bitwise the tile kernel's S-way split (same K ranges, same slab +
reduce pass). Shapes: the packed step's four products over 3200 token rows, partial tiles and a row count that is no
multiple of 64; fp32 gradients with beta 0 / 1; the 20-launch repeatability screen of the ring's barrier protocol."""

import pytest
import torch

from icap import ops
from gemm_helpers import _assert_same, _run, rnd

pytestmark = pytest.mark.gpu

SHAPES = [  # (N, K, rows)
    (2304, 768, 3200),
    (768, 768, 3200),
    (3072, 768, 3200),
    (768, 3072, 3200),
    (520, 200, 1000),
    (256, 136, 72),
]
NAME = "icap::gemm_kernel<unsigned short, float, 4, 1, 2, 2, 4, 4, true, 0, true>"


def _operands(dev, N, K, rows, seed):
    dY = rnd((rows, N), dev, scale=0.2, seed=seed)
    X = rnd((rows, K), dev, seed=seed + 1)
    G = rnd((N, K), dev, torch.float32, 1.0, seed=seed + 2)
    return dY, X, G


@pytest.mark.parametrize("N,K,rows", SHAPES)
@pytest.mark.parametrize("beta", [0.0, 1.0])
def test_roles_kout_unsplit_matches_tile(dev, N, K, rows, beta):
    dY, X, G = _operands(dev, N, K, rows, 1)
    C, Ct = G.clone(), G.clone()
    names = _run(lambda: ops.gemm(dY, X, C, beta=beta, M=N, N=K, K=rows, trans_ab=True, split_k=1, roles=1))
    assert names == [NAME], names
    ops.gemm(dY, X, Ct, beta=beta, M=N, N=K, K=rows, trans_ab=True, split_k=1, tile_only=True)
    torch.cuda.synchronize()
    _assert_same("dW", C, Ct)
    ref = dY.double().t() @ X.double() + beta * G.double()
    err = ((C.double() - ref).abs() / (dY.double().abs().t() @ X.double().abs() + beta * G.double().abs())).max()
    assert err.item() < 1e-5, err.item()


@pytest.mark.parametrize("N,K,rows", SHAPES[:4])
def test_roles_kout_split_matches_tile_split(dev, N, K, rows):
    """The automatic split of the roles form equals the tile kernel forced to the same split count, bit for bit."""
    from test_fused_splitk_gpu import _kernel_names

    dY, X, G = _operands(dev, N, K, rows, 5)
    C, Ct = G.clone(), G.clone()
    ws = torch.empty(8 * N * K + 64, device=dev, dtype=torch.float32)
    recs = _kernel_names(lambda: ops.gemm(dY, X, C, beta=1.0, M=N, N=K, K=rows, trans_ab=True, split_k=0, roles=1,
                                          workspace=ws))
    (name, splits, fused), = recs
    assert name == NAME and not fused, recs  # (3072 x 768: 144 tiles, unsplit)
    ops.gemm(dY, X, Ct, beta=1.0, M=N, N=K, K=rows, trans_ab=True, split_k=splits, tile_only=True, workspace=ws)
    torch.cuda.synchronize()
    _assert_same("dW", C, Ct)


def test_roles_kout_repeatable(dev):
    N, K, rows = 2304, 768, 3200
    dY, X, G = _operands(dev, N, K, rows, 9)
    outs = []
    for _ in range(20):
        C = G.clone()
        ops.gemm(dY, X, C, beta=1.0, M=N, N=K, K=rows, trans_ab=True, split_k=0, roles=1)
        outs.append(C)
    torch.cuda.synchronize()
    for i, C in enumerate(outs[1:]):
        _assert_same(f"launch {i + 1}", C, outs[0])


def test_gemm_group_matches_single_products(dev):
    """icap_gemm_group: the mapper layer's four products (and a partial-tile one) in one launch, beta 1 and 0 mixed,
    bitwise what each gives alone on the unsplit K-outer split-role kernel."""
    items, refs = [], []
    for i, (N, K, rows) in enumerate(SHAPES[:5]):
        dY, X, G = _operands(dev, N, K, 3200 if i < 4 else rows, 20 + i)
        beta = 0.0 if i == 1 else 1.0
        C, Cr = G.clone(), G.clone()
        ops.gemm(dY, X, Cr, beta=beta, M=N, N=K, K=dY.shape[0], trans_ab=True, split_k=1, roles=1)
        items.append((dY, X, C, N, K, dY.shape[0], beta))
        refs.append(Cr)
    ops.gemm_group(items)
    torch.cuda.synchronize()
    for i, (it, Cr) in enumerate(zip(items, refs)):
        _assert_same(f"product {i}", it[2], Cr)


def test_gemm_group_rejects_epilogue_operands(dev):
    from icap import _lib as L

    dY, X, G = _operands(dev, 256, 128, 64, 40)
    arr = (L.GemmArgs * 1)()
    a = arr[0]
    a.trans_ab, a.M, a.N, a.K = 1, 256, 128, 64
    a.in_dtype, a.c_dtype = L.BF16, L.F32
    a.A, a.lda, a.B, a.ldb, a.C, a.ldc = dY.data_ptr(), 256, X.data_ptr(), 128, G.data_ptr(), 128
    a.alpha, a.beta, a.split_k = 1.0, 1.0, 1
    a.bias = G.data_ptr()
    with pytest.raises(L.IcapError):
        ops.call("icap_gemm_group", arr, 1, ops._stream())


def test_gemm_group_bias_gradient_ones_column(dev):
    """The bias gradients of the fused mapper schedule: db[N] (+)= dY[rows, N]^T . ones[rows] as K-outer products
    against a ones column (N = 1, ldb = 8, C viewed [N, 1]) in the same launch as a weight product; equal to the fp64
    column sums to fp32 accumulation order (rel 1e-5 of sum |dY|)."""
    rows = 3200
    ones = torch.ones((rows, 8), device=dev, dtype=torch.bfloat16)
    dY, X, G = _operands(dev, 2304, 768, rows, 50)
    dY2 = rnd((rows, 768), dev, scale=0.3, seed=55)
    db1 = rnd((2304,), dev, torch.float32, 1.0, seed=56)
    db2 = torch.zeros(768, device=dev)
    r1 = db1.double() + dY.double().sum(0)
    r2 = dY2.double().sum(0)
    ops.gemm_group([(dY, X, G, 2304, 768, rows, 1.0), (dY, ones, db1.view(-1, 1), 2304, 1, rows, 1.0),
                    (dY2, ones, db2.view(-1, 1), 768, 1, rows, 0.0)])
    torch.cuda.synchronize()
    for got, ref, src in ((db1, r1, dY), (db2, r2, dY2)):
        err = ((got.double() - ref).abs() / (src.double().abs().sum(0) + 1e-30)).max().item()
        assert err < 1e-5, err
