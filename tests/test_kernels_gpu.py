"""Kernel-level numerics of libicap_hip.so vs plain PyTorch fp64 references of the same op.

Each reference here is the textbook definition of the op the reference model reaches
through HF transformers / torch (cited per test); tolerances are written per test.
"""

import math

import pytest
import torch

from icap import _lib as L
from icap import ops

pytestmark = pytest.mark.gpu


def rnd(shape, dev, dtype=torch.float32, scale=1.0, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.randn(shape, generator=g) * scale).to(device=dev, dtype=dtype)


def rel_err(a, b):
    a = a.double()
    b = b.double()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("M,N,K", [(128, 128, 64), (130, 200, 72), (520, 2304, 768), (7, 50304, 768), (333, 96, 3072)])
def test_gemm_plain(dev, dtype, M, N, K):
    A = rnd((M, K), dev, dtype, seed=1)
    B = rnd((N, K), dev, dtype, seed=2)
    C = torch.empty((M, N), device=dev, dtype=torch.float32)
    ops.gemm(A, B, C)
    ref = A.double() @ B.double().t()
    # fp32 inputs: exact-fp32 MFMA chain; bf16 inputs: exact products, fp32 accumulation
    tol = 2e-6 if dtype == torch.float32 else 1e-5
    err = ((C.double() - ref).abs() / (A.double().abs() @ B.double().abs().t())).max().item()
    assert err < tol, err


def test_gemm_strided_and_beta(dev):
    A_full = rnd((64, 200), dev, seed=3)
    B_full = rnd((96, 300), dev, seed=4)
    A = A_full[:, 8:8 + 128]
    B = B_full[:, 0:128]
    C0 = rnd((64, 96), dev, seed=5)
    C = C0.clone()
    ops.gemm(A, B, C, alpha=0.5, beta=1.0)
    ref = C0.double() + 0.5 * (A.double() @ B.double().t())
    assert rel_err(C, ref) < 1e-5


@pytest.mark.parametrize("act", [L.ACT_GELU_NEW, L.ACT_RELU, L.ACT_QUICK_GELU, L.ACT_TANH])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_gemm_epilogues(dev, act, dtype):
    M, N, K = 200, 384, 256
    A = rnd((M, K), dev, dtype, 0.1, seed=6)
    B = rnd((N, K), dev, dtype, 0.1, seed=7)
    bias = rnd((N,), dev, scale=0.5, seed=8)
    resid = rnd((M, N), dev, dtype, seed=9)
    C = torch.empty((M, N), device=dev, dtype=dtype)
    aux = torch.empty((M, N), device=dev, dtype=dtype)
    ops.gemm(A, B, C, bias=bias, act=act, aux=aux, resid=resid)
    z = A.double() @ B.double().t() + bias.double()
    if act == L.ACT_GELU_NEW:  # HF/activations.py:59-66
        y = 0.5 * z * (1 + torch.tanh(math.sqrt(2 / math.pi) * (z + 0.044715 * z ** 3)))
        dy = None
    elif act == L.ACT_RELU:
        y = torch.relu(z)
    elif act == L.ACT_QUICK_GELU:  # HF/activations.py:117-123
        y = z * torch.sigmoid(1.702 * z)
    else:
        y = torch.tanh(z)
    ref = y + resid.double()
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    assert rel_err(C, ref) < tol
    aux_ref = y if act == L.ACT_TANH else z
    assert rel_err(aux, aux_ref) < tol
    # backward epilogue: dZ = (G @ W) * act'(aux)
    G = rnd((M, 64), dev, dtype, seed=10)
    W = rnd((N, 64), dev, dtype, seed=11)
    dZ = torch.empty((M, N), device=dev, dtype=dtype)
    ops.gemm(G, W, dZ, dact=act, dact_src=aux)
    zz = aux.double()
    if act == L.ACT_GELU_NEW:
        zr = zz.clone().requires_grad_(True)
        yy = 0.5 * zr * (1 + torch.tanh(math.sqrt(2 / math.pi) * (zr + 0.044715 * zr ** 3)))
        d = torch.autograd.grad(yy.sum(), zr)[0]
    elif act == L.ACT_RELU:
        d = (zz > 0).double()
    elif act == L.ACT_QUICK_GELU:
        zr = zz.clone().requires_grad_(True)
        d = torch.autograd.grad((zr * torch.sigmoid(1.702 * zr)).sum(), zr)[0]
    else:
        d = 1 - zz * zz
    ref = (G.double() @ W.double().t()) * d
    assert rel_err(dZ, ref) < (1e-5 if dtype == torch.float32 else 1e-2)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_gemm_split_k_matches_single_pass(dev, dtype):
    """split-K (fp32 partial slabs + reduce/epilogue kernel) == one-pass epilogue: same dropout mask, same
    aux/activation/residual, beta accumulation, and the backward dact epilogue."""
    M, N, K = 128, 768, 1024
    A = rnd((M, K), dev, dtype, 0.1, seed=31)
    B = rnd((N, K), dev, dtype, 0.1, seed=32)
    bias = rnd((N,), dev, scale=0.5, seed=33)
    resid = rnd((M, N), dev, dtype, seed=34)
    drop = ops.Dropout(0.1, seed=77, offset=5)
    outs = {}
    for sk in (1, 3, 0):
        C = torch.empty((M, N), device=dev, dtype=dtype)
        aux = torch.empty((M, N), device=dev, dtype=dtype)
        ops.gemm(A, B, C, bias=bias, act=L.ACT_GELU_NEW, aux=aux, resid=resid, drop=drop, split_k=sk)
        dZ = torch.empty((M, N), device=dev, dtype=dtype)
        ops.gemm(A, B, dZ, dact=L.ACT_GELU_NEW, dact_src=aux, drop=drop, alpha=0.5, split_k=sk)
        Cb = rnd((M, N), dev, seed=35)
        ops.gemm(A, B, Cb, alpha=2.0, beta=1.0, split_k=sk)
        outs[sk] = (C, aux, dZ, Cb)
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    for sk in (3, 0):
        for x, y in zip(outs[sk], outs[1]):
            assert rel_err(x, y) < tol
        assert torch.equal(outs[sk][0] == resid, outs[1][0] == resid)  # identical dropout positions
    z = A.double() @ B.double().t()
    assert rel_err(outs[3][1], z + bias.double()) < tol


@pytest.mark.parametrize("M,N,K", [(768, 3072, 3200), (200, 72, 100), (130, 200, 64), (768, 768, 128), (3, 5, 7)])
@pytest.mark.parametrize("cdt", [torch.float32, torch.bfloat16])
def test_gemm_trans_ab(dev, M, N, K, cdt):
    """K-outer operands (dW = dY^T X over token rows): out = beta*out + alpha * A[K,M]^T B[K,N], strided A."""
    lda = (M + 7) // 8 * 8 + 8
    A = rnd((K, lda), dev, torch.bfloat16, seed=41)[:, :M]
    B = rnd((K, N + (8 - N % 8) % 8), dev, torch.bfloat16, seed=42)[:, :N]
    C0 = rnd((M, N), dev, cdt, seed=43)
    beta = 1.0 if cdt == torch.float32 else 0.0
    ref = beta * C0.double() + 0.5 * (A.double().t() @ B.double())
    scale = (A.double().abs().t() @ B.double().abs()) * 0.5 + beta * C0.double().abs() + 1e-30
    for sk in ((0, 3) if cdt == torch.float32 else (0,)):
        C = C0.clone()
        ops.gemm(A, B, C, alpha=0.5, beta=beta, trans_ab=True, split_k=sk)
        err = ((C.double() - ref).abs() / scale).max().item()
        assert err < (1e-5 if cdt == torch.float32 else 8e-3), (sk, err)


@pytest.mark.parametrize("transpose_out", [False, True])
def test_dw_helper_kout_matches_transpose_path(dev, transpose_out):
    """mapper DWHelper.dW (src/train.py:145 weight grads): the bf16 K-outer product equals dY^T X (fp64) and
    the transpose-then-NT path it replaced, accumulating into the existing fp32 grad."""
    from icap.mapper import DWHelper, _kout_ok

    M, N, K = 3200, 768, 3072
    dY = rnd((M, N), dev, torch.bfloat16, seed=51)
    X = rnd((M, K), dev, torch.bfloat16, seed=52)
    shape = (K, N) if transpose_out else (N, K)
    g0 = rnd(shape, dev, seed=53)
    ref = g0.double() + (X.double().t() @ dY.double() if transpose_out else dY.double().t() @ X.double())
    h = DWHelper(torch.bfloat16, dev, max_rows=M, max_cols=K, ln_rows=M, ln_D=N)
    assert _kout_ok(dY) and _kout_ok(X)
    g1 = g0.clone()
    h.dW(dY, X, g1, M=M, transpose_out=transpose_out)
    scale = (X.double().abs().t() @ dY.double().abs() if transpose_out else dY.double().abs().t() @ X.double().abs())
    assert ((g1.double() - ref).abs() / (scale + g0.double().abs())).max().item() < 1e-5
    # the transpose path (fp32 parity mode's route) on the same bf16 operands
    g2 = g0.clone()
    Mp = (M + 63) // 64 * 64
    a = h._t(h.tA, dY, M, N, Mp)
    b = h._t(h.tB, X, M, K, Mp)
    if transpose_out:
        ops.gemm(b, a, g2, beta=1.0, M=K, N=N, K=Mp)
    else:
        ops.gemm(a, b, g2, beta=1.0, M=N, N=K, K=Mp)
    assert ((g1.double() - g2.double()).abs() / (scale + g0.double().abs())).max().item() < 1e-5


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("M,N", [(128, 2304), (7, 3072), (128, 40)])
def test_gemm_fused_layernorm(dev, dtype, M, N):
    """decode-step ln_1 / ln_2 fused into the skinny GEMM == layernorm_fwd then GEMM (modeling_gpt2.py:281,301)."""
    K = 768
    x = rnd((M, K), dev, dtype, 2.0, seed=61) + 0.3
    g = rnd((K,), dev, seed=62) * 0.2 + 1
    b = rnd((K,), dev, seed=63) * 0.1
    W = rnd((N, K), dev, dtype, 0.05, seed=64)
    bias = rnd((N,), dev, scale=0.1, seed=65)
    y = torch.empty((M, K), device=dev, dtype=dtype)
    ops.layernorm_fwd(x, g, b, 1e-5, y, None, None)
    ref = torch.empty((M, N), device=dev, dtype=dtype)
    ops.gemm(y, W, ref, bias=bias, act=L.ACT_GELU_NEW)
    out = torch.empty_like(ref)
    ops.gemm(x, W, out, bias=bias, act=L.ACT_GELU_NEW, ln=(g, b, 1e-5))
    # fp32: the same arithmetic up to the stats' summation order; bf16: plus an occasional 1-ulp rounding flip
    # of a normalised input
    tol = 1e-5 if dtype == torch.float32 else 2e-2
    assert rel_err(out, ref) < tol


@pytest.mark.parametrize("offset", [0.0, 300.0, 3000.0])
def test_gemm_fused_layernorm_large_mean(dev, offset):
    """the bf16 fused LN statistics (one pass over the MFMA fragments) on rows whose mean is far larger
    than their spread. The shifted sums (x - x0) keep the variance exact where E[x^2] - mean^2 in fp32 would cancel;
    fused and unfused LN-GEMM both stay within bf16 rounding of an fp64 LN-GEMM of the same bf16 inputs."""
    M, N, K = 128, 2304, 768
    x = (rnd((M, K), dev, scale=8.0, seed=66) + offset).to(torch.bfloat16)
    g = rnd((K,), dev, seed=67) * 0.2 + 1
    b = rnd((K,), dev, seed=68) * 0.1
    W = rnd((N, K), dev, torch.bfloat16, 0.05, seed=69)
    xd = x.double()
    mu = xd.mean(1, keepdim=True)
    var = ((xd - mu) ** 2).mean(1, keepdim=True)
    yref = ((xd - mu) / torch.sqrt(var + 1e-5) * g.double() + b.double())
    ref = yref @ W.double().t()
    y = torch.empty((M, K), device=dev, dtype=torch.bfloat16)
    ops.layernorm_fwd(x, g, b, 1e-5, y, None, None)
    unf = torch.empty((M, N), device=dev, dtype=torch.float32)
    ops.gemm(y, W, unf)
    out = torch.empty((M, N), device=dev, dtype=torch.float32)
    ops.gemm(x, W, out, ln=(g, b, 1e-5))
    e_fused, e_unf = rel_err(out, ref), rel_err(unf, ref)
    print(f"offset {offset}: fused {e_fused:.3g} unfused {e_unf:.3g}")
    assert e_fused < 1.5e-2 and e_unf < 1.5e-2
    assert e_fused < 2 * e_unf + 1e-3  # no worse than the two-pass LayerNorm kernel's bf16 rounding


@pytest.mark.parametrize("patch", [32, 14])
def test_im2col_patches(dev, patch):
    """Conv2d(stride=patch) patch rows (HF/models/clip/modeling_clip.py:148-154), incl. ViT-L/14's p = 14
    (588 values per patch, rows padded to 592 with zeros)."""
    B, C, HW = 2, 3, 224
    px = rnd((B, C, HW, HW), dev, seed=71)
    G, K = HW // patch, C * patch * patch
    Kp = (K + 7) // 8 * 8
    out = torch.full((B * G * G, Kp), 7.0, device=dev)
    ops.im2col_patches(px, out, patch)
    ref = px.unfold(2, patch, patch).unfold(3, patch, patch)  # [B, C, G, G, p, p]
    ref = ref.permute(0, 2, 3, 1, 4, 5).reshape(B * G * G, K)
    assert torch.equal(out[:, :K], ref)
    assert torch.all(out[:, K:] == 0)


@pytest.mark.parametrize("B,patch,NP,N,pos,bias", [(3, 32, 1, 768, True, False),    # CLIP ViT-B/32
                                                   (2, 16, 5, 1024, False, True),   # DINOv3: CLS + 4 registers
                                                   (2, 16, 1, 768, True, True),     # ViT-B/16
                                                   (2, 14, 1, 1024, True, False),   # CLIP ViT-L/14 (p % 8 != 0)
                                                   (1, 32, 1, 200, True, True)])   # ragged N (a partial column tile)
def test_patch_embed_matches_conv(dev, B, patch, NP, N, pos, bias):
    """icap_patch_embed (round 5: the patch GEMM gathers its pixel runs itself) vs the fp64 Conv2d of the same
    bf16-rounded pixels and weights (HF modeling_clip.py:148-154,209-217; modeling_dinov3_vit.py:75-92) with the
    prefix rows, bias and positions added: each output is the fp32 sum rounded once to bf16, so |err| <= |ref| 2^-8
    (+ the accumulation-order term). And against the im2col + tile GEMM + vit_embed launches it replaces."""
    C, HW = 3, 224
    G = HW // patch
    G2, K = G * G, C * patch * patch
    Kp = (K + 7) // 8 * 8
    S = NP + G2
    px = rnd((B, C, HW, HW), dev, seed=81)
    w32 = rnd((N, C, patch, patch), dev, scale=0.02, seed=82)
    wp = torch.nn.functional.pad(w32.reshape(N, K), (0, Kp - K)).to(torch.bfloat16).contiguous()
    pre = rnd((NP, N), dev, scale=0.5, seed=83)
    pe = rnd((S, N), dev, scale=0.1, seed=84) if pos else None
    b = rnd((N,), dev, scale=0.02, seed=85) if bias else None
    out = torch.full((B * S, N), float("nan"), device=dev, dtype=torch.bfloat16)
    ops.patch_embed(px, wp, out, patch=patch, prefix=pre, pos=pe, bias=b)
    torch.cuda.synchronize()
    px16 = px.to(torch.bfloat16).double().cpu()
    w16 = wp[:, :K].double().cpu().reshape(N, C, patch, patch)
    conv = torch.nn.functional.conv2d(px16, w16, stride=patch).flatten(2).transpose(1, 2)  # [B, G2, N]
    if b is not None:
        conv = conv + b.double().cpu()
    ref = torch.cat([pre.double().cpu()[None].expand(B, NP, N), conv], 1)
    if pe is not None:
        ref = ref + pe.double().cpu()[None]
    got = out.double().cpu().reshape(B, S, N)
    err = (got - ref).abs()
    assert torch.all(err <= ref.abs() * 2 ** -8 + 1e-4), float((err - ref.abs() * 2 ** -8).max())
    # the prefix rows: prefix (+ pos) rounded once, exactly
    assert torch.equal(out.reshape(B, S, N)[:, :NP].cpu(),
                       (pre + (pe[:NP] if pe is not None else 0)).to(torch.bfloat16).cpu()[None].expand(B, NP, N))
    # the launches it replaces (im2col + GEMM + token assembly): within two bf16 roundings
    patches = torch.empty((B * G2, Kp), device=dev, dtype=torch.bfloat16)
    ops.im2col_patches(px, patches, patch)
    pe_rows = torch.empty((B * G2, N), device=dev, dtype=torch.bfloat16)
    ops.gemm(patches, wp, pe_rows, bias=b)
    old = torch.empty((B * S, N), device=dev, dtype=torch.bfloat16)
    if pe is not None and NP == 1:
        ops.vit_embed(pe_rows, pre.reshape(-1), pe, old, B, G2, N)
    else:
        ops.prefix_embed(pe_rows, pre, old, B, G2, N, pos=pe)
    torch.cuda.synchronize()
    # (the old path rounds the patch product to bf16 before adding the positions: where they cancel, its own error
    # is |patch| 2^-8, not |result| 2^-8 — so this bound is on the largest magnitude)
    d = (out.double() - old.double()).abs()
    assert float(d.max()) <= float(old.double().abs().max()) * 2 ** -7


def test_gemm_dropout_statistics(dev):
    M, N, K = 512, 512, 64
    A = torch.ones((M, K), device=dev)
    B = torch.full((N, K), 1.0 / K, device=dev)
    C = torch.empty((M, N), device=dev)
    ops.gemm(A, B, C, drop=ops.Dropout(0.1, seed=1234))
    kept = (C != 0).double().mean().item()
    assert abs(kept - 0.9) < 0.005
    assert torch.allclose(C[C != 0], torch.full_like(C[C != 0], 1 / 0.9), rtol=1e-6)
    C2 = torch.empty_like(C)
    ops.gemm(A, B, C2, drop=ops.Dropout(0.1, seed=1234))
    assert torch.equal(C, C2)  # deterministic mask


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_layernorm(dev, dtype):
    rows, D = 333, 768
    x = rnd((rows, D), dev, dtype, 2.0, seed=12) + 0.5
    g = rnd((D,), dev, seed=13) * 0.2 + 1
    b = rnd((D,), dev, seed=14) * 0.1
    y = torch.empty_like(x)
    mean = torch.empty(rows, device=dev)
    rstd = torch.empty(rows, device=dev)
    ops.layernorm_fwd(x, g, b, 1e-5, y, mean, rstd)
    xr = x.double().requires_grad_(True)
    gr = g.double().requires_grad_(True)
    br = b.double().requires_grad_(True)
    yr = torch.nn.functional.layer_norm(xr, (D,), gr, br, 1e-5)
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    assert rel_err(y, yr) < tol
    dy = rnd((rows, D), dev, dtype, seed=15)
    dres = rnd((rows, D), dev, dtype, seed=16)
    dx = torch.empty_like(x)
    dg = torch.zeros(D, device=dev)
    db = torch.zeros(D, device=dev)
    ws = torch.empty(ops.layernorm_bwd_workspace(rows, D), dtype=torch.uint8, device=dev)
    ops.layernorm_bwd(x, g, mean, rstd, dy, dx, dres=dres, dgamma=dg, dbeta=db, workspace=ws)
    gx, gg, gb = torch.autograd.grad(yr, (xr, gr, br), dy.double())
    assert rel_err(dx, gx + dres.double()) < (1e-5 if dtype == torch.float32 else 2e-2)
    assert rel_err(dg, gg) < (1e-5 if dtype == torch.float32 else 1e-2)
    assert rel_err(db, gb) < 1e-5


def ref_attention(q, k, v, scale, causal, key_mask):
    # q,k,v: [B,H,S,hd] float64; mask rule HF/masking_utils.py:76-80 (causal) & padding
    s = (q @ k.transpose(-1, -2)) * scale
    S = q.shape[-2]
    allowed = torch.ones((S, S), dtype=torch.bool, device=q.device)
    if causal:
        allowed = torch.tril(allowed)
    allowed = allowed[None, None]
    if key_mask is not None:
        allowed = allowed & key_mask.bool()[:, None, None, :]
    s = s.masked_fill(~allowed, float("-inf"))
    p = torch.softmax(s, -1)
    return p @ v


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B,S,H,hd,causal,masked", [(3, 65, 12, 64, True, True), (2, 25, 8, 96, False, False),
                                                    (2, 50, 12, 64, False, False), (2, 25, 8, 128, False, False),
                                                    (2, 60, 4, 128, True, True)])
def test_attention(dev, dtype, B, S, H, hd, causal, masked):
    D = H * hd
    qkv = rnd((B * S, 3 * D), dev, dtype, seed=20)
    key_mask = None
    if masked:
        km = torch.ones((B, S), dtype=torch.int32)
        km[0, 30:] = 0
        km[1, 40:] = 0
        key_mask = km.to(dev)
    out = torch.empty((B * S, D), device=dev, dtype=dtype)
    lse = torch.empty(B * H * S, device=dev)
    scale = 1.0 / math.sqrt(hd)
    ops.attention_fwd(qkv, out, B=B, S=S, H=H, hd=hd, scale=scale, causal=causal, key_mask=key_mask, lse=lse)
    x = qkv.double().view(B, S, 3, H, hd).permute(2, 0, 3, 1, 4).requires_grad_(True)
    o = ref_attention(x[0], x[1], x[2], scale, causal, key_mask)
    o2 = o.permute(0, 2, 1, 3).reshape(B * S, D)
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    assert rel_err(out, o2) < tol
    dout = rnd((B * S, D), dev, dtype, seed=21)
    (gx,) = torch.autograd.grad(o2, x, dout.double())
    g = gx.permute(1, 3, 0, 2, 4).reshape(B * S, 3 * D)
    # without O (transposing backward) and with O (delta = rowsum(dO o O), transpose-free MFMA backward)
    for o_arg in (None, out):
        dqkv = torch.empty_like(qkv)
        ops.attention_bwd(qkv, dout, lse, dqkv, B=B, S=S, H=H, hd=hd, scale=scale, causal=causal,
                          key_mask=key_mask, out=o_arg)
        assert rel_err(dqkv, g) < (1e-5 if dtype == torch.float32 else 2e-2)


@pytest.mark.parametrize("B,S,H,hd,causal,masked", [(2, 257, 16, 64, False, False), (2, 200, 4, 64, True, True),
                                                    (1, 300, 4, 96, False, False)])
def test_attention_long_sequence_forward(dev, B, S, H, hd, causal, masked):
    """bf16 forward past 8 key tiles (ViT-L/14 at 224 px: S = 257, BASELINE configs[3]): online-softmax MFMA
    kernel vs the fp64 definition; lse checked against the reference logsumexp."""
    D = H * hd
    qkv = rnd((B * S, 3 * D), dev, torch.bfloat16, seed=22)
    key_mask = None
    if masked:
        km = torch.ones((B, S), dtype=torch.int32)
        km[0, 150:] = 0
        key_mask = km.to(dev)
    out = torch.empty((B * S, D), device=dev, dtype=torch.bfloat16)
    lse = torch.empty(B * H * S, device=dev)
    scale = 1.0 / math.sqrt(hd)
    ops.attention_fwd(qkv, out, B=B, S=S, H=H, hd=hd, scale=scale, causal=causal, key_mask=key_mask, lse=lse)
    x = qkv.double().view(B, S, 3, H, hd).permute(2, 0, 3, 1, 4)
    o = ref_attention(x[0], x[1], x[2], scale, causal, key_mask)
    assert rel_err(out, o.permute(0, 2, 1, 3).reshape(B * S, D)) < 1e-2
    s_ = torch.einsum("bhqd,bhkd->bhqk", x[0], x[1]) * scale
    if causal:
        s_ = s_.masked_fill(torch.ones(S, S, dtype=torch.bool, device=dev).triu(1), float("-inf"))
    if key_mask is not None:
        s_ = s_.masked_fill(key_mask[:, None, None, :] == 0, float("-inf"))
    ref_lse = torch.logsumexp(s_, dim=-1).reshape(-1)
    assert (lse.double() - ref_lse).abs().max().item() < 2e-2


@pytest.mark.parametrize("B,S,H,hd,causal", [(3, 65, 12, 64, True), (2, 25, 8, 96, False), (2, 128, 4, 64, True)])
def test_attention_bwd_dropout_paths_agree(dev, B, S, H, hd, causal):
    """bf16 backward with attention dropout: the O-based (v2) and the transposing (v1) backward see the same
    counter-based mask (index (b*H+h)*S*S + q*S + k) and agree."""
    D = H * hd
    qkv = rnd((B * S, 3 * D), dev, torch.bfloat16, seed=23)
    out = torch.empty((B * S, D), device=dev, dtype=torch.bfloat16)
    lse = torch.empty(B * H * S, device=dev)
    drop = ops.Dropout(0.1, seed=99, offset=7)
    scale = 1.0 / math.sqrt(hd)
    ops.attention_fwd(qkv, out, B=B, S=S, H=H, hd=hd, scale=scale, causal=causal, lse=lse, drop=drop)
    dout = rnd((B * S, D), dev, torch.bfloat16, seed=24)
    d1, d2 = torch.empty_like(qkv), torch.empty_like(qkv)
    ops.attention_bwd(qkv, dout, lse, d1, B=B, S=S, H=H, hd=hd, scale=scale, causal=causal, drop=drop)
    ops.attention_bwd(qkv, dout, lse, d2, B=B, S=S, H=H, hd=hd, scale=scale, causal=causal, drop=drop, out=out)
    assert rel_err(d2, d1) < 2e-2


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_attention_decode_matches_full(dev, dtype):
    B, H, hd, T = 4, 12, 64, 20
    D = H * hd
    qkv = rnd((T * B, 3 * D), dev, dtype, seed=22)  # position-major rows t*B+b
    out = torch.empty((B, D), device=dev, dtype=dtype)
    pos = T - 1
    ops.attention_decode(qkv, out, B=B, H=H, hd=hd, pos=pos, scale=0.125)
    x = qkv.double().view(T, B, 3, H, hd).permute(2, 1, 3, 0, 4)  # [3,B,H,T,hd]
    o = ref_attention(x[0], x[1], x[2], 0.125, True, None)[:, :, pos]  # [B,H,hd]
    assert rel_err(out, o.reshape(B, D)) < (1e-5 if dtype == torch.float32 else 1e-2)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_cross_entropy(dev, dtype):
    rows, V, ld = 130, 50257, 50304
    logits = torch.zeros((rows, ld), device=dev, dtype=dtype)
    logits[:, :V] = rnd((rows, V), dev, dtype, 3.0, seed=30)
    g = torch.Generator().manual_seed(31)
    labels = torch.randint(0, V, (rows,), generator=g, dtype=torch.int32)
    labels[::3] = -100
    labels = labels.to(dev)
    nvalid = (labels != -100).sum().to(torch.int32).reshape(1)
    loss = torch.empty(1, device=dev)
    dl = torch.empty_like(logits)
    ws = torch.empty(ops.cross_entropy_workspace(rows), dtype=torch.uint8, device=dev)
    ops.cross_entropy(logits, V, labels, nvalid, loss, dl, ws)
    x = logits[:, :V].double().requires_grad_(True)
    ref = torch.nn.functional.cross_entropy(x, labels.long(), ignore_index=-100)  # HF/loss/loss_utils.py:32-46
    (gx,) = torch.autograd.grad(ref, x)
    assert abs(loss.item() - ref.item()) < 1e-5 * max(1, abs(ref.item()))
    assert rel_err(dl[:, :V], gx) < (1e-4 if dtype == torch.float32 else 1e-2)
    assert torch.all(dl[:, V:] == 0)


def test_adamw_matches_torch(dev):
    n = 100003
    p0 = rnd((n,), dev, seed=40)
    steps = 4
    grads = [rnd((n,), dev, scale=0.01 * (k + 1), seed=41 + k) for k in range(steps)]
    # reference: clip_grad_norm_ + AdamW + linear schedule (src/train.py:94-103,150-156)
    pr = torch.nn.Parameter(p0.clone())
    opt = torch.optim.AdamW([pr], lr=1e-3, weight_decay=0.01)
    total = 10
    sched = torch.optim.lr_scheduler.LambdaLR(opt, lambda s: max(0.0, (total - s) / total))
    P = p0.clone()
    M1 = torch.zeros_like(P)
    M2 = torch.zeros_like(P)
    st = torch.zeros(16, dtype=torch.float32, device=dev)
    ws = torch.empty(ops.adamw_workspace(n), dtype=torch.uint8, device=dev)
    out16 = torch.empty(n, dtype=torch.bfloat16, device=dev)
    for k in range(steps):
        pr.grad = grads[k].clone()
        torch.nn.utils.clip_grad_norm_([pr], max_norm=1.0)
        opt.step()
        sched.step()
        ops.adamw_step(P, grads[k].clone(), M1, M2, st, ws, lr=1e-3, weight_decay=0.01, max_norm=1.0,
                       num_training_steps=total, bf16_out=out16)
    assert rel_err(P, pr.detach()) < 1e-6
    assert torch.equal(out16, P.to(torch.bfloat16))
    assert st[:2].view(torch.int64).item() == steps


def test_transpose_colsum_dropout(dev):
    x = rnd((77, 130), dev, seed=50)
    t = torch.full((130, 96), 7.0, device=dev)
    ops.transpose(x, t, rows_pad=96)
    assert torch.equal(t[:, :77], x.t())
    assert torch.all(t[:, 77:] == 0)
    cs = torch.ones(130, device=dev)
    ws = torch.empty(ops.colsum_workspace(77, 130), dtype=torch.uint8, device=dev)
    ops.colsum(x, cs, ws, accumulate=True)
    assert rel_err(cs, 1 + x.double().sum(0)) < 1e-6
    y = torch.empty_like(x)
    ctr = torch.zeros(1, dtype=torch.int64, device=dev)
    ops.dropout_apply(x, y, ops.Dropout(0.5, 99, 0, ctr))
    y2 = torch.empty_like(x)
    ops.counter_increment(ctr)
    ops.dropout_apply(x, y2, ops.Dropout(0.5, 99, 0, ctr))
    assert not torch.equal(y, y2)
    m = y != 0
    assert torch.allclose(y[m], 2 * x[m])


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_greedy_next_argmax(dev, dtype):
    """icap_greedy_next == torch.argmax (NaN first, ties -> smallest index) + EOS/forced bookkeeping and the
    fused next-token embedding (src/models.py:320-330 greedy loop)."""
    B, V, ld, D, eos = 6, 50257, 50304, 64, 50256
    g = torch.Generator().manual_seed(60)
    lg = torch.randn((B, ld), generator=g).to(dtype)
    lg[1, 1000] = lg[1, 40000] = 100.0        # tie -> 1000
    lg[2, 50250] = 1e4                         # winner in the unaligned tail
    lg[3, 7] = float("nan")                    # NaN wins
    lg[4, V:] = 1e9                            # padding columns must be ignored
    finished = torch.tensor([0, 0, 0, 0, 0, 1], dtype=torch.int32)
    tokens = torch.zeros((B, 4), dtype=torch.int64)
    wte = torch.randn((V, D), generator=g).to(dtype)
    wpe = torch.randn((10, D), generator=g).to(dtype)
    x = torch.empty((B, D), dtype=dtype)
    lgd, fd, td, xd = lg.to(dev), finished.to(dev), tokens.to(dev), x.to(dev)
    ops.greedy_next(lgd, V, eos, fd, td, 2, wte.to(dev), wpe.to(dev), 5, D, xd)
    ref = torch.argmax(lg[:, :V].float(), dim=-1)
    ref[5] = eos
    assert td[:, 2].cpu().tolist() == ref.tolist()
    assert td[:, 2].cpu()[1].item() == 1000 and td[:, 2].cpu()[3].item() == 7
    assert fd.cpu().tolist() == [int(t == eos) or f for t, f in zip(ref.tolist(), finished.tolist())]
    xr = (wte.float()[ref] + wpe.float()[5]).to(dtype)
    assert torch.equal(xd.cpu(), xr)


@pytest.mark.parametrize("rows,cols,rows_pad", [(3200, 768, 3200), (77, 136, 128), (130, 96, 192)])
def test_transpose_colsum_bf16_vector_paths(dev, rows, cols, rows_pad):
    """16-byte transpose / 4-column colsum fast paths (dW operand staging of the mapper, bias grads)."""
    x = rnd((rows, cols), dev, torch.bfloat16, seed=51)
    t = torch.full((cols, rows_pad), 3.0, device=dev, dtype=torch.bfloat16)
    ops.transpose(x, t, rows_pad=rows_pad)
    assert torch.equal(t[:, :rows], x.t())
    assert torch.all(t[:, rows:] == 0)
    cs = torch.zeros(cols, device=dev)
    ws = torch.empty(ops.colsum_workspace(rows, cols), dtype=torch.uint8, device=dev)
    ops.colsum(x, cs, ws, accumulate=False)
    assert rel_err(cs, x.double().sum(0)) < 1e-5


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_colsum_batch_bitwise(dev, dtype):
    """icap_colsum_batch (the mapper's four bias gradients per layer in two launches) stores, per item, exactly
    what icap_colsum gives for it (same chunking and summation order), accumulating and not; items the batched
    kernel cannot take (N % 4 != 0, here 130) go through icap_colsum inside ops.colsum_batch."""
    M = 3200
    widths = [768, 3072, 768, 2304, 132, 130]
    src = [rnd((M, n + 4), dev, dtype, seed=60 + i)[:, 2:2 + n] if i == 4 else rnd((M, n), dev, dtype, seed=60 + i)
           for i, n in enumerate(widths)]  # item 4: strided rows, src offset by 2 elements (misaligned -> fallback)
    ws = torch.empty(ops.colsum_workspace(M, sum(widths)), dtype=torch.uint8, device=dev)
    for acc in (False, True):
        init = [torch.randn(n, generator=torch.Generator().manual_seed(70 + i)).to(dev) for i, n in enumerate(widths)]
        want = [t.clone() for t in init]
        got = [t.clone() for t in init]
        for s, o in zip(src, want):
            ops.colsum(s, o, ws, accumulate=acc)
        ops.colsum_batch([(s, o, None) for s, o in zip(src, got)], M, ws, accumulate=acc)
        for i, (a, b) in enumerate(zip(want, got)):
            assert torch.equal(a, b), (acc, i)
        assert rel_err(got[1] - (init[1] if acc else 0), src[1].double().sum(0)) < 1e-5


def test_caption_prep_target_compaction(dev):
    """row_slot / labels_compact / n_valid vs a host restatement of the shifted-label rule
    (HF/loss/loss_utils.py:49-71 shift, src/models.py:296-317 prefix labels -100)."""
    B, P, L_ = 37, 15, 50
    g = torch.Generator().manual_seed(40)
    labels = torch.randint(0, 50257, (B, L_), generator=g)
    lens = torch.randint(0, L_ + 1, (B,), generator=g)
    for b in range(B):
        labels[b, lens[b]:] = -100
    mask = (labels != -100).long()
    S = P + L_
    km, ls = torch.empty(B * S, dtype=torch.int32, device=dev), torch.empty(B * S, dtype=torch.int32, device=dev)
    nv = torch.empty(1, dtype=torch.int32, device=dev)
    slot = torch.empty(B * S, dtype=torch.int32, device=dev)
    labc = torch.full((B * L_,), -7, dtype=torch.int32, device=dev)
    ops.caption_prep(B, P, L_, mask.to(dev), labels.to(dev), km, ls, nv, slot, labc)
    full = torch.cat([torch.full((B, P), -100, dtype=torch.long), labels], 1)
    shifted = torch.cat([full[:, 1:], torch.full((B, 1), -100, dtype=torch.long)], 1).reshape(-1)
    valid = shifted != -100
    exp_slot = torch.where(valid, torch.cumsum(valid.int(), 0) - 1, torch.full_like(shifted, -1))
    n = int(valid.sum())
    assert int(nv.item()) == n
    assert torch.equal(ls.cpu().long(), shifted)
    assert torch.equal(slot.cpu().long(), exp_slot)
    assert torch.equal(labc[:n].cpu().long(), shifted[valid])


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_gemm_device_row_count(dev, dtype):
    """m_dev: rows >= *m_dev are neither computed nor stored; rows below equal the full product."""
    for M, N, K, mv in [(700, 1000, 768, 333), (100, 50304, 768, 41), (6400, 768, 512, 1), (256, 256, 64, 0)]:
        A, Bw = rnd((M, K), dev, dtype, seed=41), rnd((N, K), dev, dtype, seed=42)
        ref = torch.empty((M, N), device=dev, dtype=dtype)
        ops.gemm(A, Bw, ref)
        out = torch.full((M, N), 7.0, device=dev, dtype=dtype)
        ops.gemm(A, Bw, out, m_dev=torch.tensor([mv], dtype=torch.int32, device=dev))
        assert torch.equal(out[:mv], ref[:mv]), (M, N, K)
        assert torch.all(out[mv:] == 7.0), (M, N, K)


def test_cross_entropy_rows_dev(dev):
    rows, V, ld, nr = 64, 1000, 1024, 23
    logits = rnd((rows, ld), dev, torch.float32, 2.0, seed=43)
    labels = torch.randint(0, V, (rows,), generator=torch.Generator().manual_seed(44), dtype=torch.int32).to(dev)
    nv = torch.tensor([nr], dtype=torch.int32, device=dev)
    loss = torch.empty(1, device=dev)
    dl = torch.full_like(logits, 5.0)
    ws = torch.empty(ops.cross_entropy_workspace(rows), dtype=torch.uint8, device=dev)
    ops.cross_entropy(logits, V, labels, nv, loss, dl, ws, rows_dev=nv)
    x = logits[:nr, :V].double().requires_grad_(True)
    ref = torch.nn.functional.cross_entropy(x, labels[:nr].long())
    (gx,) = torch.autograd.grad(ref, x)
    assert abs(loss.item() - ref.item()) < 1e-5 * max(1, abs(ref.item()))
    assert rel_err(dl[:nr, :V], gx) < 1e-4
    assert torch.all(dl[nr:] == 5.0)


def test_transpose_batch_equals_single(dev):
    """icap_transpose_batch (one launch over the mapper's transposed weight copies) == per-matrix transposes,
    including an item the tile path cannot take (rows % 64 != 0: falls back inside the library)"""
    shapes = [(2304, 768), (768, 768), (3072, 768), (768, 3072), (130, 96)] * 7  # 35 items: two launches
    srcs = [rnd(sh, dev, torch.bfloat16, seed=70 + i) for i, sh in enumerate(shapes)]
    outs = [torch.full((sh[1], sh[0]), 5.0, device=dev, dtype=torch.bfloat16) for sh in shapes]
    ops.transpose_batch(zip(srcs, outs))
    torch.cuda.synchronize()
    for s_, o in zip(srcs, outs):
        assert torch.equal(o, s_.t())


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_layernorm_param_reduce_batch_bitwise(dev, dtype):
    """The mapper's deferred dgamma / dbeta reduces (layernorm_bwd(defer_params=True) + one ln_param_reduce_batch per
    layer, include/icap.h icap_ln_param_reduce_batch) store bitwise what the per-call reduce stores, in both the
    accumulate and the overwrite form; the dx outputs are untouched by the deferral."""
    rows, D = 3200, 768
    xs = [rnd((rows, D), dev, dtype, seed=60 + i) for i in range(2)]
    dys = [rnd((rows, D), dev, dtype, seed=70 + i) for i in range(2)]
    gms = [rnd((D,), dev, scale=0.5, seed=80 + i) + 1 for i in range(2)]
    stats = []
    for x, g in zip(xs, gms):
        mean, rstd = torch.empty(rows, device=dev), torch.empty(rows, device=dev)
        ops.layernorm_fwd(x, g, torch.zeros(D, device=dev), 1e-5, torch.empty_like(x), mean, rstd)
        stats.append((mean, rstd))
    wsz = ops.layernorm_bwd_workspace(rows, D)
    for acc in (True, False):
        res = {}
        for mode in ("call", "batch"):
            wss = [torch.empty(wsz, dtype=torch.uint8, device=dev) for _ in range(2)]
            dg = [rnd((D,), dev, seed=90 + i) for i in range(2)]
            db = [rnd((D,), dev, seed=95 + i) for i in range(2)]
            dxs = [torch.empty_like(xs[0]) for _ in range(2)]
            for i in range(2):
                ops.layernorm_bwd(xs[i], gms[i], stats[i][0], stats[i][1], dys[i], dxs[i], dgamma=dg[i], dbeta=db[i],
                                  workspace=wss[i], param_accumulate=acc, defer_params=(mode == "batch"))
            if mode == "batch":
                ops.ln_param_reduce_batch([(wss[i], rows, D, dg[i], db[i], acc) for i in range(2)])
            res[mode] = (dg, db, dxs)
        torch.cuda.synchronize()
        for a, b in zip(res["call"], res["batch"]):
            for u, v in zip(a, b):
                assert torch.equal(u, v)
