"""LayerNorm folded into the decode GEMM's weights (icap_gemm_args.ln_wsum, GPT2Core._fold_ln): the folded launch
against the LayerNorm-fused launch (ln_gamma) and an fp32 torch reference of LN(x) . W^T + b, bf16 and fp32, with
and without the GELU epilogue; and greedy decode with folding on vs off (bf16 token agreement, fp32 identical)."""

import pytest
import torch

from icap import _lib as L
from icap import ops

pytestmark = pytest.mark.gpu


def _fold(w_t32, gamma, beta, bias, dtype):
    """the GPT2Core._fold_ln arithmetic on an [N, K] fp32 weight (HIP GEMMs)"""
    N, K = w_t32.shape
    dg = torch.zeros((K, K), dtype=torch.float32, device=w_t32.device)
    dg.view(-1)[:: K + 1].copy_(gamma)
    wg = torch.empty((N, K), dtype=torch.float32, device=w_t32.device)
    ops.gemm(w_t32, dg, wg, split_k=1)
    wf = wg if dtype == torch.float32 else wg.to(dtype)
    wsum = torch.empty((1, N), dtype=torch.float32, device=w_t32.device)
    ops.gemm(torch.ones((1, K), dtype=dtype, device=w_t32.device), wf, wsum, split_k=1)
    bf = torch.empty((1, N), dtype=torch.float32, device=w_t32.device)
    ops.gemm(beta.reshape(1, K).contiguous(), w_t32, bf, bias=bias, split_k=1)
    return wf, wsum.view(N), bf.view(N)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("M,N,K,act", [(128, 2304, 768, L.ACT_NONE), (128, 3072, 768, L.ACT_GELU_NEW),
                                       (77, 768, 1024, L.ACT_NONE), (128, 5120, 1280, L.ACT_GELU_NEW)])
def test_folded_ln_gemm(dev, dtype, M, N, K, act):
    g = torch.Generator().manual_seed(M + N + K)
    x32 = torch.randn((M, K), generator=g) * 2 + 0.5
    x32[:, 7] += 30.0  # a large-magnitude feature (GPT-2's residual stream has them)
    w = (torch.randn((N, K), generator=g) * 0.05).to(dev)
    gamma = (1 + 0.2 * torch.randn(K, generator=g)).to(dev)
    beta = (0.1 * torch.randn(K, generator=g)).to(dev)
    bias = (0.1 * torch.randn(N, generator=g)).to(dev)
    x = x32.to(dev, dtype)
    eps = 1e-5
    wf, wsum, bf = _fold(w, gamma, beta, bias, dtype)
    out_fold = torch.empty((M, N), device=dev, dtype=dtype)
    ops.gemm(x, wf, out_fold, bias=bf, act=act, ln_fold=(wsum, eps))
    out_ln = torch.empty((M, N), device=dev, dtype=dtype)
    ops.gemm(x, w.to(dtype), out_ln, bias=bias, act=act, ln=(gamma, beta, eps))
    torch.cuda.synchronize()
    xr = torch.nn.functional.layer_norm(x.float(), (K,), gamma, beta, eps)
    ref = xr @ w.t() + bias
    if act == L.ACT_GELU_NEW:
        ref = torch.nn.functional.gelu(ref, approximate="tanh")
    scale = float(ref.abs().max())
    ef = float((out_fold.float() - ref).abs().max()) / scale
    el = float((out_ln.float() - ref).abs().max()) / scale
    tol = 2e-2 if dtype == torch.bfloat16 else 2e-5
    assert ef < tol, (ef, el)
    assert ef < 2.5 * el + (1e-6 if dtype == torch.float32 else 2e-3), (ef, el)  # no worse than the fused form


def test_greedy_fold_vs_fused(dev, monkeypatch):
    """bf16 greedy decode (B=32, 20 tokens) with the folded weights vs the LayerNorm-fused GEMMs"""
    from types import SimpleNamespace

    import icap.gpt2 as G
    from icap import GPT2LMHeadModel, ImageCaptioningModel, TransformerMappingNetwork

    emb = torch.randn((32, 512), generator=torch.Generator().manual_seed(5)).to(dev)
    emb = emb / emb.norm(dim=-1, keepdim=True)
    outs = []
    for fold in (True, False):
        monkeypatch.setattr(G, "LN_FOLD", fold)
        torch.manual_seed(0)
        model = ImageCaptioningModel(TransformerMappingNetwork.random_init(), tokenizer=SimpleNamespace(eos_token_id=50256),
                                     gpt=GPT2LMHeadModel.random_init(), compute_dtype=torch.bfloat16).to(dev)
        outs.append(model.generate(emb, max_length=20, temperature=0.0, early_exit=False).cpu())
        del model
    agree = float((outs[0] == outs[1]).float().mean())
    assert agree >= 0.9, agree
