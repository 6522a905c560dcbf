"""Top-p (nucleus) sampling, SURVEY.md §8a a14 (src/models.py:400-449).

CPU: the fixed-point restatement of the kernel's arithmetic (oracle.topp_sample_fixed) keeps the same token set
as the reference's own torch filter (oracle.topp_filter_reference: sort, cumsum(softmax), shift, scatter) on
every row whose boundary is not within the fixed-point resolution of top_p, and its draws follow the renormalised
kept distribution.
GPU: icap_topp_sample is token-exact against topp_sample_fixed (same seed/step), fp32 and bf16 logits, incl.
heavy ties at the boundary, top_p >= 1, finished rows and the unaligned vocabulary tail.

Tolerance: the kept set equals the reference filter exactly except where the reference's fp32 cumsum at the
boundary rank is within 1e-5 of top_p (fp32 cumsum over 50k terms and the 2^-31 fixed point disagree only there).
The draw itself is not comparable to torch.multinomial's stream (not reproducible across devices); its
distribution is checked with a chi-square bound.
"""

import numpy as np
import pytest
import torch

from oracle import icap_oracle as O

V_GPT2, LD, EOS = 50257, 50304, 50256


def _logits(B, V, seed, scale=3.0, ties=False):
    g = torch.Generator().manual_seed(seed)
    lg = torch.randn((B, V), generator=g) * scale
    if ties:  # coarse grid: many equal logits, incl. at the nucleus boundary
        lg = torch.round(lg * 2.0) / 2.0
    return lg


def _ambiguous(lg, temperature, top_p):
    """Rows whose reference boundary cumsum sits within 1e-5 of top_p."""
    l = lg.double() / temperature
    sl, _ = torch.sort(l, descending=True, stable=True)
    cp = torch.cumsum(torch.softmax(sl, dim=-1), dim=-1)
    return ((cp - top_p).abs() < 1e-5).any(dim=-1)


@pytest.mark.parametrize("temperature,top_p,ties", [(1.0, 0.9, False), (0.7, 0.5, False), (1.3, 0.95, True),
                                                    (1.0, 0.3, True), (0.5, 1.0, False)])
def test_fixed_point_filter_matches_reference_filter(temperature, top_p, ties):
    B, V = 16, 4096
    lg = _logits(B, V, 11, ties=ties)
    ref = O.topp_filter_reference(lg, temperature, top_p)
    _, kept = O.topp_sample_fixed(lg.numpy(), temperature, top_p, seed=5, step=0)
    amb = _ambiguous(lg, temperature, top_p).numpy()
    for b in range(B):
        if not amb[b]:
            assert np.array_equal(kept[b], ref[b].numpy()), b


def test_finished_rows_reference_semantics():
    """Finished rows: the reference zeroes their logits (uniform over V) and the EOS latch overwrites the draw."""
    lg = _logits(3, 512, 3)
    fin = np.array([False, True, False])
    toks, _ = O.topp_sample_fixed(lg.numpy(), 1.0, 0.9, seed=1, step=4, finished=fin, eos=511)
    assert toks[1] == 511
    kept = O.topp_filter_reference(lg, 1.0, 0.9, finished=torch.tensor(fin))
    assert int(kept[1].sum()) == int(np.ceil(0.9 * 512))  # uniform row keeps ceil(top_p * V) tokens


def test_fixed_point_draw_distribution():
    """Draws over many rows of one logit vector follow softmax over the kept set (chi-square, 8 kept tokens)."""
    V, B = 64, 4000
    base = np.full(V, -30.0, dtype=np.float32)
    base[[3, 9, 17, 20, 33, 41, 50, 63]] = [2.0, 1.5, 1.0, 0.8, 0.5, 0.2, 0.0, -0.3]
    toks, kept = O.topp_sample_fixed(np.tile(base, (B, 1)), 1.0, 0.97, seed=7, step=2)
    k = np.nonzero(kept[0])[0]
    p = np.exp(base[k] - base[k].max())
    p /= p.sum()
    obs = np.array([(toks == j).sum() for j in k])
    assert obs.sum() == B
    chi2 = float(((obs - B * p) ** 2 / (B * p)).sum())
    assert chi2 < 30.0, (chi2, obs, B * p)  # dof <= 7: p(chi2 > 30) ~ 1e-4


# ------------------------------------------------------------------------------------------------------ GPU


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("temperature,top_p,ties", [(1.0, 0.9, False), (0.7, 0.5, True), (1.0, 1.0, False),
                                                    (1.5, 0.95, True), (0.3, 0.8, False)])
def test_topp_sample_kernel_token_exact(dev, dtype, temperature, top_p, ties):
    from icap import ops

    B = 24
    lg = torch.zeros((B, LD))
    lg[:, :V_GPT2] = _logits(B, V_GPT2, 21, ties=ties)
    lg[3, V_GPT2 - 1] = 40.0           # winner in the unaligned tail
    lg[4, V_GPT2:] = 1e9               # padding columns are ignored
    lg[5, 100:110] = 30.0              # 10-way tie at the top
    lg = lg.to(dtype)
    fin = torch.zeros(B, dtype=torch.int32)
    fin[7] = 1
    out = torch.full((B,), -1, dtype=torch.int64, device=dev)
    for step in (0, 3):
        ops.topp_sample(lg.to(dev), V_GPT2, temperature, top_p, fin.to(dev), 1234567, step, EOS, out)
        torch.cuda.synchronize()
        ref, _ = O.topp_sample_fixed(lg[:, :V_GPT2].float().numpy(), temperature, top_p, 1234567, step,
                                     finished=fin.numpy().astype(bool), eos=EOS)
        got = out.cpu().numpy()
        assert np.array_equal(got, ref), (np.nonzero(got != ref)[0], got[got != ref], ref[got != ref])
        assert got[7] == EOS and 100 <= got[5] < 110


@pytest.mark.gpu
def test_topp_sample_kernel_distribution(dev):
    """4096 rows of one logit vector: device draws follow the kept softmax (chi-square) and are token-exact."""
    from icap import ops

    V, B = 50257, 4096
    base = torch.full((V,), -40.0)
    idx = torch.tensor([5, 999, 20000, 31000, 45000, 50256])
    base[idx] = torch.tensor([1.0, 0.7, 0.4, 0.1, -0.2, -2.5])
    lg = base.repeat(B, 1)
    out = torch.empty(B, dtype=torch.int64, device=dev)
    ops.topp_sample(lg.to(dev), V, 1.0, 0.9, None, 99, 1, EOS, out)
    got = out.cpu().numpy()
    ref, kept = O.topp_sample_fixed(lg.numpy()[:64], 1.0, 0.9, 99, 1)
    assert np.array_equal(got[:64], ref)
    k = np.nonzero(kept[0])[0]
    assert set(np.unique(got)) <= set(k.tolist())
    p = torch.softmax(base[k], 0).numpy()
    obs = np.array([(got == j).sum() for j in k])
    chi2 = float(((obs - B * p) ** 2 / (B * p)).sum())
    assert chi2 < 30.0, (chi2, obs, B * p)

