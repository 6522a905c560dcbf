"""Packed token rows (include/icap.h icap_caption_pack; GPT2Core.alloc_train(pack=True), the trainer's default).

Each caption keeps its prefix and caption positions up to its last loss target; the dead tail of the padded
[B, P + L] grid (positions after the last target, which the causal mask keeps out of every loss term) is never
computed. Checked here:
  - icap_caption_pack against a numpy restatement (lengths, offsets, packed key mask / shifted labels, target
    compaction in the padded layout's row order), on ragged captions incl. one with no target and mask holes;
  - attention over packed sequences equals the padded launch on the live rows (fp32 VALU and bf16 MFMA kernels;
    forward output + lse, backward dQKV) — bitwise: the dropped keys only ever contributed exact zeros;
  - whole train steps, packed vs padded, dropout off: fp32 and bf16 losses and mapper parameters within 1e-6
    relative (the same kernels run the same per-row arithmetic; only the split / tile placement of GEMM rows can
    change the summation order), eager and HIP-graph replay.
"""

import numpy as np
import pytest
import torch

from icap import CaptionTrainer, ops
from test_model_gpu import TINY_G, TINY_M, build

pytestmark = pytest.mark.gpu


def ragged_batch(B, L, vocab, eos, E, seed):
    """Captions of random length 0..L-1 tokens + EOS; sequence 1 has no target at all; sequence 2 a mask hole."""
    g = torch.Generator().manual_seed(seed)
    ids = torch.randint(0, vocab - 1, (B, L), generator=g, dtype=torch.int64)
    mask = torch.zeros((B, L), dtype=torch.int64)
    lens = torch.randint(0, L, (B,), generator=g)
    for b in range(B):
        n = int(lens[b])
        ids[b, n] = eos
        ids[b, n + 1:] = eos
        mask[b, : n + 1] = 1
    labels = ids.clone()
    labels[mask == 0] = -100
    labels[1] = -100  # no target: the sequence keeps its P prefix rows only
    if L > 3 and B > 2:
        mask[2, 1] = 0  # a hole inside the live span (kept, masked as a key)
        labels[2, 1] = -100
    emb = torch.randn((B, E), generator=g)
    emb = emb / emb.norm(dim=-1, keepdim=True)
    return ids, mask, labels, emb


def pack_ref(B, P, L, mask, labels):
    """numpy restatement of icap_caption_pack."""
    S = P + L
    mask, labels = mask.numpy(), labels.numpy()

    def lab(b, t):
        tn = t + 1
        return int(labels[b, tn - P]) if (P <= tn < S) else -100

    seq_len = np.array([max([P] + [t + 1 for t in range(P, S) if lab(b, t) != -100]) for b in range(B)], np.int32)
    seq_off = np.concatenate([[0], np.cumsum(seq_len)[:-1]]).astype(np.int32)
    m = int(seq_len.sum())
    km = np.zeros(B * S, np.int32)
    ls = np.full(B * S, -100, np.int32)
    for b in range(B):
        for t in range(seq_len[b]):
            r = seq_off[b] + t
            km[r] = 1 if t < P else int(mask[b, t - P] != 0)
            ls[r] = lab(b, t)
    slot = np.full(B * S, -1, np.int32)
    tgt = np.nonzero(ls != -100)[0]
    slot[tgt] = np.arange(len(tgt))
    return seq_off, seq_len, m, km, ls, slot, ls[tgt]


@pytest.mark.parametrize("B,P,L", [(5, 4, 9), (128, 15, 50), (1100, 3, 6), (40, 0, 70), (2100, 2, 5)])
def test_caption_pack_layout(dev, B, P, L):
    ids, mask, labels, _ = ragged_batch(B, L, 100, 99, 8, seed=B)
    S = P + L
    i32 = dict(dtype=torch.int32, device=dev)
    so, sl, ml = torch.empty(B, **i32), torch.empty(B, **i32), torch.empty(1, **i32)
    km, ls, slot = (torch.full((B * S,), 7, **i32) for _ in range(3))
    labc, nv = torch.full((B * L,), 7, **i32), torch.empty(1, **i32)
    ops.caption_pack(B, P, L, mask.to(dev), labels.to(dev), so, sl, ml, km, ls, nv, slot, labc)
    r_off, r_len, r_m, r_km, r_ls, r_slot, r_labc = pack_ref(B, P, L, mask, labels)
    assert np.array_equal(sl.cpu().numpy(), r_len) and np.array_equal(so.cpu().numpy(), r_off)
    assert int(ml.item()) == r_m
    assert np.array_equal(km.cpu().numpy(), r_km) and np.array_equal(ls.cpu().numpy(), r_ls)
    assert np.array_equal(slot.cpu().numpy(), r_slot)
    assert int(nv.item()) == len(r_labc) and np.array_equal(labc.cpu().numpy()[: len(r_labc)], r_labc)
    # the same targets, in the same order, as the padded layout's compaction (icap_caption_prep)
    ks, ls2, slot2 = (torch.empty(B * S, **i32) for _ in range(3))
    labc2, nv2 = torch.empty(B * L, **i32), torch.empty(1, **i32)
    ops.caption_prep(B, P, L, mask.to(dev), labels.to(dev), ks, ls2, nv2, slot2, labc2)
    assert int(nv2.item()) == int(nv.item())
    assert torch.equal(labc2[: int(nv.item())], labc[: int(nv.item())])


def _pack_dev(B, P, L, mask, labels, dev):
    S = P + L
    i32 = dict(dtype=torch.int32, device=dev)
    so, sl, ml = torch.empty(B, **i32), torch.empty(B, **i32), torch.empty(1, **i32)
    km, ls = torch.empty(B * S, **i32), torch.empty(B * S, **i32)
    ops.caption_pack(B, P, L, mask.to(dev), labels.to(dev), so, sl, ml, km, ls, None)
    return so, sl, km


@pytest.mark.parametrize("dtype,H,hd,P,L", [(torch.float32, 2, 32, 5, 12), (torch.bfloat16, 12, 64, 15, 50),
                                             (torch.bfloat16, 2, 96, 5, 12)])
def test_attention_packed_equals_padded(dev, dtype, H, hd, P, L):
    B = 6
    S, D = P + L, H * hd
    _, mask, labels, _ = ragged_batch(B, L, 100, 99, 8, seed=3)
    so, sl, km_packed = _pack_dev(B, P, L, mask, labels, dev)
    key_mask = torch.cat([torch.ones((B, P), dtype=torch.int64), mask], 1).reshape(-1).to(torch.int32).to(dev)
    g = torch.Generator().manual_seed(11)
    qkv = torch.randn((B * S, 3 * D), generator=g).to(dev, dtype)
    lens, offs = sl.cpu().tolist(), so.cpu().tolist()
    rows = torch.cat([torch.arange(b * S, b * S + lens[b]) for b in range(B)]).to(dev)
    dout = torch.zeros((B * S, D), dtype=dtype, device=dev)  # dead rows feed no loss: their gradient is 0
    dout[rows] = torch.randn((len(rows), D), generator=g).to(dev, dtype)
    kw = dict(B=B, S=S, H=H, hd=hd, scale=hd ** -0.5, causal=True)
    # padded reference launch
    o_pad = torch.zeros((B * S, D), dtype=dtype, device=dev)
    lse_pad = torch.full((B * H * S,), 7.0, device=dev)
    ops.attention_fwd(qkv, o_pad, key_mask=key_mask, lse=lse_pad, **kw)
    d_pad = torch.zeros_like(qkv)
    ops.attention_bwd(qkv, dout, lse_pad, d_pad, key_mask=key_mask, out=o_pad, **kw)
    # packed launch over the live rows
    qkv_p = qkv[rows].contiguous()
    dout_p = dout[rows].contiguous()
    cap = B * S
    qkv_c = torch.zeros((cap, 3 * D), dtype=dtype, device=dev)
    qkv_c[: len(rows)] = qkv_p
    dout_c = torch.zeros((cap, D), dtype=dtype, device=dev)
    dout_c[: len(rows)] = dout_p
    o_pk = torch.zeros((cap, D), dtype=dtype, device=dev)
    lse_pk = torch.full((B * H * S,), 7.0, device=dev)
    ops.attention_fwd(qkv_c, o_pk, key_mask=km_packed, lse=lse_pk, seqs=(so, sl), **kw)
    d_pk = torch.zeros_like(qkv_c)
    ops.attention_bwd(qkv_c, dout_c, lse_pk, d_pk, key_mask=km_packed, out=o_pk, seqs=(so, sl), **kw)
    torch.cuda.synchronize()
    n = len(rows)
    assert torch.equal(o_pk[:n], o_pad[rows])
    assert torch.equal(d_pk[:n], d_pad[rows])
    lp, lq = lse_pad.view(B, H, S), lse_pk.view(B, H, S)
    for b in range(B):
        assert torch.equal(lq[b, :, : lens[b]], lp[b, :, : lens[b]]), b
    assert offs == sorted(offs)


def _train(dtype, dev, pack, graph, batch):
    ids, mask, labels, emb = batch
    model = build(TINY_G, TINY_M, dtype, dev)
    t = CaptionTrainer(model, ids.shape[0], ids.shape[1], lr=1e-3, num_training_steps=4, dropout=False,
                       pack_rows=pack, seed=5)
    assert t.gws.pack == pack
    t.load_batch(ids.to(dev), mask.to(dev), labels.to(dev), emb.to(dev))
    losses = []
    for _ in range(3):
        t.micro_step(use_graph=graph)
        losses.append(t.last_loss.item())
    return losses, {k: v.detach().clone() for k, v in model.mapping_network.state_dict().items()}


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("graph", [False, True])
def test_packed_step_equals_padded(dev, dtype, graph):
    batch = ragged_batch(7, 12, TINY_G.vocab_size, TINY_G.eos, TINY_M.embed_dim, seed=9)
    lp, sp = _train(dtype, dev, True, graph, batch)
    lq, sq = _train(dtype, dev, False, graph, batch)
    assert np.allclose(lp, lq, rtol=1e-6, atol=0), (lp, lq)
    for k in sp:
        a, b = sp[k].double(), sq[k].double()
        assert float((a - b).abs().max()) <= 1e-6 * float(b.abs().max()) + 1e-12, k


def test_packed_step_with_dropout_runs(dev):
    """Dropout on: the packed step draws its masks by packed row (a different, equally distributed draw from the
    padded layout's), so only finiteness and descent are checked."""
    ids, mask, labels, emb = ragged_batch(7, 12, TINY_G.vocab_size, TINY_G.eos, TINY_M.embed_dim, seed=4)
    model = build(TINY_G, TINY_M, torch.float32, dev)
    t = CaptionTrainer(model, 7, 12, lr=3e-3, num_training_steps=20, dropout=True, seed=2)
    assert t.gws.pack
    t.load_batch(ids.to(dev), mask.to(dev), labels.to(dev), emb.to(dev))
    losses = []
    for _ in range(12):
        t.micro_step(use_graph=True)
        losses.append(t.last_loss.item())
    assert all(np.isfinite(losses)) and losses[-1] < losses[0], losses


@pytest.mark.parametrize("N,K,epi", [(768, 3072, "resid_drop"), (768, 2304, "plain"), (768, 1160, "f32"),
                                     (640, 3072, "plain")])
def test_packed_gemm_kernel_equals_tile_kernel(dev, N, K, epi):
    """The packed step's N <= 1024 products with the expected live-row count (m_hint) take the split-role ring on
    96 x 128 tiles (round 6, icap_gemm variant 27: one round of tiles, no split of K); it runs the tile kernel's MFMA
    chain in natural k order, so its live rows equal the 128-row tile path's (tile_only) bitwise and rows past the
    device count stay untouched; close to fp32 torch. (Round 3's 4-stage ring, variant 16, took these launches
    before; the unhinted plan sizes its choice for the capacity rows and keeps the split / 128-row kernels.)"""
    from icap import _lib as L

    mcap, mlive = 8320, 3584
    g = torch.Generator().manual_seed(K + N)
    A = (torch.rand((mcap, K), generator=g) * 2 - 1).to(dev, torch.bfloat16)
    B = (torch.rand((N, K), generator=g) * 2 - 1).to(dev, torch.bfloat16)
    cdt = torch.float32 if epi == "f32" else torch.bfloat16
    kw = {}
    if epi == "resid_drop":
        kw = dict(bias=torch.randn(N, generator=g).to(dev), resid=torch.randn((mcap, N), generator=g).to(dev, cdt),
                  drop=ops.Dropout(0.1, 7))
    mdev = torch.tensor([mlive], dtype=torch.int32, device=dev)
    outs = []
    for form in ("hint", "tile"):
        C = torch.zeros((mcap, N), device=dev, dtype=cdt)
        extra = dict(m_hint=mlive) if form == "hint" else dict(tile_only=True)
        outs.append(ops.gemm(A, B, C, m_dev=mdev, split_k=1, **extra, **kw))
    ga = L.GemmArgs()
    ga.M, ga.N, ga.K, ga.in_dtype, ga.c_dtype = mcap, N, K, L.BF16, ops.dtype_code(cdt)
    ga.A, ga.lda, ga.B, ga.ldb, ga.C, ga.ldc = A.data_ptr(), K, B.data_ptr(), K, outs[0].data_ptr(), N
    ga.m_dev, ga.m_hint = mdev.data_ptr(), mlive
    ga.alpha, ga.split_k = 1.0, 1
    if epi == "resid_drop":
        ga.resid, ga.ldr = kw["resid"].data_ptr(), N
    name = L.load().icap_gemm_kernel_name(ga).decode()
    torch.cuda.synchronize()
    assert "5, 1, 2, 2, 3, 4" in name and name.endswith(", true>"), name
    assert torch.equal(outs[0][:mlive], outs[1][:mlive])
    assert torch.count_nonzero(outs[0][mlive:]) == 0  # rows past the device count untouched
    if epi != "resid_drop":
        ref = A[:mlive].float() @ B.float().t()
        assert float((outs[0][:mlive].float() - ref).abs().max() / ref.abs().max()) < 1e-2


def test_attention_short_only_equals_both_passes(dev):
    """icap_attn_args.short_only: with every packed sequence <= 32 tokens in a launch of S = 65, the short pass alone
    stores what the two passes store (the long pass only exits), forward and backward, bitwise."""
    B, P, L, H, hd = 9, 15, 50, 12, 64
    S, D = P + L, H * hd
    _, mask, labels, _ = ragged_batch(B, L, 100, 99, 8, seed=5)
    labels[:, 17:] = -100  # every caption's last target within the first 17 positions: sequences <= 15 + 16 = 31
    mask[:, 18:] = 0
    from icap.engine import max_seq_len
    assert max_seq_len(labels, P) <= 32
    so, sl, km = _pack_dev(B, P, L, mask, labels, dev)
    g = torch.Generator().manual_seed(12)
    qkv = torch.randn((B * S, 3 * D), generator=g).to(dev, torch.bfloat16)
    dout = torch.randn((B * S, D), generator=g).to(dev, torch.bfloat16)
    kw = dict(B=B, S=S, H=H, hd=hd, scale=hd ** -0.5, causal=True, key_mask=km, seqs=(so, sl))
    res = []
    for short in (False, True):
        o = torch.zeros((B * S, D), dtype=torch.bfloat16, device=dev)
        lse = torch.full((B * H * S,), 7.0, device=dev)
        ops.attention_fwd(qkv, o, lse=lse, short_only=short, **kw)
        d = torch.zeros_like(qkv)
        ops.attention_bwd(qkv, dout, lse, d, out=o, short_only=short, **kw)
        torch.cuda.synchronize()
        res.append((o, lse, d))
    for a, b in zip(*res):
        assert torch.equal(a, b)


def test_trainer_short_only_switches_graphs(dev, monkeypatch):
    """The trainer takes short_only from each batch's labels and keys its captured graphs on it: a short batch, then
    one with a sequence past 32 tokens, then the short one again (graph replay) give the losses of a trainer that
    always launches both passes (ICAP_SHORT_ONLY=0), bitwise."""
    import icap.engine as E
    short = ragged_batch(6, 30, TINY_G.vocab_size, TINY_G.eos, TINY_M.embed_dim, seed=21)
    ids, mask, labels, emb = short
    labels[:, 12:] = -100
    mask[:, 13:] = 0
    long_ = ragged_batch(6, 30, TINY_G.vocab_size, TINY_G.eos, TINY_M.embed_dim, seed=22)
    long_[2][0, :] = torch.arange(30) % TINY_G.vocab_size  # caption 0 has targets up to position 30
    long_[1][0, :] = 1
    out = {}
    for flag in (True, False):
        monkeypatch.setattr(E, "SHORT_ONLY", flag)
        model = build(TINY_G, TINY_M, torch.float32, dev)
        t = CaptionTrainer(model, 6, 30, lr=1e-3, num_training_steps=8, dropout=False, seed=5)
        P = t.P
        assert E.max_seq_len(labels, P) <= 32 and E.max_seq_len(long_[2], P) > 32
        losses = []
        for ids_, mask_, labels_, emb_ in (short, long_, short, long_, short):
            t.load_batch(ids_, mask_, labels_, emb_.to(dev))  # host labels: the trainer reads short_only from them
            t.micro_step(use_graph=True)
            losses.append(t.last_loss.item())
        out[flag] = losses
        if flag:
            assert {k[2] for k in t.graphs} == {True, False}
    assert out[True] == out[False], out
