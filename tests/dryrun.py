"""Dry-run harness: run the icap host schedules on the CPU with the C-ABI calls RECORDED instead of launched,
then check every pointer range each call will touch against the allocations that exist.

A GPU memory fault can reset a shared machine, so every kernel schedule (train step, decode, CLIP) is
bounds-checked here, on the CPU, before it is run on a GPU. The extents below restate each entry point's
access pattern from include/icap.h."""

from __future__ import annotations

import ctypes as C
import gc
from contextlib import contextmanager

import torch

from icap import _lib, ops

ES = {0: 4, 1: 2, 2: 1}


def _extent(ptr, nbytes):
    return (int(ptr), int(ptr) + int(nbytes)) if ptr else None


def _rows(n, ld, w, es):
    return 0 if n <= 0 else ((n - 1) * ld + w) * es


def accesses(name, args):
    """[(label, ptr, nbytes)] for one recorded call."""
    a = args
    out = []
    if name == "icap_gemm":
        g = a[0]._obj
        ei, ec = ES[g.in_dtype], ES[g.c_dtype]
        if g.trans_ab:  # K-outer operands: [K][lda] / [K][ldb]
            out += [("A", g.A, _rows(g.K, g.lda, g.M, ei)), ("B", g.B, _rows(g.K, g.ldb, g.N, ei))]
        else:
            out += [("A", g.A, _rows(g.M, g.lda, g.K, ei)), ("B", g.B, _rows(g.N, g.ldb, g.K, ei))]
        out += [
                ("C", g.C, _rows(g.M, g.ldc, g.N, ec)), ("bias", g.bias, g.N * 4),
                ("aux", g.aux, _rows(g.M, g.ldaux, g.N, ec)), ("dact_src", g.dact_src, _rows(g.M, g.ld_dact, g.N, ec)),
                ("resid", g.resid, _rows(g.M, g.ldr, g.N, ec)), ("seed_ptr", g.seed_ptr, 8),
                ("workspace", g.workspace, g.workspace_bytes), ("m_dev", g.m_dev, 4),
                ("ln_gamma", g.ln_gamma, g.K * 4), ("ln_beta", g.ln_beta, g.K * 4),
                ("tickets", g.tickets, g.tickets_len * 4), ("ln_wsum", g.ln_wsum, g.N * 4),
                ("ln_stats_out", g.ln_stats_out, g.M * (g.N // 32) * 8), ("ln_stats_in", g.ln_stats_in, g.M * (g.K // 32) * 8),
                ("ln_mean_out", g.ln_mean_out, g.M * 4), ("ln_rstd_out", g.ln_rstd_out, g.M * 4)]
        if g.in_dtype == 2:  # MX block scales (include/icap.h a_scale / b_scale layout)
            out += [("a_scale", g.a_scale, ops.mx_scale_bytes(g.M, g.K)), ("b_scale", g.b_scale, ops.mx_scale_bytes(g.N, g.K))]
    elif name == "icap_gemm_group":  # n K-outer products (icap_gemm_group): A [K][lda], B [K][ldb], C [M][ldc] fp32
        arr, n = a[0], a[1]
        for i in range(n):
            g = arr[i]
            ei, ec = ES[g.in_dtype], ES[g.c_dtype]
            out += [(f"A{i}", g.A, _rows(g.K, g.lda, g.M, ei)), (f"B{i}", g.B, _rows(g.K, g.ldb, g.N, ei)),
                    (f"C{i}", g.C, _rows(g.M, g.ldc, g.N, ec))]
    elif name in ("icap_attention_fwd", "icap_attention_bwd"):
        t = a[0]._obj
        es = ES[t.dtype]
        D = t.H * t.hd
        maxrow = (t.B - 1) * t.row_stride_b + (t.S - 1) * t.row_stride_s
        if t.seq_off:  # packed sequences: rows seq_off[b] + s < B*S (the offsets live on the device)
            maxrow = t.B * t.S - 1
            out += [("seq_off", t.seq_off, t.B * 4), ("seq_len", t.seq_len, t.B * 4)]
        out += [("qkv", t.qkv, (maxrow * t.ld_qkv + 3 * D) * es), ("lse", t.lse, t.B * t.H * t.S * 4),
                ("key_mask", t.key_mask, t.B * t.S * 4), ("seed_ptr", t.seed_ptr, 8)]
        if name == "icap_attention_fwd":
            out.append(("out", t.out, (maxrow * t.ld_out + D) * es))
        else:
            out += [("dout", t.dout, (maxrow * t.ld_dout + D) * es), ("dqkv", t.dqkv, (maxrow * t.ld_dqkv + 3 * D) * es),
                    ("out", t.out, (maxrow * t.ld_out + D) * es)]
    elif name == "icap_adamw_step":
        t = a[0]._obj
        n = t.n
        out += [("params", t.params, n * 4), ("grads", t.grads, n * 4), ("m", t.exp_avg, n * 4),
                ("v", t.exp_avg_sq, n * 4), ("bf16_out", t.bf16_out, n * 2), ("state", t.state, 64),
                ("ws", a[1], ops.adamw_workspace(n))]
    elif name == "icap_layernorm_fwd":
        dt, rows, D, x, ldx, gm, bt, _, y, ldy, mean, rstd, ymap, rdev, _s = a
        es = ES[dt]
        # with a row map the stored rows are the compacted slots (< n_valid <= B*L, set on the device by
        # icap_caption_prep): only the first row is checkable here
        yrows = 1 if ymap else rows
        out += [("x", x, _rows(rows, ldx, D, es)), ("gamma", gm, D * 4), ("beta", bt, D * 4),
                ("y", y, _rows(yrows, ldy, D, es)), ("mean", mean, rows * 4), ("rstd", rstd, rows * 4),
                ("y_rowmap", ymap, rows * 4), ("rows_dev", rdev, 4)]
    elif name == "icap_layernorm_bwd":
        (dt, rows, D, x, ldx, gm, mean, rstd, dy, lddy, dres, lddres, dx, lddx, dxd, _p, _sd, _o, sp, dg, db, ws,
         dymap, rdev, _acc, _s) = a
        es = ES[dt]
        dyrows = 1 if dymap else rows  # row map: compacted slots (see layernorm_fwd)
        out += [("x", x, _rows(rows, ldx, D, es)), ("gamma", gm, D * 4), ("mean", mean, rows * 4),
                ("rstd", rstd, rows * 4), ("dy", dy, _rows(dyrows, lddy, D, es)),
                ("dres", dres, _rows(rows, lddres, D, es)), ("dx", dx, _rows(rows, lddx, D, es)),
                ("dx_drop", dxd, _rows(rows, lddx, D, es)), ("seed_ptr", sp, 8), ("dgamma", dg, D * 4),
                ("dbeta", db, D * 4), ("dy_rowmap", dymap, rows * 4), ("rows_dev", rdev, 4)]
        if dg or db:
            out.append(("ws", ws, ops.layernorm_bwd_workspace(rows, D)))
    elif name == "icap_ln_param_reduce_batch":
        n, arr = a[0], a[1]
        for i in range(n):
            it = arr[i]
            out += [(f"ws{i}", it.workspace, ops.layernorm_bwd_workspace(it.rows, it.D)),
                    (f"dgamma{i}", it.dgamma, it.D * 4), (f"dbeta{i}", it.dbeta, it.D * 4)]
    elif name == "icap_gpt2_embed":
        dt, B, P, L, D, pre, pbs, wte, wpe, ids, x, _p, _sd, _o, sp, so, sl, _s = a
        es = ES[dt]
        out += [("prefix", pre, ((B - 1) * pbs + P * D) * es if P else 0), ("wte", wte, D * es),
                ("wpe", wpe, (P + L) * D * es), ("ids", ids, B * L * 8), ("x", x, B * (P + L) * D * es),
                ("seed_ptr", sp, 8), ("seq_off", so, B * 4), ("seq_len", sl, B * 4)]
    elif name == "icap_caption_prep":
        B, P, L, mask, labels, km, ls, nv, slot, labc, _s = a
        out += [("mask", mask, B * L * 8), ("labels", labels, B * L * 8), ("key_mask", km, B * (P + L) * 4),
                ("labels_shift", ls, B * (P + L) * 4), ("n_valid", nv, 4), ("row_slot", slot, B * (P + L) * 4),
                ("labels_compact", labc, B * L * 4)]
    elif name == "icap_caption_pack":
        B, P, L, mask, labels, so, sl, ml, km, ls, nv, slot, labc, _s = a
        n = B * (P + L)
        out += [("mask", mask, B * L * 8), ("labels", labels, B * L * 8), ("seq_off", so, B * 4),
                ("seq_len", sl, B * 4), ("m_live", ml, 4), ("key_mask", km, n * 4), ("labels_shift", ls, n * 4),
                ("n_valid", nv, 4), ("row_slot", slot, n * 4), ("labels_compact", labc, B * L * 4)]
    elif name == "icap_rows_unpack":
        dt, B, P, D, src, so, sl, dst, dbs, _s = a
        # src rows seq_off[b] + t < seq_off[b] + seq_len[b] <= the packed row count (checked: first row)
        out += [("src", src, D * ES[dt]), ("seq_off", so, B * 4), ("seq_len", sl, B * 4),
                ("dst", dst, ((B - 1) * dbs + P * D) * ES[dt])]
    elif name == "icap_cross_entropy":
        dt, rows, V, lg, ld, lab, nv, loss, dl, _g, ws, rdev, _s = a
        es = ES[dt]
        out += [("logits", lg, _rows(rows, ld, V, es)), ("labels", lab, rows * 4), ("n_valid", nv, 4),
                ("loss", loss, 4), ("dlogits", dl, _rows(rows, ld, ld, es)), ("ws", ws, rows * 4),
                ("rows_dev", rdev, 4)]
    elif name == "icap_transpose":
        dt, rows, cols, src, lds, dst, ldd, rp, _s = a
        es = ES[dt]
        out += [("src", src, _rows(rows, lds, cols, es)), ("dst", dst, _rows(cols, ldd, rp, es))]
    elif name == "icap_transpose_batch":
        n, ptr, _s = a
        from icap import _lib as _L
        addr = ptr.value if hasattr(ptr, "value") else ptr
        for it in (_L.TransposeItem * n).from_address(addr):
            out += [("src", it.src, _rows(it.rows, it.lds, it.cols, 2)), ("dst", it.dst, _rows(it.cols, it.ldd, it.rows, 2))]
    elif name == "icap_colsum":
        dt, M, N, src, ld, o, _acc, ws, _s = a
        out += [("src", src, _rows(M, ld, N, ES[dt])), ("out", o, N * 4), ("ws", ws, ops.colsum_workspace(M, N))]
    elif name == "icap_colsum_batch":
        dt, M, n, ptr, _acc, ws, _s = a
        from icap import _lib as _L
        addr = ptr.value if hasattr(ptr, "value") else ptr
        items = list((_L.ColsumItem * n).from_address(addr))
        for it in items:
            out += [("src", it.src, _rows(M, it.ld, it.N, ES[dt])), ("out", it.out, it.N * 4)]
        out.append(("ws", ws, ops.colsum_workspace(M, sum(it.N for it in items))))
    elif name == "icap_dropout_apply":
        dt, M, N, src, lds, dst, ldd, _p, _sd, _o, sp, _s = a
        out += [("src", src, _rows(M, lds, N, ES[dt])), ("dst", dst, _rows(M, ldd, N, ES[dt])), ("seed_ptr", sp, 8)]
    elif name == "icap_convert":
        sdt, ddt, M, N, src, lds, dst, ldd, _s = a
        out += [("src", src, _rows(M, lds, N, ES[sdt])), ("dst", dst, _rows(M, ldd, N, ES[ddt]))]
    elif name == "icap_broadcast_rows":
        dt, B, R, D, src, dst, bs, _s = a
        out += [("src", src, R * D * 4), ("dst", dst, ((B - 1) * bs + R * D) * ES[dt])]
    elif name == "icap_quantize_mx":
        dt, R, K, x, ldx, q, ldq, sc, rdev, _s = a
        out += [("x", x, _rows(R, ldx, K, ES[dt])), ("q", q, _rows(R, ldq, K, 1)), ("scales", sc, ops.mx_scale_bytes(R, K)),
                ("rows_dev", rdev, 4)]
    elif name == "icap_counter_increment":
        out.append(("counter", a[0], 8))
    elif name == "icap_im2col_patches":
        dt, B, Cc, HW, p, px, pt, _s = a
        kp = (Cc * p * p + 7) // 8 * 8  # rows padded to a multiple of 8 elements
        out += [("pixels", px, B * Cc * HW * HW * 4), ("patches", pt, B * (HW // p) ** 2 * kp * ES[dt])]
    elif name == "icap_vit_embed":
        dt, B, G2, D, pe, cls, pos, x, _s = a
        out += [("pe", pe, B * G2 * D * ES[dt]), ("cls", cls, D * 4), ("pos", pos, (G2 + 1) * D * 4),
                ("x", x, B * (G2 + 1) * D * ES[dt])]
    elif name == "icap_prefix_embed":
        dt, B, G2, NP, D, pe, pf, pos, x, _s = a
        out += [("pe", pe, B * G2 * D * ES[dt]), ("prefix", pf, NP * D * 4), ("x", x, B * (G2 + NP) * D * ES[dt])]
        if pos:
            out.append(("pos", pos, (G2 + NP) * D * 4))
    elif name == "icap_patch_embed":
        B, Cc, HW, p, NP, N, px, w, ldw, Kp, bias, pos, pf, o, ldo, _s = a
        S = NP + (HW // p) ** 2
        out += [("pixels", px, B * Cc * HW * HW * 4), ("w", w, _rows(N, ldw, Kp, 2)), ("bias", bias, N * 4),
                ("pos", pos, S * N * 4), ("prefix", pf, NP * N * 4), ("out", o, _rows(B * S, ldo, N, 2))]
    elif name == "icap_rope_patches":
        dt, B, S, NP, H, hd, q, ld, cs, sn, _s = a
        out += [("qkv", q, _rows(B * S, ld, 2 * H * hd, ES[dt])), ("cos", cs, (S - NP) * hd * 4),
                ("sin", sn, (S - NP) * hd * 4)]
    elif name == "icap_l2norm_rows":
        dt, rows, D, x, ldx, o, ldo, _s = a
        out += [("x", x, _rows(rows, ldx, D, ES[dt])), ("out", o, _rows(rows, ldo, D, 4))]
    elif name == "icap_greedy_next":
        dt, B, V, lg, ld, _eos, forced, fin, tok, ldt, step, wte, wpe, pos, D, x, _s = a
        es = ES[dt]
        out += [("logits", lg, _rows(B, ld, V, es)), ("forced", forced, B * 8), ("finished", fin, B * 4),
                ("tokens", tok, ((B - 1) * ldt + step + 1) * 8), ("wte", wte, D * es),
                ("wpe", wpe, (pos + 1) * D * es), ("x", x, B * D * es)]
    elif name == "icap_topp_sample":
        dt, B, V, lg, ld, _t, _p, fin, _seed, seed_ptr, _step, _eos, outp, _s = a
        out += [("logits", lg, _rows(B, ld, V, ES[dt])), ("finished", fin, B * 4), ("seed_ptr", seed_ptr, 8),
                ("out", outp, B * 8)]
    elif name == "icap_add_position":
        dt, B, npos, D, src, sbs, sts, wpe, pos0, x, _s = a
        es = ES[dt]
        out += [("src", src, ((B - 1) * sbs + (npos - 1) * sts + D) * es), ("wpe", wpe, (pos0 + npos) * D * es),
                ("x", x, npos * B * D * es)]
    elif name == "icap_attention_decode":
        dt, B, H, hd, pos, cache, ldc, o, ldo, _sc, _s = a
        es = ES[dt]
        out += [("cache", cache, ((pos + 1) * B - 1) * ldc * es + 3 * H * hd * es), ("out", o, _rows(B, ldo, H * hd, es))]
    elif name in ("icap_beam_init", "icap_beam_update", "icap_beam_finalize"):
        b = a[0]._obj
        R = b.B * b.W
        out += [("ws", b.ws, _lib.load().icap_beam_workspace_bytes(b.B, b.W, b.T, b.max_len))]
        if name == "icap_beam_update":
            es = ES[b.dtype]
            out += [("top_val", b.top_val, R * b.K * 4), ("top_idx", b.top_idx, R * b.K * 4), ("top_m", b.top_m, R * 4),
                    ("top_ls", b.top_ls, R * 4), ("x", b.x, R * b.D * es), ("wte", b.wte, b.V * b.D * es),
                    ("wpe", b.wpe, b.n_positions * b.D * es)]
        if name == "icap_beam_finalize":
            out += [("out", a[1], b.B * b.max_len * 8), ("out_len", a[2], b.B * 4)]
    elif name == "icap_beam_rowtop":
        dt, R, V, lg, ld, K, tv, ti, tm, tl, _s = a
        out += [("logits", lg, _rows(R, ld, V, ES[dt])), ("top_val", tv, R * K * 4), ("top_idx", ti, R * K * 4),
                ("top_m", tm, R * 4), ("top_ls", tl, R * 4)]
    elif name == "icap_attention_decode_anc":
        dt, B, H, hd, pos, cache, ldc, anc, o, ldo, _sc, _s = a
        es = ES[dt]
        out += [("cache", cache, ((pos + 1) * B - 1) * ldc * es + 3 * H * hd * es), ("anc", anc, (pos + 1) * B * 4),
                ("out", o, _rows(B, ldo, H * hd, es))]
    elif name == "icap_embedding_scatter_add":
        dt, B, P, L, D, dx, ids, dw, _s = a
        out += [("dx", dx, B * (P + L) * D * ES[dt]), ("ids", ids, B * L * 8), ("dwte", dw, D * 4)]
    else:
        raise KeyError(f"dry-run: no extent model for {name}")
    return [(lbl, int(p), int(n)) for lbl, p, n in out if p and n > 0]


def live_storages():
    """(start, end) of every live CPU tensor storage."""
    ranges = set()
    for o in gc.get_objects():
        try:
            if isinstance(o, torch.Tensor) and o.device.type == "cpu" and not o.is_meta:
                st = o.untyped_storage()
                ranges.add((st.data_ptr(), st.data_ptr() + st.nbytes()))
        except Exception:  # noqa: BLE001
            pass
    return sorted(ranges)


class Recorder:
    """Records calls and checks each call's extents against the allocations live AT CALL TIME
    (the live-range table is rescanned only when an extent is not found in the cached one)."""

    def __init__(self):
        self.calls = []
        self.ranges = []
        self.bad = []

    def _inside(self, p, n):
        return any(lo <= p and p + n <= hi for lo, hi in self.ranges)

    def __call__(self, name, *args):
        for lbl, p, n in accesses(name, args):
            if not self._inside(p, n):
                self.ranges = live_storages()
                if not self._inside(p, n):
                    self.bad.append(f"{name}.{lbl}: [{p:#x}, +{n}) outside every live allocation")
        self._record(name, args)

    def _record(self, name, args):
        # keep ctypes structs alive and snapshot them
        snap = []
        for x in args:
            if hasattr(x, "_obj"):
                obj = type(x._obj)()
                C.pointer(obj)[0] = x._obj
                snap.append(C.byref(obj))
            else:
                snap.append(x)
        self.calls.append((name, tuple(snap)))

    def check(self):
        return list(self.bad)


@contextmanager
def dry_run():
    """Patch the binding so ops record instead of launching; model/cores work on CPU tensors."""
    rec = Recorder()
    saved = (_lib.require_device, ops.call, ops._stream)
    _lib.require_device = lambda d: None
    ops.call = rec
    ops._stream = lambda: None
    # keep every tensor allocated during the dry run alive, so workspaces freed before check() still count
    keep = []
    factories = ("empty", "zeros", "ones", "full", "empty_like", "zeros_like", "full_like", "randn")
    orig = {n: getattr(torch, n) for n in factories}

    def wrap(fn):
        def f(*a, **k):
            t = fn(*a, **k)
            keep.append(t)
            return t
        return f

    for n in factories:
        setattr(torch, n, wrap(orig[n]))
    rec.keep = keep
    try:
        yield rec
    finally:
        _lib.require_device, ops.call, ops._stream = saved
        for n in factories:
            setattr(torch, n, orig[n])
