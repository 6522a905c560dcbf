"""Thin torch-tensor wrappers over the C-ABI (include/icap.h).

Tensors are PyTorch-owned device memory; every wrapper passes raw pointers,
element strides and the current HIP stream to libicap_hip.so. No wrapper does
arithmetic itself and none falls back to PyTorch or the CPU.
"""

from __future__ import annotations

import contextlib
import ctypes as C
import os
import gc
from typing import Optional, Tuple

import torch

from . import _lib as L
from ._lib import AdamWArgs, AttnArgs, GemmArgs, call

Tensor = torch.Tensor


def dtype_code(t: torch.dtype) -> int:
    if t == torch.float32:
        return L.F32
    if t == torch.bfloat16:
        return L.BF16
    raise L.IcapError(f"unsupported storage dtype {t} (float32 or bfloat16)")


def _p(t: Optional[Tensor]):
    return None if t is None else t.data_ptr()


def _ld(t: Tensor) -> int:
    if t.dim() == 1:
        return t.shape[0]
    if t.stride(-1) != 1:
        raise L.IcapError("operand must have unit stride in its last dimension")
    return t.stride(-2)


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _rows(t: Tensor) -> int:
    return t.shape[0] if t.dim() >= 1 else 1


@contextlib.contextmanager
def graph_capture(g):
    """torch.cuda.graph(g) with Python's cyclic garbage collector held off for the capture. The decode / beam
    runners and their cores reference each other, so dropped ones are freed by the collector, and a collection
    that runs inside a capture destroys their HIP graphs and frees their memory mid-capture, which the runtime
    does not allow (the process aborts). Collect first, then capture with the collector disabled."""
    gc.collect()
    was = gc.isenabled()
    gc.disable()
    try:
        with torch.cuda.graph(g):
            yield g
    finally:
        if was:
            gc.enable()


class Dropout:
    """Dropout descriptor: (p, seed, offset, device seed counter)."""

    __slots__ = ("p", "seed", "offset", "counter")

    def __init__(self, p: float = 0.0, seed: int = 0, offset: int = 0, counter: Optional[Tensor] = None):
        self.p, self.seed, self.offset, self.counter = float(p), int(seed) & (2**64 - 1), int(offset), counter

    def at(self, offset: int) -> "Dropout":
        return Dropout(self.p, self.seed, offset, self.counter)

    @property
    def ptr(self):
        return None if self.counter is None else self.counter.data_ptr()


NO_DROP = Dropout()


class MXTensor:
    """An ICAP_FP8_MX GEMM operand: e4m3 bytes q [R, K] (uint8, row stride % 16 == 0) + E8M0 block scales in the
    layout icap_quantize_mx writes (include/icap.h icap_gemm_args.a_scale). Row views (rows r0:r1 with r0 % 64 == 0)
    are not supported: an operand is always the whole quantised matrix."""

    __slots__ = ("q", "scale", "R", "K")

    def __init__(self, q: Tensor, scale: Tensor, R: int, K: int):
        if q.dtype != torch.uint8 or scale.dtype != torch.uint8:
            raise L.IcapError("MXTensor: q and scale must be uint8")
        self.q, self.scale, self.R, self.K = q, scale, R, K

    @staticmethod
    def empty(R: int, K: int, device) -> "MXTensor":
        nb = mx_scale_bytes(R, K)
        return MXTensor(torch.empty((R, K), dtype=torch.uint8, device=device),
                        torch.empty(nb, dtype=torch.uint8, device=device), R, K)

    @property
    def shape(self):
        return (self.R, self.K)

    @property
    def device(self):
        return self.q.device

    @property
    def dtype(self):
        return "fp8_mx"

    @property
    def is_cuda(self):
        return self.q.is_cuda

    def data_ptr(self):
        return self.q.data_ptr()


def mx_scale_bytes(R: int, K: int) -> int:
    n = int(L.load().icap_mx_scale_bytes(R, K))
    if n == 0 and R * K:
        raise L.IcapError(f"mx_scale_bytes: K = {K} must be a multiple of 128")
    return n


def quantize_mx(x: Tensor, out: Optional[MXTensor] = None, rows: Optional[int] = None,
                rows_dev: Optional[Tensor] = None) -> MXTensor:
    """x [R, K] (f32 / bf16) -> MX e4m3 + E8M0 per-32 scales (icap_quantize_mx). rows_dev: device int32 row count
    (rows past it are not read)."""
    R = x.shape[0] if rows is None else rows
    K = x.shape[1]
    if out is None:
        out = MXTensor.empty(R, K, x.device)
    if out.R != R or out.K != K:
        raise L.IcapError("quantize_mx: output shape mismatch")
    call("icap_quantize_mx", dtype_code(x.dtype), R, K, x.data_ptr(), _ld(x), out.q.data_ptr(), _ld(out.q),
         out.scale.data_ptr(), _p(rows_dev), _stream())
    return out


def gemm(A: Tensor, B: Tensor, out: Tensor, *, bias: Optional[Tensor] = None, act: int = L.ACT_NONE,
         aux: Optional[Tensor] = None, dact: int = L.ACT_NONE, dact_src: Optional[Tensor] = None,
         resid: Optional[Tensor] = None, alpha: float = 1.0, beta: float = 0.0, drop: Dropout = NO_DROP,
         M: Optional[int] = None, N: Optional[int] = None, K: Optional[int] = None,
         alg_flops: Optional[float] = None, split_k: int = 0, m_dev: Optional[Tensor] = None,
         trans_ab: bool = False, ln: Optional[tuple] = None, workspace: Optional[Tensor] = None,
         tile_only: bool = False, g256: bool = False, g8p: int = 0, r256: bool = False, w192: bool = False,
         roles: int = 0, m_hint: Optional[int] = None,
         ln_fold: Optional[tuple] = None, ln_stats_out: Optional[Tensor] = None,
         ln_stats_in: Optional[Tensor] = None, ln_rows_out: Optional[tuple] = None,
         diag_stamps: Optional[Tensor] = None) -> Tensor:
    """out[M,N] = epi(alpha * A[M,K] @ B[N,K]^T) — see icap_gemm in include/icap.h.
    workspace: fp32 split-K scratch; by default one buffer per (device, stream), so GEMMs issued on different
    streams never share slabs (gemm_workspace). The split count depends on the shape alone, so the result is
    bitwise the same with any workspace; one too small for the shape's split raises.
    trans_ab: A and B are K-outer ([K, M] / [K, N] row-major: out = epi(alpha * A^T @ B)), bf16 only.
    ln: (gamma, beta, eps) — A is LayerNorm-ed over its K columns inside the GEMM (M <= 128 launches).
    ln_fold: (wsum, eps) — LayerNorm folded into the weights (fold_layernorm): B = W*gamma, bias = b + W.beta,
    out = rstd * (A.B^T - mean * wsum) + bias with A's row statistics taken in the launch (M <= 128 launches).
    alg_flops: algorithmic FLOPs when M/N/K include padding (vocab 50257->50304, dW rows -> multiple of 64).
    split_k: 0 = automatic split-K for launches of <= 64 output tiles, 1 = never, > 1 = forced.
    m_dev: device int32 row count <= M (rows past it are neither computed nor stored); m_hint: its expected value
    (kernel choice only).
    tile_only: the 128-row tile kernels only; g256: the 256 x 256 kernel wherever eligible; g8p = 128 / 256: the
    256-row 8-phase kernel with that tile width wherever eligible; r256: the 256 x 128 ring tile kernel (variant
    22) wherever eligible, unsplit (A/B measurements, path-equality tests); w192: 192 x 64 tiles (variant 24)
    wherever eligible, unsplit (same use); roles = 256 / 96 / 192: the split-role ring kernel on 128 x 256 (variant
    26) / 96 x 128 (variant 27) / 192 x 256 (variant 28) tiles wherever eligible, unsplit (same use); roles = 1 with
    trans_ab: the K-outer split-role kernel (variant 31, 128 x 128 tiles; split_k 0 = its own split rule); roles = 160:
    160 x 128 tiles (variant 32).
    ln_stats_out: fp32 [M, N/32, 2] — this (producer) launch also writes (mean, M2) of each row's 32-column groups of
    the stored C; ln_stats_in (with ln_fold = (wsum, eps)): the LayerNorm of A folded into the epilogue from the
    producer's statistics (tile kernels, any M); ln_rows_out: (mean, rstd) fp32 [M] of that LayerNorm (for its
    backward). include/icap.h icap_gemm_args.ln_stats_out."""
    mx = isinstance(A, MXTensor)
    if mx != isinstance(B, MXTensor):
        raise L.IcapError("gemm: A and B must both be MXTensor (fp8 MX) or both plain tensors")
    if trans_ab:
        M = A.shape[1] if M is None else M
        K = A.shape[0] if K is None else K
        N = B.shape[1] if N is None else N
    else:
        M = A.shape[0] if M is None else M
        K = A.shape[1] if K is None else K
        N = B.shape[0] if N is None else N
    a = GemmArgs()
    a.trans_ab = 1 if trans_ab else 0
    a.M, a.N, a.K = M, N, K
    a.c_dtype = dtype_code(out.dtype)
    if mx:
        if M != A.R or N != B.R or K != A.K or K != B.K:
            raise L.IcapError("gemm: MX operands are whole matrices (M, N, K must equal their shapes)")
        a.in_dtype = L.FP8_MX
        a.A, a.lda = A.q.data_ptr(), _ld(A.q)
        a.B, a.ldb = B.q.data_ptr(), _ld(B.q)
        a.a_scale, a.b_scale = A.scale.data_ptr(), B.scale.data_ptr()
    else:
        a.in_dtype = dtype_code(A.dtype)
        if B.dtype != A.dtype:
            raise L.IcapError("gemm: A and B must share a dtype")
        a.A, a.lda = A.data_ptr(), _ld(A)
        a.B, a.ldb = B.data_ptr(), _ld(B)
    a.C, a.ldc = out.data_ptr(), _ld(out)
    a.alpha, a.beta = alpha, beta
    a.bias = _p(bias)
    a.act = act
    if aux is not None:
        a.aux, a.ldaux = aux.data_ptr(), _ld(aux)
    a.dact = dact
    if dact_src is not None:
        a.dact_src, a.ld_dact = dact_src.data_ptr(), _ld(dact_src)
    if resid is not None:
        a.resid, a.ldr = resid.data_ptr(), _ld(resid)
    a.drop_p, a.seed, a.offset, a.seed_ptr = drop.p, drop.seed, drop.offset, drop.ptr
    ws = gemm_workspace(A.device, torch.cuda.current_stream(A.device) if A.is_cuda else None) \
        if workspace is None else workspace
    a.workspace, a.workspace_bytes, a.split_k = ws.data_ptr(), ws.numel() * 4, split_k
    tk = _gemm_tickets.get(ws.data_ptr())  # the workspace's zero-initialised split-K tickets (in-launch combine)
    if tk is not None and FUSED_SPLIT_K:
        a.tickets, a.tickets_len = tk.data_ptr(), tk.numel()
    a.m_dev = _p(m_dev)
    a.m_hint = int(m_hint) if (m_hint is not None and m_dev is not None) else 0
    a.path = (1 if tile_only else 3 if g256 else 4 if g8p == 128 else 5 if g8p == 256 else 6 if r256 else
              7 if w192 else 8 if roles == 256 else 9 if roles == 96 else 10 if roles == 192 else
              11 if roles == 1 else 12 if roles == 160 else 0)
    if ln is not None:
        a.ln_gamma, a.ln_beta, a.ln_eps = ln[0].data_ptr(), ln[1].data_ptr(), float(ln[2])
    if ln_fold is not None:
        a.ln_wsum, a.ln_eps = ln_fold[0].data_ptr(), float(ln_fold[1])
    if ln_stats_out is not None:
        a.ln_stats_out = ln_stats_out.data_ptr()
    if ln_stats_in is not None:
        a.ln_stats_in = ln_stats_in.data_ptr()
    if ln_rows_out is not None:
        a.ln_mean_out, a.ln_rstd_out = ln_rows_out[0].data_ptr(), ln_rows_out[1].data_ptr()
    if diag_stamps is not None:  # (read only by a -DICAP_STAMPS build: tools/gemm_stamps.py)
        a.diag_stamps = diag_stamps.data_ptr()
    if GEMM_TIMER is None:
        call("icap_gemm", C.byref(a), _stream())
    else:  # per-launch HIP-event timing (bench.py kernel roofline pass; never inside a captured graph)
        name = L.load().icap_gemm_kernel_name(C.byref(a))  # the instantiation rocprofv3 will name
        key = (name.decode() if name else "?",
               f"{M}x{N}x{K} act{act} dact{dact} drop{int(drop.p > 0)} res{int(resid is not None)} "
               f"aux{int(aux is not None)} beta{beta:g}{' m_dev' if m_dev is not None else ''}"
               f"{' kout' if trans_ab else ''}{' ln' if ln is not None else ''}{' lnfold' if ln_fold is not None else ''}"
               f"{' lnS' if ln_stats_out is not None else ''}{' lnF' if ln_stats_in is not None else ''}")
        GEMM_TIMER.launch(key, 2.0 * M * N * K if alg_flops is None else alg_flops,
                          lambda: call("icap_gemm", C.byref(a), _stream()))
    return out


def gemm_group(items) -> None:
    """K-outer weight-gradient products in one launch (include/icap.h icap_gemm_group): items = [(A, B, out, M, N, K,
    beta), ...] with out[M, N] = A^T B (+ beta out), A [K, M] and B [K, N] bf16 read in place, out fp32; 1 ... 8
    products, each bitwise what gemm(A, B, out, beta=beta, M=M, N=N, K=K, trans_ab=True, split_k=1, roles=1) gives."""
    n = len(items)
    arr = (GemmArgs * n)()
    for i, (A, B, out, M, N, K, beta) in enumerate(items):
        a = arr[i]
        a.trans_ab = 1
        a.M, a.N, a.K = M, N, K
        a.in_dtype, a.c_dtype = dtype_code(A.dtype), dtype_code(out.dtype)
        if B.dtype != A.dtype:
            raise L.IcapError("gemm_group: A and B must share a dtype")
        a.A, a.lda = A.data_ptr(), _ld(A)
        a.B, a.ldb = B.data_ptr(), _ld(B)
        a.C, a.ldc = out.data_ptr(), _ld(out)
        a.alpha, a.beta = 1.0, beta
        a.split_k = 1
    if GEMM_TIMER is None:
        call("icap_gemm_group", arr, n, _stream())
    else:
        key = ("icap::gemm_group_kernel(icap::GemmGroup)", " + ".join(f"{it[3]}x{it[4]}x{it[5]} kout" for it in items))
        GEMM_TIMER.launch(key, sum(2.0 * it[3] * it[4] * it[5] for it in items),
                          lambda: call("icap_gemm_group", arr, n, _stream()))


def ln_fold_ok(D: int) -> bool:
    """The LayerNorm-statistics hand-off's shape rule (csrc/gemm.hip gemm_plan): the producer stores (mean, M2) per
    32-column group (N % 32 == 0) and the consumer tile GEMM combines them in its prologue, K % 128 == 0 and
    K <= 1280. A model whose width breaks it (e.g. GPT-2 XL's 1600, or 192) keeps the standalone LayerNorm launches."""
    return D % 128 == 0 and D <= 1280


GEMM_WORKSPACE_BYTES = 192 << 20  # split-K slabs up to splits*M*N fp32 (LM-head dX: 6 x 6400 x 768)
GEMM_TICKETS = 1 << 16  # int32 per-tile counters of the in-launch split-K combine (2 per 128 x 128 tile)
# False: split-K always through a reduce pass (module constant for A/B tools; the two forms are bitwise equal)
FUSED_SPLIT_K = True
_gemm_ws = {}
_gemm_tickets = {}  # workspace data_ptr -> its tickets (zeroed once; every launch leaves them zero)


def _new_workspace(device) -> Tensor:
    ws = torch.empty(GEMM_WORKSPACE_BYTES // 4, dtype=torch.float32, device=device)
    _gemm_tickets[ws.data_ptr()] = torch.zeros(GEMM_TICKETS, dtype=torch.int32, device=device)
    return ws


def gemm_workspace(device, stream=None) -> Tensor:
    """fp32 split-K scratch of one (device, stream): launches ordered on one stream reuse a buffer safely, and
    eager launches on two streams get two buffers, so concurrent split-K GEMMs never overwrite each other's slabs
    (a GEMM's slabs are written and reduced inside its own stream-ordered launches).
    Under HIP-graph capture no memory may be allocated (a block of the graph's private pool outlives the graph
    here and aborts the allocator when that graph is destroyed), so every capture uses one per-device graph
    buffer, allocated with the device's first eager buffer: graphs replayed one after another (the trainer's step
    / segment graphs, decode chunks) share it as eager launches on one stream share theirs; two graphs that
    contain split-K GEMMs must not be replayed concurrently on different streams. A side stream registered with
    register_side_stream (a concurrent branch inside one captured graph: the trainer's weight-gradient stream)
    has a graph buffer of its own."""
    sid = 0 if stream is None else int(stream.cuda_stream)
    if stream is not None and torch.cuda.is_current_stream_capturing():
        ws = _gemm_ws.get((device.type, device.index, "graph", sid))
        if ws is None:
            ws = _gemm_ws.get((device.type, device.index, "graph"))
        if ws is None:
            raise L.IcapError("gemm: a split-K workspace is needed inside graph capture; run one eager GEMM on "
                              "this device first (or pass workspace=)")
        return ws
    key = (device.type, device.index, sid)
    ws = _gemm_ws.get(key)
    if ws is None:
        ws = _new_workspace(device)
        _gemm_ws[key] = ws
        gkey = (device.type, device.index, "graph")
        if stream is not None and gkey not in _gemm_ws:
            _gemm_ws[gkey] = _new_workspace(device)
    return ws


_KEPT_EVENTS = []
KEEP_EVENTS = 4096  # events kept alive (a few steps' worth of the trainer's cross-stream waits)


def keep_event(ev) -> None:
    """Hold a reference to a cross-stream event until KEEP_EVENTS newer ones exist: destroying a HIP event while a
    stream's wait on it is still queued can let that wait go early, so the trainer's fork / join events outlive
    the work they order (a step records ~70; this keeps dozens of steps)."""
    _KEPT_EVENTS.append(ev)
    if len(_KEPT_EVENTS) > KEEP_EVENTS:
        del _KEPT_EVENTS[: KEEP_EVENTS // 2]


def register_side_stream(stream) -> None:
    """Give `stream` its own eager and graph-capture split-K workspaces (allocated now, outside any capture), so
    GEMMs it runs concurrently with the capture stream's inside one graph never share slabs or tickets."""
    dev = stream.device
    gemm_workspace(dev, stream)
    gkey = (dev.type, dev.index, "graph", int(stream.cuda_stream))
    if gkey not in _gemm_ws:
        _gemm_ws[gkey] = _new_workspace(dev)


GEMM_TIMER = None  # set to an object with .launch(key, flops, fn) to time every GEMM (and attention) launch
TIMER_TAG = None  # label the timer records of the launches issued inside timer_tag(...) (bench roofline groups)
TAG_HOOK = None  # bench.py: callable(tag, entering) run at each timer_tag boundary (marker launches in a graph)


@contextlib.contextmanager
def timer_tag(tag: str):
    """Label every launch GEMM_TIMER records in this block (e.g. "gpt2_block": bench.py's GPT-2-block roofline)."""
    global TIMER_TAG
    old, TIMER_TAG = TIMER_TAG, tag
    if TAG_HOOK is not None:
        TAG_HOOK(tag, True)
    try:
        yield
    finally:
        TIMER_TAG = old
        if TAG_HOOK is not None:
            TAG_HOOK(tag, False)


def _timed(kind: str, desc: str, flops: Optional[float], fn) -> None:
    """Run fn (one C-ABI launch); under GEMM_TIMER with HIP events around it (never inside a captured graph)."""
    if GEMM_TIMER is None or flops is None:
        fn()
    else:
        GEMM_TIMER.launch((kind, desc), flops, fn)


def layernorm_fwd(x: Tensor, gamma: Tensor, beta: Tensor, eps: float, y: Tensor, mean: Optional[Tensor],
                  rstd: Optional[Tensor], rows: Optional[int] = None, y_rowmap: Optional[Tensor] = None,
                  rows_dev: Optional[Tensor] = None) -> Tensor:
    """y_rowmap: int32 [rows]; row r goes to y row y_rowmap[r] (skipped when < 0).
    rows_dev: device int32 row count <= rows (packed token rows): rows past it are untouched."""
    rows = _rows(x) if rows is None else rows
    D = gamma.shape[0]
    call("icap_layernorm_fwd", dtype_code(x.dtype), rows, D, x.data_ptr(), _ld(x), gamma.data_ptr(),
         beta.data_ptr(), eps, y.data_ptr(), _ld(y), _p(mean), _p(rstd), _p(y_rowmap), _p(rows_dev), _stream())
    return y


def layernorm_bwd_workspace(rows: int, D: int) -> int:
    return int(L.load().icap_layernorm_bwd_workspace_bytes(rows, D))


def layernorm_bwd(x: Tensor, gamma: Tensor, mean: Tensor, rstd: Tensor, dy: Tensor, dx: Tensor, *,
                  dres: Optional[Tensor] = None, dx_drop: Optional[Tensor] = None, drop: Dropout = NO_DROP,
                  dgamma: Optional[Tensor] = None, dbeta: Optional[Tensor] = None,
                  workspace: Optional[Tensor] = None, rows: Optional[int] = None,
                  dy_rowmap: Optional[Tensor] = None, rows_dev: Optional[Tensor] = None,
                  param_accumulate: bool = True, defer_params: bool = False) -> Tensor:
    """dy_rowmap: int32 [rows]; dy of row r is dy row dy_rowmap[r] (zero when < 0). rows_dev: as layernorm_fwd.
    param_accumulate: dgamma / dbeta += (True) or = (False: the first micro-batch of a cycle).
    defer_params: leave the dgamma / dbeta partials in `workspace` for ln_param_reduce_batch (no reduce launch)."""
    rows = _rows(x) if rows is None else rows
    D = gamma.shape[0]
    call("icap_layernorm_bwd", dtype_code(x.dtype), rows, D, x.data_ptr(), _ld(x), gamma.data_ptr(),
         mean.data_ptr(), rstd.data_ptr(), dy.data_ptr(), _ld(dy), _p(dres), _ld(dres) if dres is not None else 0,
         dx.data_ptr(), _ld(dx), _p(dx_drop), drop.p, drop.seed, drop.offset, drop.ptr, _p(dgamma), _p(dbeta),
         _p(workspace), _p(dy_rowmap), _p(rows_dev), (0 if param_accumulate else 1) | (2 if defer_params else 0),
         _stream())
    return dx


def ln_param_reduce_batch(items) -> None:
    """The deferred dgamma / dbeta reduces of several layernorm_bwd(..., defer_params=True) calls in one launch
    (include/icap.h icap_ln_param_reduce_batch): items = [(workspace, rows, D, dgamma, dbeta, accumulate), ...];
    bitwise the per-call reduce."""
    n = len(items)
    if n == 0:
        return
    arr = (L.LnParamItem * n)()
    for i, (ws, rows, D, dg, db, acc) in enumerate(items):
        arr[i].workspace, arr[i].rows, arr[i].D = ws.data_ptr(), rows, D
        arr[i].dgamma, arr[i].dbeta, arr[i].overwrite = _p(dg), _p(db), 0 if acc else 1
    call("icap_ln_param_reduce_batch", n, arr, _stream())


def _attn_args(qkv: Tensor, B: int, S: int, H: int, hd: int, rsb: int, rss: int, scale: float, causal: bool,
               key_mask: Optional[Tensor], lse: Optional[Tensor], drop: Dropout, seqs=None,
               short_only: bool = False) -> AttnArgs:
    a = AttnArgs()
    if seqs is not None:  # packed sequences: (seq_off, seq_len) int32 [B] (icap_caption_pack)
        a.seq_off, a.seq_len = seqs[0].data_ptr(), seqs[1].data_ptr()
        a.short_only = 1 if short_only else 0
    a.dtype = dtype_code(qkv.dtype)
    a.B, a.S, a.H, a.hd = B, S, H, hd
    a.row_stride_b, a.row_stride_s = rsb, rss
    a.qkv, a.ld_qkv = qkv.data_ptr(), _ld(qkv)
    a.lse = _p(lse)
    a.key_mask = _p(key_mask)
    a.causal = 1 if causal else 0
    a.scale = scale
    a.drop_p, a.seed, a.offset, a.seed_ptr = drop.p, drop.seed, drop.offset, drop.ptr
    return a


def attention_fwd(qkv: Tensor, out: Tensor, *, B: int, S: int, H: int, hd: int, scale: float,
                  causal: bool = False, key_mask: Optional[Tensor] = None, lse: Optional[Tensor] = None,
                  drop: Dropout = NO_DROP, rsb: Optional[int] = None, rss: int = 1, seqs=None,
                  alg_flops: Optional[float] = None, short_only: bool = False) -> Tensor:
    """seqs: (seq_off, seq_len) device int32 [B] — packed sequences (include/icap.h icap_attn_args).
    short_only (packed): the caller guarantees every seq_len <= 32 — only the short-sequence pass is launched.
    alg_flops: algorithmic FLOPs of the launch (bench timing only; None: not timed)."""
    a = _attn_args(qkv, B, S, H, hd, S if rsb is None else rsb, rss, scale, causal, key_mask, lse, drop, seqs,
                   short_only)
    a.out, a.ld_out = out.data_ptr(), _ld(out)
    _timed("attn_fwd", f"B{B} S{S} H{H} hd{hd}{' packed' if seqs is not None else ''}", alg_flops,
           lambda: call("icap_attention_fwd", C.byref(a), _stream()))
    return out


def attention_bwd(qkv: Tensor, dout: Tensor, lse: Tensor, dqkv: Tensor, *, B: int, S: int, H: int, hd: int,
                  scale: float, causal: bool = False, key_mask: Optional[Tensor] = None, drop: Dropout = NO_DROP,
                  rsb: Optional[int] = None, rss: int = 1, out: Optional[Tensor] = None, seqs=None,
                  alg_flops: Optional[float] = None, short_only: bool = False) -> Tensor:
    """out: the forward's O (optional; enables the transpose-free bf16 MFMA backward). seqs, short_only: as
    attention_fwd."""
    a = _attn_args(qkv, B, S, H, hd, S if rsb is None else rsb, rss, scale, causal, key_mask, lse, drop, seqs,
                   short_only)
    if out is not None:
        a.out, a.ld_out = out.data_ptr(), _ld(out)
    a.dout, a.ld_dout = dout.data_ptr(), _ld(dout)
    a.dqkv, a.ld_dqkv = dqkv.data_ptr(), _ld(dqkv)
    _timed("attn_bwd", f"B{B} S{S} H{H} hd{hd}{' packed' if seqs is not None else ''}", alg_flops,
           lambda: call("icap_attention_bwd", C.byref(a), _stream()))
    return dqkv


def attention_decode(cache: Tensor, out: Tensor, *, B: int, H: int, hd: int, pos: int, scale: float,
                     anc: Optional[Tensor] = None) -> Tensor:
    """anc: int32 [>= pos+1, B] KV ancestry (beam search; include/icap.h icap_attention_decode_anc)."""
    if anc is None:
        call("icap_attention_decode", dtype_code(cache.dtype), B, H, hd, pos, cache.data_ptr(), _ld(cache),
             out.data_ptr(), _ld(out), scale, _stream())
    else:
        if anc.dtype != torch.int32 or anc.numel() < (pos + 1) * B:
            raise L.IcapError("attention_decode: anc must be int32 with >= (pos+1)*B entries")
        call("icap_attention_decode_anc", dtype_code(cache.dtype), B, H, hd, pos, cache.data_ptr(), _ld(cache),
             anc.data_ptr(), out.data_ptr(), _ld(out), scale, _stream())
    return out


# ---------------------------------------------------------------------------------------------- beam search
BEAM_LAYOUT_FIELDS = ("run_score", "run_seq", "fin_score", "fin_len", "fin_seq", "fin_cnt", "done", "anc", "total")


def beam_layout(B: int, W: int, T: int, max_len: int) -> dict:
    """The beam workspace's word offsets as beam.hip lays it out (icap_beam_layout)."""
    offs = (C.c_int64 * 9)()
    if L.load().icap_beam_layout(B, W, T, max_len, offs) != 0:  # host-only query (also in dry runs)
        raise L.IcapError(f"icap_beam_layout failed: {L.last_error()}")
    return dict(zip(BEAM_LAYOUT_FIELDS, list(offs)))


class BeamState:
    """Device state of one beam search (include/icap.h icap_beam_*): B captions x W beams, token budget
    max_len, T = P + max_len cache positions. Owns the workspace and the per-row candidate buffers."""

    def __init__(self, B: int, W: int, V: int, max_len: int, T: int, eos: int, length_penalty: float,
                 dev: torch.device):
        self.B, self.W, self.V, self.max_len, self.T = B, W, V, max_len, T
        self.K = 8 if W <= 4 else 16
        R = B * W
        nbytes = int(L.load().icap_beam_workspace_bytes(B, W, T, max_len))
        if nbytes == 0:
            raise L.IcapError("beam: bad sizes")
        self.ws = torch.empty(nbytes // 4, dtype=torch.int32, device=dev)
        self.top_val = torch.empty((R, self.K), dtype=torch.float32, device=dev)
        self.top_idx = torch.empty((R, self.K), dtype=torch.int32, device=dev)
        self.top_m = torch.empty(R, dtype=torch.float32, device=dev)
        self.top_ls = torch.empty(R, dtype=torch.float32, device=dev)
        self.out = torch.empty((B, max_len), dtype=torch.int64, device=dev)
        self.out_len = torch.empty(B, dtype=torch.int32, device=dev)
        self.args = L.BeamArgs()
        a = self.args
        a.B, a.W, a.V, a.max_len, a.eos, a.length_penalty, a.K, a.T = B, W, V, max_len, eos, float(length_penalty), \
            self.K, T
        a.top_val, a.top_idx = self.top_val.data_ptr(), self.top_idx.data_ptr()
        a.top_m, a.top_ls = self.top_m.data_ptr(), self.top_ls.data_ptr()
        a.ws = self.ws.data_ptr()
        # word offsets of the per-caption done flags and the ancestry table, from the library (icap_beam_layout)
        offs = beam_layout(B, W, T, max_len)
        self.done = self.ws[offs["done"]: offs["done"] + B]
        self.anc = self.ws[offs["anc"]: offs["anc"] + T * R]

    def set_embedding(self, dtype: torch.dtype, D: int, n_positions: int, wte: Tensor, wpe: Tensor,
                      x: Optional[Tensor]) -> None:
        a = self.args
        a.dtype, a.D, a.n_positions = dtype_code(dtype), D, n_positions
        a.wte, a.wpe, a.x = wte.data_ptr(), wpe.data_ptr(), _p(x)

    def init(self, P: int) -> None:
        call("icap_beam_init", C.byref(self.args), P, _stream())

    def step(self, logits: Tensor, step: int, pos: int, x: Optional[Tensor]) -> None:
        R = self.B * self.W
        call("icap_beam_rowtop", dtype_code(logits.dtype), R, self.V, logits.data_ptr(), _ld(logits), self.K,
             self.top_val.data_ptr(), self.top_idx.data_ptr(), self.top_m.data_ptr(), self.top_ls.data_ptr(),
             _stream())
        self.args.x = _p(x)
        call("icap_beam_update", C.byref(self.args), step, pos, _stream())

    def finalize(self) -> Tuple[Tensor, Tensor]:
        call("icap_beam_finalize", C.byref(self.args), self.out.data_ptr(), self.out_len.data_ptr(), _stream())
        return self.out, self.out_len


def gpt2_embed(prefix: Optional[Tensor], prefix_bstride: int, wte: Tensor, wpe: Tensor, ids: Optional[Tensor],
               x: Tensor, *, B: int, P: int, L_: int, D: int, drop: Dropout = NO_DROP, seqs=None) -> Tensor:
    """seqs: (seq_off, seq_len) — write the live tokens of each sequence at its packed rows."""
    so, sl = (seqs[0].data_ptr(), seqs[1].data_ptr()) if seqs is not None else (None, None)
    call("icap_gpt2_embed", dtype_code(x.dtype), B, P, L_, D, _p(prefix), prefix_bstride, wte.data_ptr(),
         wpe.data_ptr(), _p(ids), x.data_ptr(), drop.p, drop.seed, drop.offset, drop.ptr, so, sl, _stream())
    return x


def caption_prep(B: int, P: int, L_: int, mask: Optional[Tensor], labels: Optional[Tensor],
                 key_mask: Optional[Tensor], labels_shift: Optional[Tensor], n_valid: Optional[Tensor],
                 row_slot: Optional[Tensor] = None, labels_compact: Optional[Tensor] = None) -> None:
    """row_slot/labels_compact: the target-row compaction (include/icap.h icap_caption_prep)."""
    for t in (mask, labels):
        if t is not None and t.dtype != torch.int64:
            raise L.IcapError("caption_prep: mask/labels must be int64")
    call("icap_caption_prep", B, P, L_, _p(mask), _p(labels), _p(key_mask), _p(labels_shift), _p(n_valid),
         _p(row_slot), _p(labels_compact), _stream())


def caption_pack(B: int, P: int, L_: int, mask: Optional[Tensor], labels: Tensor, seq_off: Tensor, seq_len: Tensor,
                 m_live: Tensor, key_mask: Tensor, labels_shift: Tensor, n_valid: Optional[Tensor],
                 row_slot: Optional[Tensor] = None, labels_compact: Optional[Tensor] = None) -> None:
    """Packed token rows of a training batch (include/icap.h icap_caption_pack): each sequence keeps its prefix
    and caption positions up to the last loss target; offsets, lengths and the live row count on the device."""
    for t in (mask, labels):
        if t is not None and t.dtype != torch.int64:
            raise L.IcapError("caption_pack: mask/labels must be int64")
    for t in (seq_off, seq_len, m_live, key_mask, labels_shift):
        if t.dtype != torch.int32:
            raise L.IcapError("caption_pack: outputs must be int32")
    call("icap_caption_pack", B, P, L_, _p(mask), _p(labels), seq_off.data_ptr(), seq_len.data_ptr(),
         m_live.data_ptr(), key_mask.data_ptr(), labels_shift.data_ptr(), _p(n_valid), _p(row_slot),
         _p(labels_compact), _stream())


def rows_unpack(src: Tensor, seq_off: Tensor, seq_len: Tensor, dst: Tensor, *, B: int, P: int, D: int,
                dst_bstride: int) -> Tensor:
    """dst[b, t] = src[seq_off[b] + t] for the P prefix rows of each packed sequence (zero when absent)."""
    if src.dtype != dst.dtype:
        raise L.IcapError("rows_unpack: src and dst must share a dtype")
    call("icap_rows_unpack", dtype_code(src.dtype), B, P, D, src.data_ptr(), seq_off.data_ptr(), seq_len.data_ptr(),
         dst.data_ptr(), dst_bstride, _stream())
    return dst


def cross_entropy_workspace(rows: int) -> int:
    return int(L.load().icap_cross_entropy_workspace_bytes(rows))


def cross_entropy(logits: Tensor, V: int, labels: Tensor, n_valid: Tensor, loss: Tensor,
                  dlogits: Optional[Tensor], workspace: Tensor, grad_scale: float = 1.0,
                  rows: Optional[int] = None, rows_dev: Optional[Tensor] = None) -> Tensor:
    """rows_dev: device int32 row count (compacted targets); rows past it are untouched."""
    rows = logits.shape[0] if rows is None else rows
    call("icap_cross_entropy", dtype_code(logits.dtype), rows, V, logits.data_ptr(), _ld(logits),
         labels.data_ptr(), n_valid.data_ptr(), loss.data_ptr(), _p(dlogits), grad_scale, workspace.data_ptr(),
         _p(rows_dev), _stream())
    return loss


def adamw_workspace(n: int) -> int:
    return int(L.load().icap_adamw_workspace_bytes(n))


def adamw_step(params: Tensor, grads: Tensor, exp_avg: Tensor, exp_avg_sq: Tensor, state: Tensor,
               workspace: Tensor, *, lr: float, betas=(0.9, 0.999), eps: float = 1e-8,
               weight_decay: float = 0.01, max_norm: float = 1.0, num_warmup_steps: int = 0,
               num_training_steps: int = 1, bf16_out: Optional[Tensor] = None) -> None:
    a = AdamWArgs()
    a.n = params.numel()
    a.params, a.grads, a.exp_avg, a.exp_avg_sq = (params.data_ptr(), grads.data_ptr(), exp_avg.data_ptr(),
                                                  exp_avg_sq.data_ptr())
    a.bf16_out = _p(bf16_out)
    a.state = state.data_ptr()
    a.lr, a.beta1, a.beta2, a.eps, a.weight_decay = lr, betas[0], betas[1], eps, weight_decay
    a.max_norm = max_norm
    a.num_warmup_steps, a.num_training_steps = num_warmup_steps, num_training_steps
    call("icap_adamw_step", C.byref(a), workspace.data_ptr(), _stream())


def sqnorm(x: Tensor, out: Tensor, workspace: Tensor) -> Tensor:
    call("icap_sqnorm", x.numel(), x.data_ptr(), out.data_ptr(), workspace.data_ptr(), _stream())
    return out


def transpose(src: Tensor, dst: Tensor, rows_pad: Optional[int] = None, rows: Optional[int] = None,
              cols: Optional[int] = None) -> Tensor:
    rows = src.shape[0] if rows is None else rows
    cols = src.shape[1] if cols is None else cols
    call("icap_transpose", dtype_code(src.dtype), rows, cols, src.data_ptr(), _ld(src), dst.data_ptr(), _ld(dst),
         rows if rows_pad is None else rows_pad, _stream())
    return dst


def transpose_batch(pairs) -> None:
    """dst = src^T for every (src, dst) of bf16 matrices in one launch (icap_transpose_batch; items it cannot tile
    fall back to icap_transpose inside the library)."""
    pairs = list(pairs)
    if not pairs:
        return
    items = (L.TransposeItem * len(pairs))()
    for it, (src, dst) in zip(items, pairs):
        if src.dtype != torch.bfloat16 or dst.dtype != torch.bfloat16:
            raise L.IcapError("transpose_batch: bf16 matrices only")
        it.src, it.lds, it.dst, it.ldd = src.data_ptr(), _ld(src), dst.data_ptr(), _ld(dst)
        it.rows, it.cols = src.shape[0], src.shape[1]
    call("icap_transpose_batch", len(pairs), C.cast(items, C.c_void_p), _stream())


def colsum_workspace(M: int, N: int) -> int:
    return int(L.load().icap_colsum_workspace_bytes(M, N))


def colsum(src: Tensor, out: Tensor, workspace: Tensor, accumulate: bool = True, M: Optional[int] = None,
           N: Optional[int] = None) -> Tensor:
    M = src.shape[0] if M is None else M
    N = src.shape[1] if N is None else N
    call("icap_colsum", dtype_code(src.dtype), M, N, src.data_ptr(), _ld(src), out.data_ptr(),
         1 if accumulate else 0, workspace.data_ptr(), _stream())
    return out


COLSUM_BATCH = 16  # include/icap.h ICAP_COLSUM_BATCH


def colsum_batch(items, M: int, workspace: Tensor, accumulate: bool = True) -> None:
    """out (+)= colsum(src[:M, :N]) for every (src, out, N) (N None = src.shape[1]) over the same M rows, in two
    launches (icap_colsum_batch; bitwise what icap_colsum gives per item). Items the batched kernel cannot take
    (N or ld not a multiple of 4, a misaligned src, mixed dtypes) go through icap_colsum one by one."""
    items = [(s, o, s.shape[1] if n is None else n) for s, o, n in items]
    if not items:
        return
    dt = items[0][0].dtype
    ok = [it for it in items if it[0].dtype == dt and it[2] % 4 == 0 and _ld(it[0]) % 4 == 0
          and it[0].data_ptr() % (4 * it[0].element_size()) == 0]
    for s, o, n in items:
        if not any(s is t[0] and o is t[1] for t in ok):
            colsum(s, o, workspace, accumulate=accumulate, M=M, N=n)
    for i in range(0, len(ok), COLSUM_BATCH):
        part = ok[i: i + COLSUM_BATCH]
        arr = (L.ColsumItem * len(part))()
        for it, (s, o, n) in zip(arr, part):
            it.src, it.ld, it.N, it.out = s.data_ptr(), _ld(s), n, o.data_ptr()
        call("icap_colsum_batch", dtype_code(dt), M, len(part), C.cast(arr, C.c_void_p), 1 if accumulate else 0,
             workspace.data_ptr(), _stream())


def dropout_apply(src: Tensor, dst: Tensor, drop: Dropout, M: Optional[int] = None,
                  N: Optional[int] = None) -> Tensor:
    M = src.shape[0] if M is None else M
    N = src.shape[1] if N is None else N
    call("icap_dropout_apply", dtype_code(src.dtype), M, N, src.data_ptr(), _ld(src), dst.data_ptr(), _ld(dst),
         drop.p, drop.seed, drop.offset, drop.ptr, _stream())
    return dst


def counter_increment(counter: Tensor) -> None:
    call("icap_counter_increment", counter.data_ptr(), _stream())


def convert(src: Tensor, dst: Tensor) -> Tensor:
    """dst = src cast to dst.dtype (2-D, strided rows)."""
    s2 = src if src.dim() == 2 else src.reshape(-1, src.shape[-1])
    d2 = dst if dst.dim() == 2 else dst.reshape(-1, dst.shape[-1])
    call("icap_convert", dtype_code(src.dtype), dtype_code(dst.dtype), s2.shape[0], s2.shape[1], s2.data_ptr(),
         _ld(s2), d2.data_ptr(), _ld(d2), _stream())
    return dst


def broadcast_rows(src: Tensor, dst: Tensor, B: int, dst_bstride: int) -> Tensor:
    R, D = src.shape
    call("icap_broadcast_rows", dtype_code(dst.dtype), B, R, D, src.data_ptr(), dst.data_ptr(), dst_bstride,
         _stream())
    return dst


def patch_embed(pixels: Tensor, w: Tensor, out: Tensor, *, patch: int, prefix: Optional[Tensor],
                pos: Optional[Tensor] = None, bias: Optional[Tensor] = None) -> Tensor:
    """Patch Conv2d (stride = kernel = patch) + token assembly in one launch (include/icap.h icap_patch_embed):
    out[b*S + r] = prefix[r] (+ pos[r]) for r < NP, out[b*S + NP + i] = patch_i . w^T (+ bias) (+ pos[NP + i]).
    pixels fp32 [B, C, H, H]; w bf16 [N, Kp] in (c, ky, kx) order, zero past C*p*p; out bf16 [B*S, N]."""
    if pixels.dtype != torch.float32 or not pixels.is_contiguous() or pixels.dim() != 4:
        raise L.IcapError("patch_embed: pixels must be contiguous fp32 [B,C,H,H]")
    if w.dtype != torch.bfloat16 or out.dtype != torch.bfloat16:
        raise L.IcapError("patch_embed: w and out must be bf16")
    B, Cc, H, W = pixels.shape
    if H != W:  # the kernel indexes the pixels as H x H
        raise L.IcapError("patch_embed: pixels must be square [B,C,H,H]")
    NP = 0 if prefix is None else prefix.shape[0]
    N = w.shape[0]
    S = NP + (H // patch) ** 2
    if out.shape[0] < B * S or out.shape[1] < N:
        raise L.IcapError("patch_embed: out is too small")
    for t in (prefix, pos, bias):
        if t is not None and (t.dtype != torch.float32 or not t.is_contiguous()):
            raise L.IcapError("patch_embed: prefix / pos / bias must be contiguous fp32")
    # every per-column operand is indexed with stride N = w.shape[0] (the output columns)
    if pos is not None and (pos.shape[-1] != N or pos.numel() < S * N):
        raise L.IcapError("patch_embed: pos must be [S, N] with N = w.shape[0]")
    if prefix is not None and prefix.shape[-1] != N:
        raise L.IcapError("patch_embed: prefix must be [NP, N] with N = w.shape[0]")
    if bias is not None and bias.numel() < N:
        raise L.IcapError("patch_embed: bias must hold N = w.shape[0] values")
    call("icap_patch_embed", B, Cc, H, patch, NP, N, pixels.data_ptr(), w.data_ptr(), _ld(w), w.shape[1], _p(bias),
         _p(pos), _p(prefix), out.data_ptr(), _ld(out), _stream())
    return out


def im2col_patches(pixels: Tensor, patches: Tensor, patch: int) -> Tensor:
    B, Cc, H, W = pixels.shape
    if H != W or pixels.dtype != torch.float32 or not pixels.is_contiguous():
        raise L.IcapError("im2col_patches: pixels must be contiguous fp32 [B,C,H,H]")
    call("icap_im2col_patches", dtype_code(patches.dtype), B, Cc, H, patch, pixels.data_ptr(), patches.data_ptr(),
         _stream())
    return patches


def vit_embed(patch_emb: Tensor, cls: Tensor, pos: Tensor, x: Tensor, B: int, G2: int, D: int) -> Tensor:
    call("icap_vit_embed", dtype_code(x.dtype), B, G2, D, patch_emb.data_ptr(), cls.data_ptr(), pos.data_ptr(),
         x.data_ptr(), _stream())
    return x


def prefix_embed(patch_emb: Tensor, prefix: Tensor, x: Tensor, B: int, G2: int, D: int,
                 pos: Optional[Tensor] = None) -> Tensor:
    """x[b] = [prefix tokens (fp32 [NP, D]) || patch_emb rows of image b] (+ pos) — icap_prefix_embed."""
    call("icap_prefix_embed", dtype_code(x.dtype), B, G2, prefix.shape[0], D, patch_emb.data_ptr(),
         prefix.data_ptr(), _p(pos), x.data_ptr(), _stream())
    return x


def rope_patches(qkv: Tensor, cos: Tensor, sin: Tensor, *, B: int, S: int, NP: int, H: int, hd: int) -> Tensor:
    """In-place rotary embedding of the patch rows' q and k (icap_rope_patches)."""
    call("icap_rope_patches", dtype_code(qkv.dtype), B, S, NP, H, hd, qkv.data_ptr(), _ld(qkv), cos.data_ptr(),
         sin.data_ptr(), _stream())
    return qkv


def l2norm_rows(x: Tensor, out: Tensor, rows: Optional[int] = None) -> Tensor:
    rows = x.shape[0] if rows is None else rows
    call("icap_l2norm_rows", dtype_code(x.dtype), rows, x.shape[-1], x.data_ptr(), _ld(x), out.data_ptr(),
         _ld(out), _stream())
    return out


def greedy_next(logits: Tensor, V: int, eos: int, finished: Tensor, tokens: Tensor, step: int,
                wte: Optional[Tensor], wpe: Optional[Tensor], pos: int, D: int, x: Optional[Tensor],
                forced: Optional[Tensor] = None) -> None:
    B = finished.shape[0]
    call("icap_greedy_next", dtype_code(logits.dtype), B, V, logits.data_ptr(), _ld(logits), eos, _p(forced),
         finished.data_ptr(), tokens.data_ptr(), _ld(tokens), step, _p(wte), _p(wpe), pos, D, _p(x), _stream())


def topp_sample(logits: Tensor, V: int, temperature: float, top_p: float, finished: Optional[Tensor], seed: int,
                step: int, eos: int, out: Tensor, seed_ptr: Optional[Tensor] = None) -> Tensor:
    """Temperature + nucleus draw of one token per row (src/models.py:400-449) -> out int64 [B]."""
    B = out.shape[0]
    if B and logits.shape[0] < B:
        raise ValueError("topp_sample: logits has fewer rows than out")
    call("icap_topp_sample", dtype_code(logits.dtype), B, V, logits.data_ptr(), _ld(logits), float(temperature),
         float(top_p), _p(finished), seed & (2**64 - 1), _p(seed_ptr), step, eos, out.data_ptr(), _stream())
    return out


def add_position(src: Tensor, src_bstride: int, src_tstride: int, wpe: Tensor, x: Tensor, *, B: int, npos: int,
                 D: int, pos0: int) -> Tensor:
    call("icap_add_position", dtype_code(x.dtype), B, npos, D, src.data_ptr(), src_bstride, src_tstride,
         wpe.data_ptr(), pos0, x.data_ptr(), _stream())
    return x


def embedding_scatter_add(dx: Tensor, ids: Tensor, dwte: Tensor, *, B: int, P: int, L_: int, D: int) -> Tensor:
    call("icap_embedding_scatter_add", dtype_code(dx.dtype), B, P, L_, D, dx.data_ptr(), ids.data_ptr(),
         dwte.data_ptr(), _stream())
    return dwte


# ---------------------------------------------------------------------------------------------- CLIP input
def _pillow_window(in_size: int, out_size: int, xx: int):
    """Pillow Resample.c precompute_coeffs window of output index xx: (xmin, taps) (same double math)."""
    scale = in_size / out_size
    filterscale = max(scale, 1.0)
    support = 2.0 * filterscale
    center = (xx + 0.5) * scale
    xmin = max(int(center - support + 0.5), 0)
    xmax = min(int(center + support + 0.5), in_size)
    return xmin, xmax - xmin


def clip_preprocess_geometry(sizes, size: int = 224, crop: int = 224):
    """Per image (h, w): the int64 geo row icap_clip_preprocess takes, and the tmp rows it needs."""
    from .clip import resize_shortest_edge

    geo, src_off, tmp_off = [], 0, 0
    for h, w in sizes:
        new_w, new_h = resize_shortest_edge((w, h), size)
        if new_w < crop or new_h < crop:
            raise L.IcapError(f"clip_preprocess: resized {new_w}x{new_h} is smaller than the {crop} crop")
        top, left = (new_h - crop) // 2, (new_w - crop) // 2
        if new_h == h:
            y_first, rows = top, crop
        else:
            y_first = _pillow_window(h, new_h, top)[0]
            lo, n = _pillow_window(h, new_h, top + crop - 1)
            rows = lo + n - y_first
        geo.append([src_off, h, w, new_h, new_w, top, left, tmp_off, y_first, rows])
        src_off += h * w * 3
        tmp_off += rows * crop * 3
    return geo, tmp_off


def clip_preprocess(images, device, size: int = 224, crop: int = 224, mean=None, std=None) -> Tensor:
    """Decoded RGB uint8 images ([H, W, 3] numpy / torch, any sizes) -> fp32 [n, 3, crop, crop] on `device`,
    equal to CLIPImageProcessor(images).pixel_values (src/embeddings/clip.py:129; PIL-backed HF processor)."""
    import numpy as np

    arrs = [np.ascontiguousarray(np.asarray(im, dtype=np.uint8)) for im in images]
    for a in arrs:
        if a.ndim != 3 or a.shape[2] != 3:
            raise L.IcapError("clip_preprocess: images must be RGB uint8 [H, W, 3]")
    if not arrs:
        return torch.empty((0, 3, crop, crop), dtype=torch.float32, device=device)
    packed = torch.from_numpy(np.concatenate([a.reshape(-1) for a in arrs]))
    return clip_preprocess_packed(packed, [a.shape[:2] for a in arrs], device, size, crop, mean, std)


_NORM_CONSTS = {}


def _norm_consts(device, mean: tuple, std: tuple):
    """(mean, std) fp32 device tensors, uploaded once per (device, values)."""
    key = (str(torch.device(device)), mean, std)
    if key not in _NORM_CONSTS:
        _NORM_CONSTS[key] = (torch.tensor(mean, dtype=torch.float32).to(device),
                             torch.tensor(std, dtype=torch.float32).to(device))
    return _NORM_CONSTS[key]


def clip_preprocess_packed(packed: Tensor, sizes, device, size: int = 224, crop: int = 224, mean=None,
                           std=None) -> Tensor:
    """clip_preprocess of images already packed back to back: `packed` uint8 [sum H*W*3] (host — pinned for an
    asynchronous copy — or device), `sizes` [(H, W)] in order. The extraction loop's workers pack each batch
    (icap.images.ImageDirectoryDataset.packed_collate), so the main process makes one copy per batch."""
    from .clip import CLIP_MEAN, CLIP_STD

    sizes = [(int(h), int(w)) for h, w in sizes]
    n = len(sizes)
    out = torch.empty((n, 3, crop, crop), dtype=torch.float32, device=device)
    if n == 0:
        return out
    if packed.dtype != torch.uint8 or packed.numel() != sum(h * w * 3 for h, w in sizes):
        raise L.IcapError("clip_preprocess_packed: packed must be uint8 holding every image's H*W*3 bytes")
    geo, tmp_bytes = clip_preprocess_geometry(sizes, size, crop)
    max_rows = max(g[9] for g in geo)
    px = packed.to(device, non_blocking=True)
    # no host-blocking copies per batch (a pageable copy waits for the stream, i.e. for the previous batch's
    # kernels): the geometry table from pinned memory, mean / std uploaded once per device
    geo_h = torch.tensor(geo, dtype=torch.int64)
    geo_t = (geo_h.pin_memory() if torch.device(device).type == "cuda" else geo_h).to(device, non_blocking=True)
    tmp = torch.empty(tmp_bytes, dtype=torch.uint8, device=device)
    m, s = _norm_consts(device, tuple(CLIP_MEAN if mean is None else mean), tuple(CLIP_STD if std is None else std))
    call("icap_clip_preprocess", n, px.data_ptr(), geo_t.data_ptr(), crop, max_rows, tmp.data_ptr(), m.data_ptr(),
         s.data_ptr(), out.data_ptr(), _stream())
    return out
