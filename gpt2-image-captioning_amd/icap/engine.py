"""The fused captioning train step: CLIP fwd (optional) -> mapper fwd -> GPT-2 fwd -> LM head + CE ->
GPT-2 dX backward -> mapper backward -> (RCCL all-reduce) -> clip_grad_norm + AdamW + LR schedule.

This is src/train.py:119-166 (one inner iteration) as an explicit schedule of libicap_hip.so kernels on
one HIP stream, with all buffers preallocated so the whole step can be captured into a HIP graph and
replayed (torch.cuda.CUDAGraph is only the capture/replay plumbing). Trainable parameters, their grads and
the AdamW moments live in one flat fp32 buffer each (weights.FlatParams); the bf16 compute copy of the
trainable weights is written by the AdamW kernel itself.
"""

from __future__ import annotations

from types import SimpleNamespace
from typing import List, Optional, Tuple

import torch

from . import ops
from .mapper import DWHelper, MLPMapperCore, TransformerMapperCore
from .models import _embedding_grads

# Schedule constants (module attributes, not process environment: A/B tools and tests set them explicitly).
# packed attention launches skip their long-sequence pass when every sequence of the batch is short (set per batch in
# load_batch); False always launches both passes
SHORT_ONLY = True
# the first micro-batch of an accumulation cycle writes the trained mapper's gradients (each is produced once per
# micro-batch) instead of zeroing the flat gradient buffer and accumulating into it; False restores the zero_() +
# accumulate form
GRAD_OVERWRITE = True

Tensor = torch.Tensor


def _async_src(t: Tensor) -> bool:
    """A host-to-device copy may be queued asynchronously only from pinned memory; device sources always may."""
    return t.device.type != "cpu" or t.is_pinned()


class CaptionTrainer:
    def __init__(self, model, batch_size: int, caption_len: int, *, lr: float = 1e-4, weight_decay: float = 0.01,
                 betas=(0.9, 0.999), eps: float = 1e-8, max_norm: float = 1.0, num_warmup_steps: int = 0,
                 num_training_steps: int = 1, dropout: bool = True, seed: int = 0, clip_model=None,
                 grad_accum_steps: int = 1, process_group=None, compact_head: bool = True,
                 pack_rows: bool = True, dp_overlap: bool = True, dp_bf16: bool = False, force_overlap: bool = False,
                 mapper_dw: str = "fused"):
        """pack_rows: packed token rows (GPT2Core.alloc_train); dp_overlap: with N > 1 ranks, all-reduce each backward
        segment's gradient bucket beside the later segments (False: one whole-buffer all-reduce after the backward);
        dp_bf16: exchange the gradients as bf16 (half the bytes; rounds the sum over ranks); force_overlap: take the
        bucketed communication-stream step at world size 1 too (exercises the RCCL calls on one GPU).
        mapper_dw (transformer mapper, GPU): where its weight-gradient products run — "serial" (in the dX chain,
        split-K), "side" (a second stream beside the dX chain), "group" (a layer's four products unsplit on four
        streams at the end of its step) or "fused" (a layer's four products in one grouped launch at the end of its
        step, icap_gemm_group; the default since round 6: 13.99k vs 13.41k images/s for "serial" in one session,
        profiles/r06_mapper_dw_ab.txt). All give the same gradients up to the summation order of the split ("fused"
        and "group" bitwise equal); "side" and "group" measured no faster than "serial" (DESIGN.md "Concurrency: the
        packed-FP32 race")."""
        self.model = model
        self.dtype = model.compute_dtype
        self.B, self.Lc = batch_size, caption_len
        self.hp = SimpleNamespace(lr=lr, weight_decay=weight_decay, betas=betas, eps=eps, max_norm=max_norm,
                                  num_warmup_steps=num_warmup_steps, num_training_steps=num_training_steps)
        self.dropout = dropout
        self.seed = seed
        self.grad_accum_steps = grad_accum_steps
        self.pg = process_group
        self.world = 1
        self.distributed = process_group is not None or (torch.distributed.is_available()
                                                         and torch.distributed.is_initialized())
        if self.distributed:
            self.world = torch.distributed.get_world_size(process_group)
            # DDP's construction-time guarantee: every rank starts from rank 0's replica (trainable masters, frozen
            # GPT-2 / image-tower weights), whatever each process's RNG produced when it built the model
            broadcast_replicas([model] + ([clip_model] if clip_model is not None else []), process_group)
        # the bucketed communication-stream step also at world size 1 (exercises the RCCL calls on one GPU)
        self.force_overlap = bool(force_overlap) and self.distributed
        self.dev = model.device
        flat = model.flat()
        self.flat = flat
        self.mcore = model.mapping_network.core(self.dtype, flat)
        self.clip = clip_model.core(self.dtype) if clip_model is not None else None
        # freeze_gpt_weights=False (src/models.py:216-217, train.py:94-96): every GPT-2 tensor is in the flat
        # storage, the backward adds its dW / bias / LayerNorm / tied-wte / wpe grads, and the AdamW step is
        # followed by an in-place refresh of the GPT-2 forward-orientation copies
        self.gpt_trainable = not model.freeze_gpt_weights
        if self.gpt_trainable:
            model.gpt.invalidate_core()  # a core of its own, bound to the flat storage
            self.gcore = model.gpt.core(self.dtype)
            model.gpt.invalidate_core()
            self.gcore.bind_flat(flat)
            compact_head = False  # the tied wte gradient reads the LM-head input of every row
        else:
            self.gcore = model.gpt.core(self.dtype)
        B, Lc = batch_size, caption_len
        P = model.total_prefix_length
        self.P = P
        # (per-layer backward gradient buffers only for the schedules whose weight-gradient products trail the dX
        # chain on other streams: 433 MB at B = 128 that the default serial schedule does not need)
        per_layer = (dict(per_layer_grads=mapper_dw in ("side", "group")) if isinstance(self.mcore, TransformerMapperCore)
                     else {})
        self.mws = self.mcore.alloc(B, train=True, **per_layer)
        # packed token rows (GPT2Core.alloc_train): the blocks skip each caption's dead tail (positions after its
        # last loss target, which the causal mask keeps out of every loss term)
        self.gws = self.gcore.alloc_train(B, P, Lc, keep_for_dw=self.gpt_trainable, compact_head=compact_head,
                                          pack=pack_rows)
        D = self.gcore.D
        M2 = self.mws.M
        E = self.mcore.E
        S = self.gws.S
        max_cols = max(4 * D, 3 * D, E, self.mcore.dw_cols())
        max_rows, ln_rows, cs_cols = max(M2, B), M2, P * D
        if self.gpt_trainable:  # + the GPT-2 dW products (the tied wte: [V, D]) and the wpe column sums
            max_cols = max(max_cols, self.gcore.V)
            max_rows, ln_rows, cs_cols = max(max_rows, self.gws.M), max(M2, self.gws.M), S * D
        # colsum also reduces the prefix_const / task-prefix grads over the batch: B rows x P*D columns
        self.dwh = DWHelper(self.dtype, self.dev, max_rows=max_rows, max_cols=max_cols, ln_rows=ln_rows, ln_D=D,
                            colsum_cols=cs_cols)
        self.ggrads = model._gpt_grads(flat) if self.gpt_trainable else None
        self._gver = flat.flat._version
        self.mgrads = self.mcore.grads(flat)
        # data-parallel buckets: the flat-gradient ranges each segment of the step finalises (engine._segments)
        mapper = model.mapping_network
        if isinstance(self.mcore, TransformerMapperCore):
            groups = [list(blk.parameters()) for blk in reversed(list(mapper.transformer.layers))]
            groups.append([mapper.linear.weight, mapper.linear.bias, mapper.prefix_const])
        else:
            groups = [list(mapper.parameters())]
        self._ranges_mapper = [flat_ranges(flat, ps) for ps in groups]
        seen = {id(p) for ps in groups for p in ps}
        self._ranges_front = flat_ranges(flat, [p for p in flat.params if id(p) not in seen])
        self.dp_overlap = bool(dp_overlap)
        # opt-in: all-reduce the gradients as bf16 (half the bytes over xGMI; the sum over ranks is rounded to bf16
        # per element, so it is not the fp32 reduction the reference's single-process step corresponds to)
        self.dp_bf16 = bool(dp_bf16)
        self._g16 = None
        self.seg_graphs = {}  # zero -> [HIP graph per segment] (data-parallel overlapped step)
        self._comm = None
        if model.task_prefix_embeds is not None:
            self.task_grad = flat.grad(model.task_prefix_embeds)
            self.pre = torch.empty((B, P, D), dtype=self.dtype, device=self.dev)
        # static inputs (graph-capture friendly)
        self.ids = torch.zeros((B, Lc), dtype=torch.int64, device=self.dev)
        self.mask = torch.ones((B, Lc), dtype=torch.int64, device=self.dev)
        self.labels = torch.zeros((B, Lc), dtype=torch.int64, device=self.dev)
        self.emb = torch.zeros((B, E), dtype=torch.float32, device=self.dev)
        self.emb_c = torch.zeros((B, E), dtype=self.dtype, device=self.dev)
        self.pixels = None
        if self.clip is not None:
            c = clip_model.config
            self.pixels = torch.zeros((B, c.num_channels, c.image_size, c.image_size), dtype=torch.float32,
                                      device=self.dev)
            self.cws = self.clip.alloc(B)
        self.counter = torch.zeros(1, dtype=torch.int64, device=self.dev)
        if flat.exp_avg is None:
            flat.exp_avg = torch.zeros_like(flat.flat)
            flat.exp_avg_sq = torch.zeros_like(flat.flat)
        self.adam_state = torch.zeros(16, dtype=torch.float32, device=self.dev)
        self.adam_ws = torch.empty(ops.adamw_workspace(flat.n), dtype=torch.uint8, device=self.dev)
        self.loss_sum = torch.zeros(1, dtype=torch.float32, device=self.dev)
        self.graphs = {}  # (zero, with_optimizer) -> captured HIP graph
        self.graph_opt = None
        self._micro = 0
        self._eager_steps = 0
        self.gdr = self.gcore.drops(dropout, seed, self.counter, self.gws.M, B, self.gws.S)
        p_map = 0.1 if isinstance(self.mcore, TransformerMapperCore) else 0.0
        self.mdr = self.mcore.drops(dropout, p_map, seed, self.counter, B)
        if mapper_dw not in ("serial", "side", "group", "fused"):
            raise ValueError(f"mapper_dw must be 'serial', 'side', 'group' or 'fused', not {mapper_dw!r}")
        multi = self.dev.type == "cuda" and isinstance(self.mcore, TransformerMapperCore)
        # the mapper's weight-gradient products on a side stream beside its dX chain (mapper.backward_steps side=)
        self._side = None
        if multi and mapper_dw == "side":
            self._side = torch.cuda.Stream(self.dev)
            ops.register_side_stream(self._side)
        # the mapper's four dW products of a layer unsplit and side by side on three more streams (group=)
        self._group = None
        if multi and mapper_dw == "group" and self.dtype == torch.bfloat16:
            self._group = [torch.cuda.Stream(self.dev) for _ in range(3)]
            for sd in self._group:
                ops.register_side_stream(sd)
        # "fused": the four products of a layer in one grouped launch at the end of its step (icap_gemm_group; bf16 —
        # the fp32 parity mode keeps the serial schedule, whose per-product transposes the group has no form for)
        if mapper_dw == "fused" and isinstance(self.mcore, TransformerMapperCore) and self.dtype == torch.bfloat16:
            self._group = "fused"

    def share_state_with(self, other: "CaptionTrainer") -> None:
        """Use `other`'s optimizer step counter and dropout counter (same model, another batch shape)."""
        self.adam_state = other.adam_state
        self.counter = other.counter
        self.gdr = self.gcore.drops(self.dropout, self.seed, self.counter, self.gws.M, self.B, self.gws.S)
        p_map = 0.1 if isinstance(self.mcore, TransformerMapperCore) else 0.0
        self.mdr = self.mcore.drops(self.dropout, p_map, self.seed, self.counter, self.B)

    # -- inputs -----------------------------------------------------------------------------------------------
    def load_batch(self, ids: Tensor, mask: Tensor, labels: Tensor, emb: Optional[Tensor] = None,
                   pixels: Optional[Tensor] = None) -> None:
        if self.gws.pack and self.gws.live_rows_hint is None:
            # the first batch's packed row count (one host read, before any capture): the GEMM kernel choice for the
            # expected live rows (icap_gemm_args.m_hint); the device count of every batch is what bounds the work
            self.gws.live_rows_hint = live_rows(labels, self.P)
            self.gws.seq_sq_hint = live_rows(labels, self.P, squares=True)
        if self.gws.pack and SHORT_ONLY:
            # every packed sequence of THIS batch <= 32 tokens: the attention launches skip their long-sequence pass
            # (icap_attn_args.short_only — a guarantee, so it is taken from each batch's labels, and the captured
            # graphs are keyed on it). Read from host labels only (the data loaders deliver CPU tensors): for labels
            # already on the device the flag stays off (both passes launched; same results) rather than forcing a
            # device-to-host sync per batch
            self.gws.short_only = labels.device.type == "cpu" and max_seq_len(labels, self.P) <= 32
        # asynchronous only from pinned host memory (the loaders' batches) or device memory: a pageable source is
        # copied synchronously (non_blocking from pageable memory overlaps nothing and was part of the round-5 hang,
        # DESIGN.md "Extraction loader")
        self.ids.copy_(ids, non_blocking=_async_src(ids))
        self.mask.copy_(mask, non_blocking=_async_src(mask))
        self.labels.copy_(labels, non_blocking=_async_src(labels))
        if pixels is not None:
            if self.pixels is None:
                raise ValueError("trainer was built without a CLIP tower; pass image embeddings")
            self.pixels.copy_(pixels, non_blocking=_async_src(pixels))
        elif emb is not None:
            self.emb.copy_(emb, non_blocking=_async_src(emb))

    # -- the step ---------------------------------------------------------------------------------------------
    def _fwd_bwd(self, zero: bool, grad_scale: float) -> None:
        for _, fn in self._segments(zero, grad_scale):
            fn()

    def _segments(self, zero: bool, grad_scale: float):
        """The forward + backward as [(flat-gradient ranges finalised, fn)] in schedule order: everything up to the
        mapper backward (finalises the GPT-2 grads when it is trainable and the task-prefix grad), then one segment
        per mapper layer (top first) and the mapper's input projection. Run back to back they are the step; the
        data-parallel step all-reduces each segment's ranges while the next segments compute."""
        B, P, D = self.B, self.P, self.gcore.D
        model, mc = self.model, self.mcore
        st = SimpleNamespace()

        def front():
            st.d_emb = self._front(zero, grad_scale)

        segs = [(self._ranges_front, front)]
        if isinstance(mc, TransformerMapperCore):
            # the side stream joins at each layer step's end only when the steps are data-parallel buckets
            steps = mc.backward_steps(self.mws, self.emb_c, self.mdr, self.mgrads, self.dwh, side=self._side,
                                      join_each=self.world > 1 or self.force_overlap,
                                      overwrite=zero and self._overwrite_ok(), group=self._group)
            for (_, _, fn), rng in zip(steps, self._ranges_mapper):
                segs.append((rng, fn))
        else:
            S, Pm = self.gws.S, mc.P

            def mlp():
                d_pre = st.d_emb.view(B, S * D)[:, : P * D]
                mc.backward_from(d_pre[:, : Pm * D], S * D, self.mws, self.emb_c, self.mgrads, self.dwh)

            segs.append((self._ranges_mapper[0], mlp))
        last_rng, last_fn = segs[-1]

        def last():
            last_fn()
            self.loss_sum.add_(self.gws.loss)

        segs[-1] = (last_rng, last)
        return segs

    def _overwrite_ok(self) -> bool:
        """Every flat-gradient element is written exactly once per micro-batch (transformer mapper + optional task
        prefix; GPT-2 frozen — its trained form accumulates several products into the tied wte gradient), so a new
        cycle can overwrite instead of zeroing the 243 MB buffer first (the alignment gaps between tensors stay zero
        from allocation: nothing writes them)."""
        return GRAD_OVERWRITE and isinstance(self.mcore, TransformerMapperCore) and not self.gpt_trainable

    def _front(self, zero: bool, grad_scale: float):
        """Forward, LM head + CE, GPT-2 backward and the mapper's output gradient; returns d(inputs_embeds)."""
        B, P, D = self.B, self.P, self.gcore.D
        model = self.model
        if zero and not self._overwrite_ok():
            self.flat.flat_grad.zero_()
        if self.clip is not None:
            emb = self.clip.run(self.cws, self.pixels)
            ops.convert(emb, self.emb_c)
        else:
            ops.convert(self.emb, self.emb_c)
        if self.dropout:
            ops.counter_increment(self.counter)
        mc, gc = self.mcore, self.gcore
        mc.forward(self.mws, self.emb_c, self.mdr, train=True)
        pre, pbs = mc.prefix_view(self.mws)
        if model.task_prefix_embeds is not None:  # [image prefix ; task prefix] (src/models.py:269-283)
            Pm = mc.P
            ops.convert(_rows_view(pre, B, Pm * D, pbs), self.pre.view(B, P * D)[:, : Pm * D])
            ops.broadcast_rows(model.task_prefix_embeds.data, self.pre.view(-1)[Pm * D:], B, P * D)
            pre, pbs = self.pre, P * D
        gc.forward_train(self.gws, pre, pbs, self.ids, self.mask, self.labels, self.gdr, fuse_dlogits=True,
                         grad_scale=grad_scale)
        S = self.gws.S
        d_emb = gc.backward(self.gws, self.gdr, self.gws.key_mask, self.gws.logits, grads=self.ggrads,
                            dw=self.dwh if self.gpt_trainable else None)
        if self.gpt_trainable:
            _embedding_grads(d_emb, self.ids, B, P, self.Lc, D, self.ggrads, self.dwh)
        d_pre = d_emb.view(B, S * D)[:, : P * D]
        Pm = mc.P
        if model.task_prefix_embeds is not None:
            ops.colsum(d_emb.view(B, S * D)[:, Pm * D: P * D], self.task_grad.view(-1), self.dwh.cs_ws,
                       accumulate=not (zero and self._overwrite_ok()), M=B, N=(P - Pm) * D)
        if isinstance(mc, TransformerMapperCore):
            Hl, Sm = mc.Hl, mc.S
            ops.convert(d_pre[:, : Pm * D], self.mws.dout.view(B, Sm * D)[:, Hl * D:])
        return d_emb

    def _optimizer(self) -> None:
        hp, f = self.hp, self.flat
        ops.adamw_step(f.flat, f.flat_grad, f.exp_avg, f.exp_avg_sq, self.adam_state, self.adam_ws, lr=hp.lr,
                       betas=hp.betas, eps=hp.eps, weight_decay=hp.weight_decay, max_norm=hp.max_norm,
                       num_warmup_steps=hp.num_warmup_steps, num_training_steps=hp.num_training_steps,
                       bf16_out=f.flat_c)
        self.mcore.refresh_transposes()
        if self.gpt_trainable:
            self.gcore.refresh_from_flat()

    def _allreduce(self) -> None:
        if self.world > 1:
            if self.dp_bf16:
                g = self.flat.flat_grad
                self._to16(g, 0, g.numel())
                torch.distributed.all_reduce(self._g16, group=self.pg)
                self._from16(g, [(0, g.numel())])
            else:
                torch.distributed.all_reduce(self.flat.flat_grad, group=self.pg)

    def _to16(self, g, lo: int, hi: int) -> None:
        """bf16 staging copy of flat_grad[lo:hi] (the dp_bf16 all-reduce), on the current stream."""
        if self._g16 is None:
            self._g16 = torch.empty(g.numel(), dtype=torch.bfloat16, device=g.device)
        if g.is_cuda:
            ops.convert(g[lo:hi].view(1, -1), self._g16[lo:hi].view(1, -1))
        else:  # CPU dry runs (gloo tests): no kernels
            self._g16[lo:hi].copy_(g[lo:hi])

    def _from16(self, g, ranges) -> None:
        for lo, hi in ranges:
            if g.is_cuda:
                ops.convert(self._g16[lo:hi].view(1, -1), g[lo:hi].view(1, -1))
            else:
                g[lo:hi].copy_(self._g16[lo:hi])

    def _bucket(self, ranges, works) -> None:
        """All-reduce these flat-gradient ranges behind the work queued so far on this stream, on a communication
        stream (RCCL then runs beside the next backward segments); `works` collects the async handles."""
        g = self.flat.flat_grad
        if not ranges:
            return
        src = (lambda lo, hi: self._g16[lo:hi]) if self.dp_bf16 else (lambda lo, hi: g[lo:hi])
        if g.is_cuda:
            if self._comm is None:
                self._comm = torch.cuda.Stream(g.device)
            ev = torch.cuda.Event()
            ev.record()
            with torch.cuda.stream(self._comm):
                self._comm.wait_event(ev)
                for lo, hi in ranges:
                    if self.dp_bf16:
                        self._to16(g, lo, hi)
                    works.append(torch.distributed.all_reduce(src(lo, hi), group=self.pg, async_op=True))
        else:
            for lo, hi in ranges:
                if self.dp_bf16:
                    self._to16(g, lo, hi)
                works.append(torch.distributed.all_reduce(src(lo, hi), group=self.pg, async_op=True))
        if self.dp_bf16:
            self._pending16.extend(ranges)

    def _overlapped_step(self, zero: bool, use_graph: bool) -> None:
        """Data-parallel micro-batch that ends an accumulation cycle: each segment's gradient ranges are
        all-reduced (RCCL, async) while the later segments of the backward run; the optimizer waits for all."""
        works = []
        self._pending16 = []
        if use_graph:
            graphs = self.seg_graphs.get((zero, self.gws.short_only))
            if graphs is None:
                graphs = self._capture_segments(zero)
            for (rng, _), g in zip(self._segments(zero, self.grad_scale()), graphs):
                g.replay()
                self._bucket(rng, works)
        else:
            for rng, fn in self._segments(zero, self.grad_scale()):
                fn()
                self._bucket(rng, works)
        for w in works:
            w.wait()
        if self.dp_bf16:  # the reduced bf16 ranges back into the fp32 gradient the optimizer reads
            self._from16(self.flat.flat_grad, self._pending16)
        if use_graph:
            if self.graph_opt is None:
                self.graph_opt = self._capture_opt()
            self.graph_opt.replay()
        else:
            self._optimizer()

    def _capture_segments(self, zero: bool):
        torch.cuda.synchronize(self.dev)
        graphs = []
        for _, fn in self._segments(zero, self.grad_scale()):
            g = torch.cuda.CUDAGraph()
            with ops.graph_capture(g):
                fn()
            graphs.append(g)
        self.seg_graphs[(zero, self.gws.short_only)] = graphs
        return graphs

    def grad_scale(self) -> float:
        return 1.0 / (self.grad_accum_steps * self.world)

    def micro_step(self, use_graph: bool = False, zero: Optional[bool] = None, step: Optional[bool] = None) -> bool:
        """One micro-batch (forward + backward). Returns True when an optimizer step was taken.

        zero: start a new accumulation cycle (the gradients are cleared first); step: take the optimizer step
        after this micro-batch. Both default to this trainer's own count (a step every grad_accum_steps
        micro-batches); icap.train passes them explicitly from the batch index, as src/train.py:128-159 does
        (step when (batch_idx + 1) % grad_accum_steps == 0 or at the last batch), so a cycle may span trainers
        of different batch shapes (a short last batch) — they share one flat gradient buffer.
        With use_graph the first call runs eagerly (warm-up) and every later call replays a captured HIP graph
        (one per (zero, step) form)."""
        self.model.sync_compute_copies()
        if self.gpt_trainable and self.flat.flat._version != self._gver:  # masters written outside the optimizer
            self.gcore.refresh_from_flat()
            self._gver = self.flat.flat._version
        if zero is None:
            zero = self._micro == 0
        if step is None:
            step = self._micro + 1 >= self.grad_accum_steps
        if step and (self.world > 1 or self.force_overlap) and self.dp_overlap:
            self._overlapped_step(zero, use_graph and self._eager_steps >= 1)
            self._eager_steps += 1
        elif use_graph and self._eager_steps >= 1:
            with_opt = step and self.world == 1
            g = self.graphs.get((zero, with_opt, self.gws.short_only))
            if g is None:
                g = self._capture(zero, with_opt)
            g.replay()
            if step and self.world > 1:
                self._allreduce()
                if self.graph_opt is None:
                    self.graph_opt = self._capture_opt()
                self.graph_opt.replay()
        else:
            self._fwd_bwd(zero, self.grad_scale())
            self._eager_steps += 1
            if step:
                self._allreduce()
                self._optimizer()
        self._micro = 0 if step else self._micro + 1
        return step

    def flush(self) -> None:
        """Apply a pending partial accumulation of this trainer's own count (the last-batch rule of
        src/train.py:146-148 for callers that use the default micro_step flags)."""
        if self._micro:
            self._allreduce()
            self._optimizer()
            self._micro = 0

    @property
    def graph(self):
        """The plain-step graph (new cycle + optimizer step), once captured."""
        return self.graphs.get((True, self.world == 1))

    def _capture(self, zero: bool, with_opt: bool):
        """Capture fwd+bwd (+ optimizer) into a HIP graph (recording only: nothing executes; called after at
        least one eager step so every kernel and attribute has been initialised)."""
        torch.cuda.synchronize(self.dev)
        g = torch.cuda.CUDAGraph()
        with ops.graph_capture(g):
            self._fwd_bwd(zero, self.grad_scale())
            if with_opt:
                self._optimizer()
        self.graphs[(zero, with_opt, self.gws.short_only)] = g
        return g

    def _capture_opt(self):
        torch.cuda.synchronize(self.dev)
        g = torch.cuda.CUDAGraph()
        with ops.graph_capture(g):
            self._optimizer()
        return g

    def capture(self) -> None:
        """Capture the plain step (new cycle + optimizer) ahead of time."""
        self._capture(True, self.world == 1)
        if self.world > 1 and self.graph_opt is None:
            self.graph_opt = self._capture_opt()

    def take_loss_sum(self) -> float:
        v = float(self.loss_sum.item())
        self.loss_sum.zero_()
        return v

    @property
    def last_loss(self) -> Tensor:
        return self.gws.loss


@torch.no_grad()
def max_seq_len(labels: Tensor, P: int) -> int:
    """The longest packed sequence of a batch (icap_caption_pack's seq_len, restated on the host side of the copy)."""
    valid = (labels != -100).to(torch.int64)
    pos = torch.arange(1, labels.shape[1] + 1, device=labels.device, dtype=torch.int64)
    last = (valid * pos).max(dim=1).values
    return int((P + (last - 1).clamp_min(0)).max().item()) if labels.shape[0] else 0


def live_rows(labels: Tensor, P: int, squares: bool = False) -> int:
    """Packed token rows of a batch (icap_caption_pack's m_live, computed on the host side of the copy):
    sum over captions of max(P, P + last caption index with a target); squares: the sum of their squares (the
    attention launches' work)."""
    valid = (labels != -100).to(torch.int64)
    pos = torch.arange(1, labels.shape[1] + 1, device=labels.device, dtype=torch.int64)
    last = (valid * pos).max(dim=1).values  # last target index + 1, or 0
    lens = P + (last - 1).clamp_min(0)
    return int((lens * lens if squares else lens).sum().item())


def broadcast_replicas(modules, process_group=None) -> None:
    """Broadcast every parameter and buffer of `modules` from the group's rank 0, in place, then drop the compute
    copies derived from them (GPT-2 / mapper / image-tower cores, the mapper's bf16 flat copy) so they are rebuilt
    from the broadcast values. The trainable nn.Parameters may be views of the flat fp32 master buffer; an in-place
    broadcast into a view writes the master."""
    dist = torch.distributed
    src = dist.get_global_rank(process_group, 0) if process_group is not None else 0
    seen = set()
    for m in modules:
        for t in list(m.parameters()) + list(m.buffers()):
            if id(t) in seen or t.numel() == 0:
                continue
            seen.add(id(t))
            if t.is_contiguous():
                dist.broadcast(t.data, src=src, group=process_group)
            else:
                tmp = t.data.contiguous()
                dist.broadcast(tmp, src=src, group=process_group)
                t.data.copy_(tmp)
    for m in modules:
        for sub in m.modules():
            if hasattr(sub, "invalidate_core"):
                sub.invalidate_core()
            elif getattr(sub, "_core", None) is not None:
                sub._core = None
        f = getattr(m, "_flat", None)
        if f is not None:
            f.sync_compute_copy()
            m._synced_version = f.flat._version


def flat_ranges(flat, params) -> List[Tuple[int, int]]:
    """[lo, hi) element ranges of the flat gradient buffer that hold `params` (each parameter's segment runs to the
    next one's start, so the alignment padding is covered), adjacent segments merged."""
    idx = sorted(flat._index(p) for p in params)
    out: List[Tuple[int, int]] = []
    for i in idx:
        lo = flat.offsets[i]
        hi = flat.offsets[i + 1] if i + 1 < len(flat.offsets) else flat.n
        if out and out[-1][1] == lo:
            out[-1] = (out[-1][0], hi)
        else:
            out.append((lo, hi))
    return out


def _rows_view(t: Tensor, B: int, n: int, stride: int) -> Tensor:
    return t.as_strided((B, n), (stride, 1))
