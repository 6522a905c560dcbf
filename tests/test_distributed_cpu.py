"""world_size-2 `gloo` tests of the data-parallel path on the CPU.

The N > 1 train step is: each rank runs forward + backward on its own shard with the CE gradient scaled by
1 / (grad_accum * world) (engine.CaptionTrainer.grad_scale), one all-reduce (SUM) of the flat fp32 gradient
buffer, then clip + AdamW identically on every rank. Here the real host schedule runs with the C-ABI calls
recorded instead of launched (tests/dryrun.py), and torch.distributed runs over gloo on CPU tensors — the same
calls the GPU path issues over RCCL.

1. CaptionTrainer: world / grad scale from the process group; after a step every rank holds the same reduced
   gradient (the mean of the per-rank shard gradients) when the optimizer is called, and every launch stays
   inside live allocations.
2. train(): DistributedSampler shards the shuffled index disjointly and covers the dataset each epoch; only
   rank 0 writes checkpoints.
3. The DP contract itself, on the oracle: mean of per-rank shard gradients == full-batch gradient when the
   shards have equal valid-token counts (the synthetic COCO-shaped captions), checked through a real gloo
   all-reduce.
"""

import os
import socket
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

WORLD = 2


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _entry(rank, world, port, fn_name, q, arg):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q.put((rank, globals()[fn_name](rank, world, arg)))
    except BaseException as e:  # report, the parent asserts
        import traceback

        q.put((rank, "ERROR " + "".join(traceback.format_exception(type(e), e, e.__traceback__))))
    finally:
        dist.destroy_process_group()


def _run(fn_name, arg=None, world=WORLD):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_entry, args=(r, world, port, fn_name, q, arg)) for r in range(world)]
    for p in ps:
        p.start()
    out = {}
    for _ in range(world):
        r, v = q.get(timeout=240)
        out[r] = v
    for p in ps:
        p.join(timeout=60)
    for r, v in out.items():
        assert not (isinstance(v, str) and v.startswith("ERROR")), f"rank {r}: {v}"
    return out


# ------------------------------------------------------------------------------------------ 1. trainer step


def _trainer_allreduce(rank, world, _):
    import icap.weights
    from dryrun import dry_run
    from icap import CaptionTrainer
    from test_dryrun_bounds import batch, tiny_model

    torch.manual_seed(rank)
    with dry_run() as rec:
        icap.weights.ops.call = rec
        model = tiny_model()
        t = CaptionTrainer(model, 3, 12, num_training_steps=3)
        t.dp_overlap = False  # the single whole-buffer all-reduce path (ICAP_DP_OVERLAP=0)
        assert t.world == world and abs(t.grad_scale() - 1.0 / world) < 1e-12
        t.load_batch(*batch(3, 12))
        n = t.flat.flat_grad.numel()
        seen = {}
        orig_fb, orig_opt = t._fwd_bwd, t._optimizer

        def fwd_bwd(first, scale):  # the real schedule is recorded; stand in a known per-rank shard gradient
            orig_fb(first, scale)
            g = torch.arange(n, dtype=torch.float32) * (rank + 1) + 7.0 * rank
            t.flat.flat_grad.copy_(g * scale)

        def optimizer():
            seen["grad_at_opt"] = t.flat.flat_grad.clone()
            orig_opt()

        t._fwd_bwd, t._optimizer = fwd_bwd, optimizer
        took = t.micro_step()
        bad = rec.check()
        names = [c[0] for c in rec.calls]
    exp = sum(torch.arange(n, dtype=torch.float32) * (r + 1) + 7.0 * r for r in range(world)) / world
    return {"took": took, "bad": bad[:5], "adamw": "icap_adamw_step" in names,
            "max_err": float((seen["grad_at_opt"] - exp).abs().max()), "sum": float(seen["grad_at_opt"].sum())}


def test_trainer_gradient_allreduce_world2():
    out = _run("_trainer_allreduce")
    for r in range(WORLD):
        v = out[r]
        assert v["took"] and v["adamw"] and not v["bad"], v
        assert v["max_err"] < 1e-3, v
    assert out[0]["sum"] == out[1]["sum"]  # identical reduced gradient on every rank


def _trainer_overlap(rank, world, arg):
    """The overlapped data-parallel step: each segment of the step writes a known per-rank gradient into the flat
    ranges it finalises, right after its real (recorded) schedule; the bucketed async all-reduces must hand the
    optimizer the sum over ranks of every element (the 1/world is in the CE scale), and the segments' ranges must
    tile the buffer exactly."""
    import icap.weights
    from dryrun import dry_run
    from icap import CaptionTrainer
    from test_dryrun_bounds import batch, tiny_model

    mapper, freeze, bf16 = arg
    with dry_run() as rec:
        icap.weights.ops.call = rec
        model = tiny_model(mapper, freeze=freeze)
        t = CaptionTrainer(model, 3, 12, num_training_steps=3)
        assert t.dp_overlap
        t.dp_bf16 = bf16  # ICAP_DP_BF16=1: bf16 staging buffer all-reduced, converted back before the optimizer
        t.load_batch(*batch(3, 12))
        n = t.flat.flat_grad.numel()
        cover = torch.zeros(n, dtype=torch.int32)
        orig_segments, orig_opt = t._segments, t._optimizer
        seen = {}

        def segments(zero, scale):
            out = []
            for rng, fn in orig_segments(zero, scale):
                def run(rng=rng, fn=fn):
                    fn()
                    for lo, hi in rng:
                        cover[lo:hi] += 1
                        t.flat.flat_grad[lo:hi] = (torch.arange(lo, hi, dtype=torch.float32) * (rank + 1) + 7.0 * rank)
                out.append((rng, run))
            return out

        def optimizer():
            seen["grad_at_opt"] = t.flat.flat_grad.clone()
            orig_opt()

        t._segments, t._optimizer = segments, optimizer
        took = t.micro_step()
        bad = rec.check()
        nseg = len(orig_segments(True, 1.0))
    exp = sum(torch.arange(n, dtype=torch.float32) * (r + 1) + 7.0 * r for r in range(world))  # SUM all-reduce
    return {"took": took, "bad": bad[:5], "segments": nseg, "cover_ok": bool((cover == 1).all()),
            "max_err": float((seen["grad_at_opt"] - exp).abs().max()),
            "max_rel": float(((seen["grad_at_opt"] - exp).abs() / exp.abs().clamp_min(1.0)).max())}


@pytest.mark.parametrize("mapper,freeze,bf16", [("transformer", True, False), ("transformer", False, False),
                                                ("mlp", True, False), ("transformer", True, True)])
def test_trainer_overlapped_bucket_allreduce_world2(mapper, freeze, bf16):
    out = _run("_trainer_overlap", (mapper, freeze, bf16))
    for r in range(WORLD):
        v = out[r]
        assert v["took"] and not v["bad"] and v["cover_ok"], v
        assert v["segments"] == (2 if mapper == "mlp" else 1 + 2 + 1), v  # front + per layer (tiny: 2) + head
        if bf16:  # each rank's value and the sum rounded to bf16 (8 significant bits)
            assert v["max_rel"] < 2 ** -6, v
        else:
            assert v["max_err"] < 1e-2, v


def _replica_broadcast(rank, world, arg):
    """Ranks build their models from DIFFERENT RNG seeds; constructing the CaptionTrainer under the process group
    must leave every parameter and buffer equal to rank 0's (DDP's construction-time broadcast), including the
    trainable masters inside the flat buffer and the frozen GPT-2 weights, and a data-parallel step (stand-in
    per-rank gradients, then the real all-reduce) keeps them equal."""
    import icap.weights
    from dryrun import dry_run
    from icap import CaptionTrainer
    from test_dryrun_bounds import batch, tiny_model

    mapper, freeze = arg
    torch.manual_seed(1000 + 17 * rank)
    with dry_run() as rec:
        icap.weights.ops.call = rec
        model = tiny_model(mapper, freeze=freeze)

        def digest():
            return [float(t.detach().double().sum()) + float((t.detach().double() ** 2).sum())
                    for t in list(model.parameters()) + list(model.buffers())]

        before = digest()
        t = CaptionTrainer(model, 3, 12, num_training_steps=3)
        after = digest()
        flat_sum = float(t.flat.flat.double().sum())
        # two DP steps: the optimizer is a recorded C-ABI call, so stand in an update that depends only on the
        # reduced gradient (identical on every rank iff the all-reduce and the replicas are)
        t.dp_overlap = False
        n = t.flat.flat_grad.numel()
        orig_fb = t._fwd_bwd

        def fwd_bwd(first, scale):
            orig_fb(first, scale)
            t.flat.flat_grad.copy_((torch.arange(n, dtype=torch.float32) % 7) * (rank + 1) * scale)

        def optimizer():
            t.flat.flat.sub_(1e-3 * t.flat.flat_grad)

        t._fwd_bwd, t._optimizer = fwd_bwd, optimizer
        for _ in range(2):
            t.load_batch(*batch(3, 12))
            t.micro_step()
        stepped = digest()
        bad = rec.check()
    return {"before": before, "after": after, "flat": flat_sum, "stepped": stepped, "bad": bad[:5]}


@pytest.mark.parametrize("mapper,freeze", [("transformer", True), ("transformer", False), ("mlp", True)])
def test_trainer_broadcasts_replicas_world2(mapper, freeze):
    out = _run("_replica_broadcast", (mapper, freeze))
    assert out[0]["before"] != out[1]["before"]  # the ranks really built different models
    assert out[0]["after"] == out[1]["after"]  # bitwise-equal replicas after construction
    assert out[0]["flat"] == out[1]["flat"]
    assert out[0]["stepped"] == out[1]["stepped"] and out[0]["stepped"] != out[0]["after"]
    assert not out[0]["bad"] and not out[1]["bad"]


# ---------------------------------------------------------------------------------------- 2. train() shards


def _train_shards(rank, world, outdir):
    import icap
    import icap.weights
    from dryrun import dry_run
    from icap.dataset import SyntheticCaptionDataset
    from test_dryrun_bounds import tiny_model

    ds = SyntheticCaptionDataset(10, max_length=12, real=5, vocab_size=512, eos=511, embed_dim=64)
    seen = []
    with dry_run() as rec:
        icap.weights.ops.call = rec
        model = tiny_model()
        orig = icap.CaptionTrainer.load_batch

        def load_batch(self, ids, *a, **k):
            seen.append([int(row[0]) for row in ids])  # first token identifies the synthetic sample
            return orig(self, ids, *a, **k)

        icap.CaptionTrainer.load_batch = load_batch
        try:
            res = icap.train(ds, model, batch_size=2, num_epochs=2, num_workers=0, device=torch.device("cpu"),
                             outputs_dir=os.path.join(outdir, f"r{rank}"), save_every_epoch=1, use_graph=False)
        finally:
            icap.CaptionTrainer.load_batch = orig
        bad = rec.check()
    saved = sorted(os.listdir(os.path.join(outdir, f"r{rank}")))
    first_tok = [int(ds.ids[i, 0]) for i in range(len(ds))]
    return {"seen": seen, "first_tok": first_tok, "losses": len(res["epoch_losses"]), "bad": bad[:5],
            "saved": [s for s in saved if s.endswith(".pt")]}


def test_train_distributed_sampler_world2():
    with tempfile.TemporaryDirectory() as d:
        out = _run("_train_shards", d)
    n = len(out[0]["first_tok"])
    per_rank_batches = (n // WORLD + 1) // 2
    for epoch in range(2):
        ep = {}
        for r in range(WORLD):
            toks = [t for b in out[r]["seen"][epoch * per_rank_batches:(epoch + 1) * per_rank_batches] for t in b]
            ep[r] = toks
            assert len(toks) == n // WORLD
        assert not set(ep[0]) & set(ep[1]), ep  # disjoint shards
        assert sorted(ep[0] + ep[1]) == sorted(out[0]["first_tok"])  # together: the whole dataset
    for r in range(WORLD):
        assert out[r]["losses"] == 2 and not out[r]["bad"], out[r]
    assert out[0]["saved"] == ["model_epoch_1.pt", "model_epoch_2.pt"]
    assert out[1]["saved"] == []  # checkpoints are written by rank 0 only


# ------------------------------------------------------------------------------------ 3. DP contract (oracle)


def _oracle_dp_grad(rank, world, _):
    from oracle import icap_oracle as O

    gcfg = O.GPT2Cfg(n_layer=2, n_embd=128, n_head=2, vocab_size=512, n_positions=128, eos=511)
    mcfg = O.MapperCfg(embed_dim=64, gpt_dim=128, prefix_length=5, hidden_length=4, num_layers=2)
    gsd = O.gpt2_state_dict(gcfg, seed=0)
    msd = {k: v.clone().requires_grad_(True) for k, v in O.mapper_state_dict(mcfg, seed=0).items()}
    ids, mask, labels, emb = O.synthetic_batch(4, L=12, real=5, vocab=512, eos=511, embed_dim=64)

    def grads(sl):
        for v in msd.values():
            v.grad = None
        prefix = O.mapper_forward(msd, mcfg, emb[sl])
        loss, _ = O.caption_forward(gsd, gcfg, prefix, ids[sl], mask[sl], labels[sl])
        loss.backward()
        return torch.cat([msd[k].grad.reshape(-1) for k in sorted(msd)])

    full = grads(slice(0, 4))
    shard = grads(slice(rank * 2, rank * 2 + 2)) / world
    dist.all_reduce(shard)
    return float((shard - full).abs().max() / full.abs().max())


def test_dp_mean_of_shards_equals_full_batch_world2():
    out = _run("_oracle_dp_grad")
    for r in range(WORLD):
        assert out[r] < 1e-5, out
