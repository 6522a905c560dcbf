"""The data-parallel path on real RCCL: a world-size-1 `nccl` process group on the one GPU.

CaptionTrainer built under the group broadcasts its replicas through RCCL at construction, and with
CaptionTrainer(force_overlap=True) takes the overlapped data-parallel step even at world size 1: each segment of the step is
its own HIP graph, each segment's flat-gradient ranges are all-reduced asynchronously on the communication stream
behind an event, and the optimizer graph waits for the handles (engine.CaptionTrainer._overlapped_step). A
one-rank SUM all-reduce is the identity, so after every step the parameters must be BITWISE equal to the plain
single-graph step of an identical model with no process group (same kernels, same order, same dropout counter).
The bf16 exchange (dp_bf16=True) rounds the sum and is checked against its own bound instead."""

import os
import socket

import pytest
import torch
import torch.distributed as dist

from icap import CaptionTrainer
from oracle import icap_oracle as O
from test_model_gpu import build

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _batch(B, dev):
    ids, mask, labels, _ = O.synthetic_batch(B, 50, 13, seed=5)
    emb = torch.randn((B, 512), generator=torch.Generator().manual_seed(6))
    return ids.to(dev), mask.to(dev), labels.to(dev), (emb / emb.norm(dim=-1, keepdim=True)).to(dev)


def _run(model, batch, steps, **kw):
    t = CaptionTrainer(model, batch[0].shape[0], 50, lr=1e-3, num_training_steps=steps + 2, dropout=True, seed=11,
                       **kw)
    t.load_batch(*batch)
    losses = []
    for _ in range(steps):
        t.micro_step(use_graph=True)
        losses.append(float(t.last_loss.item()))
    torch.cuda.synchronize()
    return t, losses


class _NcclWorld1:
    def __init__(self, dev):
        self.dev = dev

    def __enter__(self):
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_port()}", rank=0, world_size=1,
                                device_id=self.dev)

    def __exit__(self, *exc):
        dist.destroy_process_group()


def test_overlapped_rccl_step_bitwise_equals_single_graph(dev, monkeypatch):
    B, steps = 16, 3
    batch = _batch(B, dev)
    ref_model = build(O.GPT2Cfg(), O.MapperCfg(), torch.bfloat16, dev)
    t_ref, l_ref = _run(ref_model, batch, steps)  # no process group: the plain single-graph step
    assert not t_ref.distributed and not t_ref.force_overlap

    with _NcclWorld1(dev):
        model = build(O.GPT2Cfg(), O.MapperCfg(), torch.bfloat16, dev)
        t, losses = _run(model, batch, steps, force_overlap=True)
    assert t.distributed and t.force_overlap and t.world == 1
    assert t.seg_graphs, "the overlapped (segment-graph + comm-stream) path did not run"
    assert losses == l_ref, (losses, l_ref)
    assert torch.equal(t.flat.flat, t_ref.flat.flat)
    assert torch.equal(t.flat.exp_avg_sq, t_ref.flat.exp_avg_sq)
    assert torch.equal(t.flat.flat_c, t_ref.flat.flat_c)


def test_overlapped_rccl_step_bf16_exchange(dev, monkeypatch):
    B, steps = 16, 2
    batch = _batch(B, dev)
    ref_model = build(O.GPT2Cfg(), O.MapperCfg(), torch.bfloat16, dev)
    init = ref_model.flat().flat.clone()
    t_ref, l_ref = _run(ref_model, batch, steps)
    with _NcclWorld1(dev):
        model = build(O.GPT2Cfg(), O.MapperCfg(), torch.bfloat16, dev)
        t, losses = _run(model, batch, steps, force_overlap=True, dp_bf16=True)
    assert t.dp_bf16 and t.seg_graphs
    assert abs(losses[0] - l_ref[0]) == 0.0  # the first loss precedes any exchange
    upd, upd_ref = t.flat.flat - init, t_ref.flat.flat - init
    cos = float(torch.nn.functional.cosine_similarity(upd.double(), upd_ref.double(), dim=0))
    assert cos > 0.98, cos  # bf16-rounded gradients, AdamW-normalised: the same update direction
