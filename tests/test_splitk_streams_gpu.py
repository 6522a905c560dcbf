"""Split-K GEMMs on two streams at once with the DEFAULT workspace.

A split-K launch writes fp32 partial slabs into a scratch buffer and a second kernel reduces them. Until r02 that
scratch was one buffer per device, so two split-K GEMMs running concurrently on different streams could overwrite
each other's slabs. ops.gemm_workspace is now keyed by (device, stream): the two chains below interleave freely on
the GPU and every output must be bitwise equal to the same GEMMs run serially on one stream."""

import pytest
import torch

from gemm_helpers import _assert_same, _run, rnd
from icap import ops

pytestmark = pytest.mark.gpu


def test_split_k_two_streams_default_workspace(dev):
    M, N, K = 256, 512, 8192  # 2 x 4 output tiles: split-K is taken (<= 64 tiles)
    names = _run(lambda: ops.gemm(rnd((M, K), dev, seed=1), rnd((N, K), dev, seed=2),
                                  torch.empty((M, N), device=dev, dtype=torch.bfloat16)))
    torch.cuda.synchronize(dev)
    assert names and ops.gemm_workspace(dev, torch.cuda.current_stream(dev)) is not None
    n = 24
    As = [rnd((M, K), dev, seed=10 + i) for i in range(2)]
    Bs = [rnd((N, K), dev, seed=20 + i) for i in range(2)]
    ref = [[torch.empty((M, N), device=dev, dtype=torch.bfloat16) for _ in range(n)] for _ in range(2)]
    for c in range(2):
        for i in range(n):
            ops.gemm(As[c], Bs[c], ref[c][i], alpha=1.0 + i / 8)
    torch.cuda.synchronize(dev)
    out = [[torch.zeros_like(r) for r in ref[c]] for c in range(2)]
    streams = [torch.cuda.Stream(dev) for _ in range(2)]
    ev = torch.cuda.Event()
    ev.record()
    for i in range(n):  # issue both chains alternately: the launches of the two streams overlap on the device
        for c in range(2):
            with torch.cuda.stream(streams[c]):
                if i == 0:
                    streams[c].wait_event(ev)
                ops.gemm(As[c], Bs[c], out[c][i], alpha=1.0 + i / 8)
    torch.cuda.synchronize(dev)
    ws = {ops.gemm_workspace(dev, s).data_ptr() for s in streams}
    assert len(ws) == 2  # two streams, two scratch buffers
    for c in range(2):
        for i in range(n):
            _assert_same(f"chain {c} gemm {i}", out[c][i], ref[c][i])
