"""Helpers of the GEMM path-equality tests (test_gemm256_gpu.py): seeded operands, the kernel-name recorder and
a bitwise comparison that reports where two outputs differ."""

import torch

from icap import ops


def rnd(shape, dev, dtype=torch.bfloat16, scale=1.0, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.randn(shape, generator=g) * scale).to(device=dev, dtype=dtype)


class _Names:
    """ops.GEMM_TIMER hook that records which kernel instantiation each launch used."""

    def __init__(self):
        self.names = []

    def launch(self, key, flops, fn):
        self.names.append(key[0])
        fn()


def _run(fn):
    rec = _Names()
    ops.GEMM_TIMER = rec
    try:
        fn()
    finally:
        ops.GEMM_TIMER = None
    return rec.names


def _assert_same(name, a, b):
    if torch.equal(a, b):
        return
    bad = (a != b).nonzero()
    d = (a.float() - b.float()).abs().max().item()
    rows = sorted(set(bad[:, 0].tolist()))
    cols = sorted(set(bad[:, 1].tolist()))
    raise AssertionError(f"{name}: {bad.shape[0]} of {a.numel()} differ (max |d| {d:.3g}); rows {rows[:12]}"
                         f"{'...' if len(rows) > 12 else ''} ({len(rows)}), cols {cols[:12]}"
                         f"{'...' if len(cols) > 12 else ''} ({len(cols)})")
