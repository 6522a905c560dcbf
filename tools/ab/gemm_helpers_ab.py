"""Kernel-name recorder for A/B drivers (the tests' gemm_helpers._Names, without pytest's path setup)."""
from icap import ops


class _Names:
    def __init__(self):
        self.names = []

    def launch(self, key, flops, fn):  # ops.GEMM_TIMER hook
        self.names.append(key[0])
        fn()


def names_of(fn):
    rec = _Names()
    ops.GEMM_TIMER = rec
    try:
        fn()
    finally:
        ops.GEMM_TIMER = None
    return ",".join(n.replace("icap::", "").replace("unsigned short", "bf16") for n in rec.names)
