"""Launch time vs M at fixed N, K (automatic plan): separates per-CU throughput limits (time linear in M) from
per-block latency limits (time stepping with the number of tile rounds over the CUs).

Usage: python tools/gemm_mscan.py [N K] ...   (default: 768 3072 and 3072 768)
"""

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpt2-image-captioning_amd")]

import torch  # noqa: E402

from icap import ops  # noqa: E402


class _Rec:
    def __init__(self):
        self.names = []

    def launch(self, key, flops, fn):
        self.names.append(key[0].replace("unsigned short", "bf16"))
        fn()


def _name(fn):
    ops.GEMM_TIMER = r = _Rec()
    try:
        fn()
    finally:
        ops.GEMM_TIMER = None
    return r.names[0] if r.names else "?"


def timeit(fn, reps=30):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


MODE = os.environ.get("MODE", "auto")  # auto | ring | tile | g256


def main():
    dev = torch.device("cuda", 0)
    args = [int(a) for a in sys.argv[1:]] or [768, 3072, 3072, 768]
    ms = [int(m) for m in os.environ.get("MS", "1024 2048 3072 4096 5120 6144 7168 8192 8320 9216 10240 12288 "
                                         "16384").split()]
    for N, K in zip(args[::2], args[1::2]):
        B = (torch.rand((N, K), device=dev) * 2 - 1).to(torch.bfloat16)
        for M in ms:
            A = (torch.rand((M, K), device=dev) * 2 - 1).to(torch.bfloat16)
            C = torch.empty((M, N), device=dev, dtype=torch.bfloat16)
            kw = {"auto": {}, "ring": {"ring": True}, "tile": {"tile_only": True}, "g256": {"g256": True}}[MODE]
            name = _name(lambda: ops.gemm(A, B, C, split_k=1, **kw))
            us = timeit(lambda: ops.gemm(A, B, C, split_k=1, **kw))
            tiles = ((M + 127) // 128) * ((N + 127) // 128)
            print(f"M={M:6d} N={N:5d} K={K:5d} tiles128={tiles:5d} per_cu={tiles / 256:5.2f} {us:8.1f} us "
                  f"{2 * M * N * K / us / 1e6:7.1f} TF/s  {name}", flush=True)


if __name__ == "__main__":
    main()
