"""Run one GEMM shape a few times (for rocprofv3 --pmc / --kernel-trace). Usage: gemm_one.py M N K [reps]"""

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpt2-image-captioning_amd")]

import torch  # noqa: E402

from icap import _lib as L  # noqa: E402
from icap import ops  # noqa: E402


def main():
    M, N, K = (int(x) for x in sys.argv[1:4])
    reps = int(sys.argv[4]) if len(sys.argv) > 4 else 5
    if os.environ.get("ICAP_LIB"):  # A/B against another build of the library
        L.load(os.environ["ICAP_LIB"], strict=False)
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(0)
    A = (torch.rand((M, K), generator=g) * 2 - 1).to(dev, torch.bfloat16)
    B = (torch.rand((N, K), generator=g) * 2 - 1).to(dev, torch.bfloat16)
    C = torch.empty((M, N), device=dev, dtype=torch.bfloat16)
    kw = dict(g256=True, split_k=1) if os.environ.get("GEMM_G256") == "1" else {}
    ops.gemm(A, B, C, **kw)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        ops.gemm(A, B, C, **kw)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / reps * 1e3
    print(f"{os.environ.get('ICAP_LIB', 'current')}: {M}x{N}x{K} {us:.1f} us ({2.0 * M * N * K / us / 1e6:.0f} TF/s)")


if __name__ == "__main__":
    main()
