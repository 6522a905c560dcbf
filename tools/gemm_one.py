"""Run one GEMM shape a few times (for rocprofv3 --pmc / --kernel-trace). Usage: gemm_one.py M N K [reps]"""

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpt2-image-captioning_amd")]

import torch  # noqa: E402

from icap import ops  # noqa: E402


def main():
    M, N, K = (int(x) for x in sys.argv[1:4])
    reps = int(sys.argv[4]) if len(sys.argv) > 4 else 5
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(0)
    A = (torch.rand((M, K), generator=g) * 2 - 1).to(dev, torch.bfloat16)
    B = (torch.rand((N, K), generator=g) * 2 - 1).to(dev, torch.bfloat16)
    C = torch.empty((M, N), device=dev, dtype=torch.bfloat16)
    for _ in range(reps):
        ops.gemm(A, B, C)
    torch.cuda.synchronize()
    print("done", M, N, K, reps)


if __name__ == "__main__":
    main()
