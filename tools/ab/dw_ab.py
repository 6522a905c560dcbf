"""Round 6: the mapper's K-outer weight-gradient products of the packed B = 128 step (dW[N, K] += dY[3200, N]^T .
X[3200, K], fp32 gradient, bf16 operands read in place) — the automatic plan (split-K slabs + reduce, or in-launch),
the unsplit K-outer kernel, and hipBLASLt (torch.mm on the transposed views, bf16 out: its fastest form). HIP graph
of 20 launches, best of 7 replays, us per launch (reduce launches included)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpt2-image-captioning_amd"), os.path.dirname(os.path.abspath(__file__))]
import torch  # noqa: E402

from icap import ops  # noqa: E402
from gemm_helpers_ab import names_of  # noqa: E402
from roles_ab import per_launch  # noqa: E402

dev = torch.device("cuda", 0)


def main():
    g = torch.Generator().manual_seed(0)
    rows = 3200
    print(f"{'product':28s} {'auto':>8s} {'unsplit':>8s} {'split2':>8s} {'split3':>8s} {'roles':>8s} {'roles1':>8s} "
          f"{'hipBLASLt':>10s}  GF   kernels(auto) | kernels(roles)")
    for N, K, what in [(2304, 768, "qkv"), (768, 768, "out_proj"), (3072, 768, "linear1"), (768, 3072, "linear2")]:
        dY = ((torch.rand((rows, N), generator=g) * 2 - 1) * 0.1).to(dev, torch.bfloat16)
        X = ((torch.rand((rows, K), generator=g) * 2 - 1)).to(dev, torch.bfloat16)
        out = torch.zeros((N, K), device=dev, dtype=torch.float32)
        cells = []
        for sk, ro in ((0, 0), (1, 0), (2, 0), (3, 0), (0, 1), (1, 1)):
            fn = lambda: ops.gemm(dY, X, out, beta=1.0, M=N, N=K, K=rows, trans_ab=True, split_k=sk, roles=ro)  # noqa: E731
            cells.append(per_launch(fn))
        names = names_of(lambda: ops.gemm(dY, X, out, beta=1.0, M=N, N=K, K=rows, trans_ab=True, split_k=0))
        names += " | " + names_of(lambda: ops.gemm(dY, X, out, beta=1.0, M=N, N=K, K=rows, trans_ab=True, split_k=0,
                                                   roles=1))
        o16 = torch.empty((N, K), device=dev, dtype=torch.bfloat16)
        lib = per_launch(lambda: torch.mm(dY.t(), X, out=o16))
        gf = 2.0 * rows * N * K / 1e9
        print(f"{what + f' {N}x{K}x{rows}':28s} " + " ".join(f"{c:8.1f}" for c in cells) + f" {lib:10.1f}  {gf:4.1f} {names}",
              flush=True)


if __name__ == "__main__":
    main()
