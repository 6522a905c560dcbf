"""Round 6: the long-K N = 768 products of the step on the 128 x 256 / 96 x 128 split-role rings with a caller's
split-K (fp32 slabs + the reduce pass) against the automatic plan (unsplit 96 x 128 ring) and hipBLASLt. 20 launches
per HIP graph, best of 7 replays (us per launch); '!' = not allclose to the automatic plan's output."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpt2-image-captioning_amd"), os.path.dirname(os.path.abspath(__file__))]
import torch  # noqa: E402

from icap import ops  # noqa: E402
from gemm_helpers_ab import names_of  # noqa: E402
from roles_ab import operands, per_launch  # noqa: E402

dev = torch.device("cuda", 0)
SHAPES = [  # (M capacity, live rows or None, N, K, epilogue, what)
    (8320, 3584, 768, 3072, "plain", "gpt2 c_fc dX"),
    (8320, 3584, 768, 2304, "plain", "gpt2 c_attn dX"),
    (3200, None, 768, 3072, "resid_drop", "mapper linear2 fwd"),
    (3200, None, 768, 3072, "plain", "mapper linear1 dX"),
    (3200, None, 768, 2304, "plain", "mapper qkv dX"),
]


def main():
    g = torch.Generator(device="cpu").manual_seed(0)
    forms = [("auto", {}), ("r256 s2", dict(roles=256, split_k=2)), ("r256 s3", dict(roles=256, split_k=3)),
             ("r96 s2", dict(roles=96, split_k=2)), ("tile s3", dict(split_k=3))]
    print(f"{'shape':40s} " + " ".join(f"{f[0]:>9s}" for f in forms) + f" {'hipBLASLt':>10s}")
    for M, live, N, K, epi, what in SHAPES:
        rows = live or M
        A, B, kw = operands(M, N, K, epi, g)
        C = torch.zeros((M, N), device=dev, dtype=torch.bfloat16)
        ws = torch.empty(4 * M * N, device=dev, dtype=torch.float32)
        if live is not None:
            kw.update(m_dev=torch.tensor([live], dtype=torch.int32, device=dev), m_hint=live)
        cells, ref, names = [], None, []
        for name, extra in forms:
            fn = lambda: ops.gemm(A, B, C, workspace=ws, **kw, **extra)  # noqa: E731
            t = per_launch(fn)
            names.append(names_of(fn).replace("gemm_kernel<bf16, bf16, ", "<"))
            got = C[:rows].float().clone()
            ref = got if ref is None else ref
            ok = torch.allclose(got, ref, rtol=2e-2, atol=2e-2)
            cells.append(f"{t:8.1f}{' ' if ok else '!'}")
        lib = ""
        if epi == "plain":
            a = A[:rows]
            lib = f"{per_launch(lambda: torch.mm(a, B.t(), out=C[:rows])):10.1f}"
        print(f"{what + f' {rows}x{N}x{K}':40s} " + " ".join(cells) + f" {lib:>10s}   " + " | ".join(names),
              flush=True)


if __name__ == "__main__":
    main()
