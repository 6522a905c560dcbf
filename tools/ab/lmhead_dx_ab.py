"""Round 6: the compact LM head's dX product (1664 live target rows of a 6272-row buffer x 768 x K = 50304, split-K
over fp32 slabs + the reduce pass) on the tile kernel and on the split-role rings at several split counts, against
hipBLASLt (torch.mm on the live rows). 10 launches per HIP graph, best of 7 replays (us per launch)."""
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
    Mcap, live, V, D = 6272, 1664, 50304, 768
    md = torch.tensor([live], dtype=torch.int32, device=dev)
    wte_t = ((torch.rand((D, V), generator=g) * 2 - 1) * 0.05).to(dev, torch.bfloat16)
    dl = ((torch.rand((Mcap, V), generator=g) * 2 - 1) * 1e-3).to(dev, torch.bfloat16)
    dh = torch.empty((Mcap, D), device=dev, dtype=torch.bfloat16)
    ws = torch.empty(16 * Mcap * D, device=dev, dtype=torch.float32)
    ref = None
    print("LM head dX 1664 x 768 x 50304 (live rows of 6272)")
    for name, kw in [("tile s6", dict(split_k=6)), ("tile s8", dict(split_k=8)),
                     ("r96 s2", dict(roles=96, split_k=2)), ("r96 s3", dict(roles=96, split_k=3)),
                     ("r96 s4", dict(roles=96, split_k=4)),
                     ("r256 s4", dict(roles=256, split_k=4)), ("r256 s6", dict(roles=256, split_k=6)),
                     ("r256 s8", dict(roles=256, split_k=8)),
                     ("r160 s2", dict(roles=160, split_k=2)), ("r160 s3", dict(roles=160, split_k=3))]:
        fn = lambda: ops.gemm(dl, wte_t, dh, m_dev=md, m_hint=live, M=Mcap, workspace=ws, **kw)  # noqa: E731
        t = per_launch(fn)
        got = dh[:live].float().clone()
        ref = got if ref is None else ref
        ok = torch.allclose(got, ref, rtol=2e-2, atol=2e-4)
        print(f"  {name:8s} {t:8.1f}{' ' if ok else '!'} {names_of(fn)}", flush=True)
    d = dl[:live]
    print(f"  hipBLASLt {per_launch(lambda: torch.mm(d, wte_t.t(), out=dh[:live])):8.1f}", flush=True)
    # the greedy decode's LM head: 128 rows x 50304 x 768 per token
    x = ((torch.rand((128, D), generator=g) * 2 - 1)).to(dev, torch.bfloat16)
    wte = wte_t.t().contiguous()
    lg = torch.empty((128, V), device=dev, dtype=torch.bfloat16)
    print("decode LM head 128 x 50304 x 768")
    ref = None
    for name, kw in [("auto", {}), ("r256", dict(roles=256)), ("r96", dict(roles=96)), ("tile", dict(tile_only=True))]:
        fn = lambda: ops.gemm(x, wte, lg, **kw)  # noqa: E731
        t = per_launch(fn)
        got = lg.float().clone()
        ref = got if ref is None else ref
        print(f"  {name:8s} {t:8.1f}{' ' if torch.equal(got, ref) else '!'} {names_of(fn)}", flush=True)
    print(f"  hipBLASLt {per_launch(lambda: torch.mm(x, wte.t(), out=lg)):8.1f}", flush=True)


if __name__ == "__main__":
    main()
