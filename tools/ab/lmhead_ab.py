"""Round 6: the compact LM head of the packed B = 128 step (1664 live target rows of a 6272-row buffer; vocab padded
to 50304; K = 768) and its dX product (K = 50304), on each GEMM form that takes a device row count, against
hipBLASLt (torch.mm on the live rows). 10 launches per HIP graph, best of 5 replays (us per launch)."""
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
    hf = (torch.rand((Mcap, D), generator=g) * 2 - 1).to(dev, torch.bfloat16)
    wte = ((torch.rand((V, D), generator=g) * 2 - 1) * 0.05).to(dev, torch.bfloat16)
    wte_t = wte.t().contiguous()
    logits = torch.empty((Mcap, V), device=dev, dtype=torch.bfloat16)
    dl = ((torch.rand((Mcap, V), generator=g) * 2 - 1) * 1e-3).to(dev, torch.bfloat16)
    dh = torch.empty((Mcap, D), device=dev, dtype=torch.bfloat16)
    forms = [("auto", {}), ("r256", dict(roles=256)), ("g8p256", dict(g8p=256)), ("g8p128", dict(g8p=128)),
             ("r96", dict(roles=96))]
    print("LM head forward 1664 x 50304 x 768 (live rows of 6272)")
    for name, kw in forms:
        fn = lambda: ops.gemm(hf, wte, logits, m_dev=md, m_hint=live, M=Mcap, **kw)  # noqa: E731
        try:
            t = per_launch(fn)
            print(f"  {name:8s} {t:8.1f}  {names_of(fn)}", flush=True)
        except Exception as e:  # a form that does not take this launch
            print(f"  {name:8s} not eligible: {e}", flush=True)
    a = hf[:live]
    print(f"  hipBLASLt {per_launch(lambda: torch.mm(a, wte.t(), out=logits[:live])):8.1f}", flush=True)
    print("LM head dX 1664 x 768 x 50304")
    for name, kw in [("auto", {}), ("split4", dict(split_k=4)), ("split8", dict(split_k=8)),
                     ("split12", dict(split_k=12)), ("split16", dict(split_k=16))]:
        fn = lambda: ops.gemm(dl, wte_t, dh, m_dev=md, m_hint=live, M=Mcap, **kw)  # noqa: E731
        t = per_launch(fn)
        print(f"  {name:8s} {t:8.1f}  {names_of(fn)}", flush=True)
    d = dl[:live]
    print(f"  hipBLASLt {per_launch(lambda: torch.mm(d, wte_t.t(), out=dh[:live])):8.1f}", flush=True)


if __name__ == "__main__":
    main()
