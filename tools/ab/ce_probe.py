"""Round 6: the compact step's cross-entropy (1664 target rows x 50257 of a 50304-wide bf16 logits buffer, loss +
dlogits in place) per launch, 20 launches per HIP graph, best of 7 replays (us). Run under ICAP_LIB to compare builds."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpt2-image-captioning_amd"), os.path.dirname(os.path.abspath(__file__))]
import torch  # noqa: E402

from icap import ops  # noqa: E402
from roles_ab import per_launch  # noqa: E402

dev = torch.device("cuda", 0)


def main():
    rows, V, ld = 1664, 50257, 50304
    g = torch.Generator().manual_seed(0)
    src = torch.zeros((rows, ld), dtype=torch.bfloat16)
    src[:, :V] = (torch.randn((rows, V), generator=g) * 3).to(torch.bfloat16)
    src = src.to(dev)
    logits = src.clone()
    labels = torch.randint(0, V, (rows,), generator=g, dtype=torch.int32).to(dev)
    nvalid = torch.tensor([rows], dtype=torch.int32, device=dev)
    loss = torch.empty(1, device=dev)
    dl = torch.empty_like(logits)
    ws = torch.empty(ops.cross_entropy_workspace(rows), dtype=torch.uint8, device=dev)
    t = per_launch(lambda: ops.cross_entropy(logits, V, labels, nvalid, loss, dl, ws))
    print(f"cross_entropy {rows} x {V}: {t:7.2f} us  loss {loss.item():.6f}", flush=True)


if __name__ == "__main__":
    main()
