"""Diagnostic for tests/test_determinism_gpu.py: which logits elements change between two identical steps, with
and without a concurrent split-K GEMM stream."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpt2-image-captioning_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402

from icap import CaptionTrainer, ops  # noqa: E402
from oracle import icap_oracle as O  # noqa: E402
from test_determinism_gpu import _batch  # noqa: E402
from test_model_gpu import build  # noqa: E402

dev = torch.device("cuda", 0)
B = 32
model = build(O.GPT2Cfg(), O.MapperCfg(), torch.bfloat16, dev)
t = CaptionTrainer(model, B, 50, lr=1e-4, num_training_steps=10, dropout=False)
t.load_batch(*_batch(B, dev))
t._fwd_bwd(True, 1.0)
torch.cuda.synchronize()
t._fwd_bwd(True, 1.0)
torch.cuda.synchronize()
nv = int(t.gws.n_valid.item())
print("n_valid", nv, "logits", tuple(t.gws.logits.shape))
ref = t.gws.logits.clone()
for mode in ("none", "plain", "splitk"):
    s = torch.cuda.Stream(dev)
    a = torch.randn((4096, 4096), device=dev).to(torch.bfloat16)
    c = torch.empty((4096, 4096), device=dev, dtype=torch.bfloat16)
    sa = torch.randn((256, 8192), device=dev).to(torch.bfloat16)
    sc = torch.empty((256, 512), device=dev, dtype=torch.bfloat16)
    torch.cuda.synchronize()
    with torch.cuda.stream(s):
        for i in range(40):
            if mode != "none":
                ops.gemm(a, a, c)
            if mode == "splitk":
                ops.gemm(sa, sa[:512], sc)
    t._fwd_bwd(True, 1.0)
    torch.cuda.synchronize()
    got = t.gws.logits
    diff = ~((got == ref) | (got.isnan() & ref.isnan()))
    idx = diff.nonzero()
    rows = sorted(set(idx[:, 0].tolist()))
    print(mode, "differ", int(diff.sum()), "rows", rows[:10], len(rows), "min row", min(rows) if rows else None,
          "ref nan there", int(ref[diff].isnan().sum()), "got nan there", int(got[diff].isnan().sum()))
    ref = got.clone()
