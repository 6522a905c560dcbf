import os, sys
sys.path[:0] = ["/root/repo", "/root/repo/gpt2-image-captioning_amd", "/root/repo/tests"]
import torch
from icap import CaptionTrainer
from oracle import icap_oracle as O
from test_model_gpu import build
from test_determinism_gpu import _batch
dev = torch.device("cuda", 0)
B = 32
model = build(O.GPT2Cfg(), O.MapperCfg(), torch.bfloat16, dev)
t = CaptionTrainer(model, B, 50, lr=1e-4, num_training_steps=10, dropout=False)
print("side", t._side)
if os.environ.get("PROBE_DW_SPLIT"):  # force the K-outer dW split count (1: no slab workspace on the side stream)
    t.dwh.split_k = int(os.environ["PROBE_DW_SPLIT"])
    print("dW split_k", t.dwh.split_k)
t.load_batch(*_batch(B, dev))
w = t.mws
def snap():
    d = {}
    for name in ("g_dz", "g_rm", "g_dqkv", "g_r", "g_m", "g_mm"):
        for l in (7, 6):
            d[f"{name}[{l}]"] = getattr(w, name)[l].clone()
    d["dout"] = w.dout.clone(); d["da"] = w.da.clone(); d["do"] = w.do.clone(); d["flat_grad"] = t.flat.flat_grad.clone()
    return d
snaps = []
for i in range(4):
    t._fwd_bwd(True, 1.0); torch.cuda.synchronize()
    snaps.append(snap())
def ndiff(a, b):
    """(elements that differ as values — NaN == NaN, never-written NaN garbage is not a difference —, max |d|)"""
    same = (a == b) | (a.isnan() & b.isnan())
    n = int((~same).sum())
    d = (a.float() - b.float()).abs()
    d = d[(~same) & d.isfinite()]
    return n, float(d.max()) if d.numel() else 0.0


for i in range(1, 4):
    diff = {k: ndiff(snaps[i][k], snaps[i - 1][k]) for k in snaps[0]}
    diff = {k: v for k, v in diff.items() if v[0]}
    print(f"call {i+1} vs call {i}: differing {diff}", flush=True)
