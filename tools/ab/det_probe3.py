"""Side-stream determinism, first layer step only: the forward + GPT-2 backward segment, then the top mapper layer's
backward step (ICAP_SIDE_DW=1 puts its four dW products on the side stream), synchronise, and compare that step's
buffers across 4 calls — localises the first buffer that differs. Diagnostic only."""
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
print("side", t._side, "fused split-K", os.environ.get("ICAP_FUSED_SPLIT_K", "1"))
t.load_batch(*_batch(B, dev))
w = t.mws
L = len(w.g_dz) - 1
names = ["dout", "g_m", "g_dz", "da_after_l1", "g_rm", "g_mm", "do", "g_dqkv", "da", "g_r"]
snaps = []
for i in range(4):
    segs = t._segments(True, 1.0)
    segs[0][1]()
    torch.cuda.synchronize()
    # layer L's step, with probes between its kernels: wrap ops.layernorm_bwd to snapshot `da` as it enters LN#2
    from icap import ops
    orig = ops.layernorm_bwd
    seen = {}
    def lnb(*a, **k):
        torch.cuda.synchronize()
        if "da_after_l1" not in seen:
            seen["da_after_l1"] = w.da.clone()
        return orig(*a, **k)
    ops.layernorm_bwd = lnb
    segs[1][1]()
    ops.layernorm_bwd = orig
    torch.cuda.synchronize()
    d = {"dout": w.dout.clone(), "g_m": w.g_m[L].clone(), "g_dz": w.g_dz[L].clone(), "g_rm": w.g_rm[L].clone(),
         "g_mm": w.g_mm[L].clone(), "do": w.do.clone(), "g_dqkv": w.g_dqkv[L].clone(), "da": w.da.clone(),
         "g_r": w.g_r[L - 1].clone(), "da_after_l1": seen["da_after_l1"]}
    snaps.append(d)
for i in range(1, 4):
    diff = [k for k in names if not torch.equal(snaps[i][k], snaps[i - 1][k])]
    print(f"call {i+1} vs call {i}: differing {diff}", flush=True)
