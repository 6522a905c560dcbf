import os, sys
sys.path[:0] = ["/root/repo", "/root/repo/gpt2-image-captioning_amd", "/root/repo/tests"]
import torch
from icap import CaptionTrainer
from oracle import icap_oracle as O
from test_model_gpu import build
from test_determinism_gpu import _batch, _noise
dev = torch.device("cuda", 0)
B = 32
model = build(O.GPT2Cfg(), O.MapperCfg(), torch.bfloat16, dev)
t = CaptionTrainer(model, B, 50, lr=1e-4, num_training_steps=10, dropout=False)
print("side", t._side)
t.load_batch(*_batch(B, dev))
main = torch.cuda.Stream(dev) if os.environ.get("MAIN_STREAM") == "1" else torch.cuda.current_stream()
print("main stream", main, flush=True)
_fb = t._fwd_bwd
def fb(*a):
    with torch.cuda.stream(main):
        _fb(*a)
    torch.cuda.synchronize()
t._fwd_bwd = fb
t._fwd_bwd(True, 1.0); torch.cuda.synchronize()
t._fwd_bwd(True, 1.0); torch.cuda.synchronize()
ref = t.flat.flat_grad.clone()
names = [n for n, _ in model.named_parameters() if _.requires_grad]
f = t.flat
for rep in range(3):
    launch, s = _noise(dev, 40) if rep > 0 else (lambda: None, torch.cuda.current_stream())
    launch()
    t._fwd_bwd(True, 1.0); torch.cuda.synchronize(); s.synchronize()
    g = t.flat.flat_grad
    bad = []
    for i, p in enumerate(f.params):
        lo = f.offsets[i]; hi = lo + p.numel()
        if not torch.equal(g[lo:hi], ref[lo:hi]):
            bad.append((i, tuple(p.shape), float((g[lo:hi]-ref[lo:hi]).abs().max())))
    idx = [b[0] for b in bad]
    lay = sorted({(i - 3) // 12 for i in idx if i >= 3})
    first = [(i, (i - 3) % 12) for i in idx if i >= 3 and (i - 3) // 12 == (max(lay) if lay else -1)]
    print("rep", rep, "noise" if rep else "quiet", "n", len(bad), "head" if any(i < 3 for i in idx) else "",
          "layers", lay, "top-layer params (idx, j)", first, flush=True)
