"""Side-stream determinism, per-launch localisation. Diagnostic only.

Runs the forward + GPT-2 backward segment, then the top two mapper layer steps with ICAP_SIDE_DW=1 (the four dW
products of each layer on the side stream). Every main-stream icap launch of those steps (ops.gemm,
ops.layernorm_bwd, ops.attention_bwd, ops.dropout_apply) is followed by a clone of its output ON THE MAIN STREAM (a
stream-ordered copy: it sees exactly what the launch wrote, without a device-wide sync that would remove the
concurrency). Over 4 calls from the same state the first launch whose output differs is reported with its max |diff|
and max |value| (ulps vs corruption). Run once per environment variant (the library reads its switches at load).
"""
import os
import sys

sys.path[:0] = ["/root/repo", "/root/repo/gpt2-image-captioning_amd", "/root/repo/tests"]
import torch  # noqa: E402

from icap import CaptionTrainer, ops  # noqa: E402
from oracle import icap_oracle as O  # noqa: E402
from test_model_gpu import build  # noqa: E402
from test_determinism_gpu import _batch  # noqa: E402

dev = torch.device("cuda", 0)
B = int(os.environ.get("PROBE_B", "32"))
model = build(O.GPT2Cfg(), O.MapperCfg(), torch.bfloat16, dev)
t = CaptionTrainer(model, B, 50, lr=1e-4, num_training_steps=10, dropout=False)
tag = " ".join(f"{k}={os.environ[k]}" for k in sorted(os.environ) if k.startswith("ICAP_"))
print("variant:", tag or "(defaults)", "side", t._side is not None, flush=True)
t.load_batch(*_batch(B, dev))

OUT_ARG = {"gemm": 2, "layernorm_bwd": 5, "attention_bwd": 3, "dropout_apply": 1}
orig = {k: getattr(ops, k) for k in OUT_ARG}
rec = []


def wrap(name):
    f = orig[name]

    def g(*a, **k):
        r = f(*a, **k)
        out = a[OUT_ARG[name]] if len(a) > OUT_ARG[name] else None
        if out is not None and torch.cuda.current_stream() == torch.cuda.default_stream():
            rec.append((f"{name}#{len(rec)} {tuple(out.shape)}", out.detach().clone()))
        return r
    return g


calls = []
for i in range(4):
    segs = t._segments(True, 1.0)
    segs[0][1]()
    torch.cuda.synchronize()
    rec.clear()
    for k in OUT_ARG:
        setattr(ops, k, wrap(k))
    segs[1][1]()  # top layer
    segs[2][1]()  # next layer
    for k, f in orig.items():
        setattr(ops, k, f)
    torch.cuda.synchronize()
    calls.append(list(rec))
    # the rest of the step (keeps the state identical from call to call: grads overwrite)
    for _, fn in segs[3:]:
        fn()
    torch.cuda.synchronize()

n_bad = 0
for i in range(1, 4):
    a, b = calls[i - 1], calls[i]
    first = None
    nd = 0
    for (na, xa), (nb, xb) in zip(a, b):
        same = ((xa == xb) | (xa.isnan() & xb.isnan())).all().item()
        if not same:
            nd += 1
            if first is None:
                d = (xa.float() - xb.float()).abs()
                d[d.isnan()] = 0
                ne = int((xa != xb).sum())
                first = (na, ne, float(d.max()), float(xa.float().abs().nan_to_num().max()))
    n_bad += nd
    print(f"call {i + 1} vs {i}: {nd} of {len(a)} launches differ; first {first}", flush=True)
print("RESULT", "deterministic" if n_bad == 0 else "NONDETERMINISTIC", tag, flush=True)
