"""AdamW update variants on the headline's flat buffer (n = trainable params of the packed B = 128 step, fp32 params /
grads / moments + the bf16 compute copy): the one-strip kernel against ICAP_ADAM_U strips per thread and
non-temporal stores (ICAP_ADAM_NT), bitwise-checked against it, each timed as a HIP graph of REPS updates;
then the gradient-norm pass alone with ICAP_SQ_U strips per pass.

    python tools/ab/adam_probe.py
"""

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpt2-image-captioning_amd")]

import torch  # noqa: E402

from icap import ops  # noqa: E402

FORMS = [("1", "0"), ("1", "1"), ("2", "0"), ("2", "1"), ("4", "0"), ("4", "1")]


def main():
    dev = torch.device("cuda", 0)
    n = int(os.environ.get("N", "60653571"))
    reps = int(os.environ.get("REPS", "20"))
    g = torch.Generator(device="cpu").manual_seed(0)
    p0 = torch.randn(n, generator=g).to(dev)
    gr = (torch.randn(n, generator=g) * 1e-3).to(dev)
    m0 = (torch.randn(n, generator=g) * 1e-4).to(dev)
    v0 = (torch.rand(n, generator=g) * 1e-6).to(dev)
    ws = torch.empty(1 << 20, device=dev)
    ref = None
    print(f"{'ICAP_ADAM_U / NT':18s} {'us':>8s} {'GB':>6s} {'TB/s':>6s}  bitwise vs one-strip")
    for u, nt in FORMS:
        os.environ["ICAP_ADAM_U"], os.environ["ICAP_ADAM_NT"] = u, nt
        p, m, v = p0.clone(), m0.clone(), v0.clone()
        out16 = torch.empty(n, dtype=torch.bfloat16, device=dev)
        st = torch.zeros(16, device=dev)
        kw = dict(lr=1e-4, num_warmup_steps=0, num_training_steps=1000, bf16_out=out16)
        ops.adamw_step(p, gr, m, v, st, ws, **kw)  # one checked update from the same start
        torch.cuda.synchronize()
        res = (p.clone(), m.clone(), v.clone(), out16.clone())
        if ref is None:
            ref = res
        same = all(torch.equal(a, b) for a, b in zip(res, ref))
        gph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gph):
            for _ in range(reps):
                ops.adamw_step(p, gr, m, v, st, ws, **kw)
        gph.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        gph.replay()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / reps
        gb = n * (4 * 4 + 3 * 4 + 2 + 4) / 1e9  # update: p g m v in, p m v + bf16 out; + the norm pass over g
        print(f"U={u} NT={nt}{'':10s} {us:8.1f} {gb:6.2f} {gb / us * 1e3:6.2f}  {same}", flush=True)
        del gph
    os.environ.pop("ICAP_ADAM_U"), os.environ.pop("ICAP_ADAM_NT")
    # the gradient norm pass alone (icap_sqnorm: partials + the fp64 finalize), ICAP_SQ_U strips per pass
    out = torch.zeros(1, device=dev)
    ref = None
    for u in ("1", "2", "4"):
        os.environ["ICAP_SQ_U"] = u
        ops.sqnorm(gr, out, ws)
        torch.cuda.synchronize()
        val = out.clone()
        ref = val if ref is None else ref
        gph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gph):
            for _ in range(reps):
                ops.sqnorm(gr, out, ws)
        gph.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        gph.replay()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / reps
        print(f"sqnorm ICAP_SQ_U={u}{'':5s} {us:8.1f} {n * 4 / 1e9:6.2f} {n * 4 / us / 1e3:6.2f}  {torch.equal(val, ref)}",
              flush=True)
        del gph
    os.environ.pop("ICAP_SQ_U")


if __name__ == "__main__":
    main()
