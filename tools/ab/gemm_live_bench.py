"""GEMMs of the packed train step (GPT2Core.alloc_train(pack=True)): the GPT-2 block products over MLIVE live token
rows of a capacity-MCAP buffer (device row count m_dev), against the same product on a plain M = MLIVE buffer and on
the padded M = MCAP. Random bf16 operands, HIP-event timing, interleaved in one process.

Usage: [MLIVE=3584] [MCAP=8320] [REPS=20] python tools/gemm_live_bench.py
"""

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpt2-image-captioning_amd")]

import torch  # noqa: E402

from icap import _lib as L  # noqa: E402
from icap import ops  # noqa: E402

# (N, K, epilogue) of one GPT-2 small block, forward then backward dX
SHAPES = [(2304, 768, "bias"), (768, 768, "resid_drop"), (3072, 768, "gelu_aux"), (768, 3072, "resid_drop"),
          (3072, 768, "dgelu"), (768, 3072, "plain"), (768, 768, "plain"), (768, 2304, "plain")]


def main():
    dev = torch.device("cuda", 0)
    mlive = int(os.environ.get("MLIVE", "3584"))
    mcap = int(os.environ.get("MCAP", "8320"))
    reps = int(os.environ.get("REPS", "20"))
    g = torch.Generator(device="cpu").manual_seed(0)
    mdev = torch.tensor([mlive], dtype=torch.int32, device=dev)
    mfull = torch.tensor([mcap], dtype=torch.int32, device=dev)
    tot = [0.0, 0.0, 0.0]
    for N, K, epi in SHAPES:
        A = (torch.rand((mcap, K), generator=g) * 2 - 1).to(dev, torch.bfloat16)
        B = (torch.rand((N, K), generator=g) * 2 - 1).to(dev, torch.bfloat16)
        C = torch.zeros((mcap, N), device=dev, dtype=torch.bfloat16)
        kw = {}
        if epi == "bias":
            kw = dict(bias=torch.zeros(N, device=dev))
        elif epi == "gelu_aux":
            kw = dict(bias=torch.zeros(N, device=dev), act=L.ACT_GELU_NEW, aux=torch.empty_like(C))
        elif epi == "dgelu":
            kw = dict(dact=L.ACT_GELU_NEW, dact_src=torch.randn((mcap, N), device=dev).to(torch.bfloat16))
        elif epi == "resid_drop":
            kw = dict(bias=torch.zeros(N, device=dev), resid=torch.empty_like(C), drop=ops.Dropout(0.1, 1))
        forms = [("padded", dict(M=mcap)), ("m_dev", dict(M=mcap, m_dev=mdev)), ("plain", dict(M=mlive))]
        if K >= 2304:  # long K: the double-buffered tile kernel (hint = capacity) vs the 4-stage ring (hint = live),
            # and the padded product forced onto the ring (m_dev = capacity, small hint)
            forms += [("nst2", dict(M=mcap, m_dev=mdev, m_hint=mcap)), ("ring", dict(M=mcap, m_dev=mdev, m_hint=mlive)),
                      ("padded-ring", dict(M=mcap, m_dev=mfull, m_hint=mlive))]
        res = []
        name = None
        for label, f in forms:
            for _ in range(3):
                ops.gemm(A, B, C, **f, **kw)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                ops.gemm(A, B, C, **f, **kw)
            e1.record()
            torch.cuda.synchronize()
            res.append(e0.elapsed_time(e1) * 1e3 / reps)
        a = L.GemmArgs()
        for i, us in enumerate(res[:3]):
            tot[i] += us
        fl_live = 2 * mlive * N * K
        extra = "".join(f" | {lab} {us:7.1f} us" for (lab, _), us in zip(forms[3:], res[3:]))
        print(f"{N:5d}x{K:5d} {epi:10s} padded(M={mcap}) {res[0]:7.1f} us | m_dev({mlive}) {res[1]:7.1f} us "
              f"{fl_live / res[1] / 1e6:6.1f} TF/s | plain(M={mlive}) {res[2]:7.1f} us {fl_live / res[2] / 1e6:6.1f} TF/s"
              + extra, flush=True)
        del a, name
    print(f"sum per block: padded {tot[0]:.1f} us, m_dev {tot[1]:.1f} us, plain {tot[2]:.1f} us")


if __name__ == "__main__":
    main()
