"""Per-launch timing of one greedy-decode token's kernels at the benchmarked shape (GPT-2 small, B=128 rows):
the four block GEMMs with their decode epilogues (LN-fused QKV / c_fc, residual out-proj / c_proj), the same GEMMs
without LN / epilogue, decode attention at several cache lengths, the LM head and the argmax/next-embedding step.
Each case is a HIP graph of REPS back-to-back launches (the decode runner replays graphs), timed with HIP events.

Usage: python tools/decode_bench.py   [REPS=200]
"""

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpt2-image-captioning_amd")]

import torch  # noqa: E402

from icap import _lib as L  # noqa: E402
from icap import ops  # noqa: E402


def timed(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    dev = torch.device("cuda", 0)
    reps = int(os.environ.get("REPS", "200"))
    B, D, H, hd, V, Vp = 128, 768, 12, 64, 50257, 50304
    bf = torch.bfloat16
    r = lambda *s: (torch.randn(*s, device=dev) * 0.05).to(bf)  # noqa: E731
    x, h1, o = r(B, D), r(B, D), r(B, D)
    f = r(B, 4 * D)
    w_attn, w_proj, w_fc, w_mp, wte = r(3 * D, D), r(D, D), r(4 * D, D), r(D, 4 * D), r(Vp, D)
    b3, b1, b4 = [torch.zeros(n, device=dev) for n in (3 * D, D, 4 * D)]
    g1, be1 = torch.ones(D, device=dev), torch.zeros(D, device=dev)
    qkv, out1, out4 = r(B, 3 * D), r(B, D), r(B, 4 * D)
    logits = r(B, Vp)
    T = 65
    cache = r(T * B, 3 * D)
    ln = (g1, be1, 1e-5)
    rows = []

    def case(name, fn, nbytes):
        us = timed(fn, reps)
        rows.append((name, us, nbytes))
        print(f"{name:44s} {us:8.2f} us  {nbytes / us / 1e6:8.3f} TB/s", flush=True)

    wb = lambda w: w.numel() * 2  # noqa: E731
    case("qkv   128x2304x768  ln+bias", lambda: ops.gemm(x, w_attn, qkv, bias=b3, M=B, ln=ln), wb(w_attn))
    wsa = w_attn.float().sum(1)
    case("qkv   128x2304x768  fold+bias", lambda: ops.gemm(x, w_attn, qkv, bias=b3, M=B, ln_fold=(wsa, 1e-5)),
         wb(w_attn))
    case("qkv   128x2304x768  bias", lambda: ops.gemm(x, w_attn, qkv, bias=b3, M=B), wb(w_attn))
    case("qkv   128x2304x768  plain", lambda: ops.gemm(x, w_attn, qkv, M=B), wb(w_attn))
    case("proj  128x768x768   bias+resid", lambda: ops.gemm(o, w_proj, out1, bias=b1, resid=x, M=B), wb(w_proj))
    case("proj  128x768x768   plain", lambda: ops.gemm(o, w_proj, out1, M=B), wb(w_proj))
    case("fc    128x3072x768  ln+bias+gelu",
         lambda: ops.gemm(h1, w_fc, out4, bias=b4, act=L.ACT_GELU_NEW, M=B, ln=ln), wb(w_fc))
    wsf = w_fc.float().sum(1)
    case("fc    128x3072x768  fold+bias+gelu",
         lambda: ops.gemm(h1, w_fc, out4, bias=b4, act=L.ACT_GELU_NEW, M=B, ln_fold=(wsf, 1e-5)), wb(w_fc))
    case("fc    128x3072x768  plain", lambda: ops.gemm(h1, w_fc, out4, M=B), wb(w_fc))
    case("mp    128x768x3072  bias+resid", lambda: ops.gemm(f, w_mp, out1, bias=b1, resid=h1, M=B), wb(w_mp))
    case("mp    128x768x3072  plain", lambda: ops.gemm(f, w_mp, out1, M=B), wb(w_mp))
    for pos in (16, 40, 64):
        kv = 2 * B * H * (pos + 1) * hd * 2
        case(f"attn_decode pos={pos}",
             lambda pos=pos: ops.attention_decode(cache, o, B=B, H=H, hd=hd, pos=pos, scale=0.125), kv)
    case("ln_f  128x768", lambda: ops.layernorm_fwd(x, g1, be1, 1e-5, h1, None, None, rows=B), 2 * B * D * 2)
    case("lm_head 128x50304x768", lambda: ops.gemm(x, wte, logits, M=B), wb(wte))
    fin = torch.zeros(B, dtype=torch.int32, device=dev)
    toks = torch.zeros((B, 50), dtype=torch.int64, device=dev)
    wpe = r(1024, D)
    case("greedy_next 128x50257", lambda: ops.greedy_next(logits, V, 50256, fin, toks, 3, wte, wpe, 70, D, x),
         B * Vp * 2)
    per_token = sum(us for n, us, _ in rows if n.startswith(("qkv   128x2304x768  fold", "proj  128x768x768   bias",
                                                               "fc    128x3072x768  fold", "mp    128x768x3072  bias",
                                                               "attn_decode pos=40")))
    head = sum(us for n, us, _ in rows if n.startswith(("ln_f", "lm_head", "greedy_next")))
    print(f"estimated token: 12 x {per_token:.1f} + head {head:.1f} = {12 * per_token + head:.1f} us")


if __name__ == "__main__":
    main()
