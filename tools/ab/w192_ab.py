"""Variant 24 (192 x 64 tiles, ops.gemm(w192=True)) against the automatic plan and hipBLASLt (torch.mm, plain
products only) on the step's N = 768 products, each captured as 20 back-to-back launches in a HIP graph and replayed
5 times (best per-launch us). w192 = path 7 (natural k order); w192s = the automatic plan with ICAP_W192=1, i.e.
variant 24 with the K-skew the plan gives the 128-row tiles — needs the diagnostic build
(ICAP_LIB=.../libicap_hip_stamps.so), where that switch is read at capture time."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpt2-image-captioning_amd"), os.path.dirname(os.path.abspath(__file__))]
import torch  # noqa: E402

from icap import _lib as L  # noqa: E402
from icap import ops  # noqa: E402
from gemm_helpers_ab import names_of  # noqa: E402

dev = torch.device("cuda", 0)
REPS = 20
SHAPES = [  # (M capacity, live rows or None, N, K, epilogue, what)
    (8320, 3584, 768, 768, "resid_drop_lns", "gpt2 attn c_proj fwd (LN stats)"),
    (8320, 3584, 768, 768, "plain", "gpt2 attn c_proj dX"),
    (8320, 3584, 768, 2304, "plain", "gpt2 c_attn dX"),
    (8320, 3584, 768, 3072, "resid_drop", "gpt2 mlp c_proj fwd"),
    (3200, None, 768, 768, "resid_drop", "mapper out_proj fwd"),
    (3200, None, 768, 768, "plain", "mapper 768 dX"),
    (3200, None, 768, 3072, "resid_drop", "mapper linear2 fwd"),
    (6400, None, 768, 768, "resid", "clip out_proj"),
    (6400, None, 768, 3072, "resid", "clip fc2"),
]


def per_launch(body):
    body()
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with ops.graph_capture(gr):
        for _ in range(REPS):
            body()
    gr.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(5):
        e0.record()
        gr.replay()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / REPS)
    del gr
    return best


g = torch.Generator(device="cpu").manual_seed(0)
print(f"{'shape':48s} {'auto':>8s} {'w192':>8s} {'w192s':>8s} {'hipBLASLt':>10s}   (us per launch, graph replay; auto kernel)")
for M, live, N, K, epi, what in SHAPES:
    rows = live or M
    A = (torch.rand((M, K), generator=g) * 2 - 1).to(dev, torch.bfloat16)
    B = (torch.rand((N, K), generator=g) * 2 - 1).to(dev, torch.bfloat16)
    C = torch.zeros((M, N), device=dev, dtype=torch.bfloat16)
    kw = {}
    if epi.startswith("resid"):
        kw = dict(bias=torch.zeros(N, device=dev), resid=torch.randn((M, N), device=dev).to(torch.bfloat16))
        if "drop" in epi:
            kw["drop"] = ops.Dropout(0.1, 1)
        if epi.endswith("lns"):
            kw["ln_stats_out"] = torch.empty((M, N // 32, 2), device=dev)
    if live is not None:
        kw.update(m_dev=torch.tensor([live], dtype=torch.int32, device=dev), m_hint=live)
    auto_name = names_of(lambda: ops.gemm(A, B, C, **kw))
    ta = per_launch(lambda: ops.gemm(A, B, C, **kw))
    ref = C[:rows].float().clone()
    tw = per_launch(lambda: ops.gemm(A, B, C, w192=True, **kw))
    ok = torch.allclose(C[:rows].float(), ref, rtol=2e-2, atol=2e-2)
    os.environ["ICAP_W192"] = "1"
    try:
        ts = per_launch(lambda: ops.gemm(A, B, C, **kw))
        sname = names_of(lambda: ops.gemm(A, B, C, **kw))
    finally:
        os.environ.pop("ICAP_W192", None)
    ok = ok and torch.allclose(C[:rows].float(), ref, rtol=2e-2, atol=2e-2) and "4, 1, 3, 4" in sname
    lib = ""
    if epi == "plain":
        a = A[:rows]
        lib = f"{per_launch(lambda: torch.mm(a, B.t(), out=C[:rows])):10.1f}"
    print(f"{what + f' {rows}x{N}x{K}':48s} {ta:8.1f} {tw:8.1f} {ts:7.1f}{' ' if ok else '!'} {lib:>10s}   {auto_name}",
          flush=True)
