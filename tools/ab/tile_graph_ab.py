"""Tile-variant A/B in graph replay (diagnostic; needs the diagnostic build: ICAP_LIB=.../libicap_hip_stamps.so, where
ICAP_FORCE_TILE is read). Each (shape, form) is captured as 20 back-to-back launches in a HIP graph with the form's
environment set at capture time (the plan is made on the host then), replayed 5 times; best per-launch us. Forms: the
automatic plan, the tile variants forced unsplit, and torch.mm (hipBLASLt) for the plain products, for scale."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpt2-image-captioning_amd"), os.path.join(ROOT, "tools")]
import torch  # noqa: E402

from gemm_tiles_ab import SHAPES  # noqa: E402
from icap import _lib as L  # noqa: E402
from icap import ops  # noqa: E402

FORMS = [("auto", None), ("v0", "0"), ("v4", "4"), ("v5", "5"), ("v16", "16"), ("g8p128", "g128"), ("r256", "r")]
dev = torch.device("cuda", 0)
REPS = 20


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
print(f"{'shape':44s} " + " ".join(f"{f[0]:>7s}" for f in FORMS) + "  hipBLASLt   (us per launch, graph replay)")
only = os.environ.get("SHAPES")
for M, live, N, K, epi, what in SHAPES:
    if only and not any(o in what for o in only.split(",")):
        continue
    rows = live or M
    A = (torch.rand((M, K), generator=g) * 2 - 1).to(dev, torch.bfloat16)
    B = (torch.rand((N, K), generator=g) * 2 - 1).to(dev, torch.bfloat16)
    C = torch.zeros((M, N), device=dev, dtype=torch.bfloat16)
    kw = {}
    if epi == "gelu_aux":
        kw = dict(bias=torch.zeros(N, device=dev), act=L.ACT_GELU_NEW, aux=torch.empty_like(C))
    elif epi == "qgelu":
        kw = dict(bias=torch.zeros(N, device=dev), act=L.ACT_QUICK_GELU)
    elif epi == "relu_drop":
        kw = dict(bias=torch.zeros(N, device=dev), act=L.ACT_RELU, drop=ops.Dropout(0.1, 1))
    elif epi == "dgelu":
        kw = dict(dact=L.ACT_GELU_NEW, dact_src=torch.randn((M, N), device=dev).to(torch.bfloat16))
    elif epi == "resid_drop":
        kw = dict(bias=torch.zeros(N, device=dev), resid=torch.randn((M, N), device=dev).to(torch.bfloat16),
                  drop=ops.Dropout(0.1, 1))
    elif epi == "resid":
        kw = dict(bias=torch.zeros(N, device=dev), resid=torch.randn((M, N), device=dev).to(torch.bfloat16))
    if live is not None:
        kw.update(m_dev=torch.tensor([live], dtype=torch.int32, device=dev), m_hint=live)
    out = []
    ref = None
    for name, fv in FORMS:
        g8 = int(fv[1:]) if fv and fv.startswith("g") else 0
        rr = fv == "r"
        if fv is None or g8 or rr:
            os.environ.pop("ICAP_FORCE_TILE", None)
        else:
            os.environ["ICAP_FORCE_TILE"] = fv
        try:
            us = per_launch(lambda: ops.gemm(A, B, C, split_k=0 if fv is None else 1, g8p=g8, r256=rr, **kw))
            got = C[:rows].clone()
            if ref is None:
                ref = got
            bad = not torch.allclose(got.float(), ref.float(), rtol=2e-2, atol=2e-2)
            out.append(f"{us:6.1f}{'!' if bad else ' '}")
        except Exception as ex:  # noqa: BLE001
            out.append(f"{'err':>7s}")
            print("   ", name, type(ex).__name__, str(ex)[:120], file=sys.stderr)
    os.environ.pop("ICAP_FORCE_TILE", None)
    lib = ""
    if epi == "plain":
        a = A[:rows]
        lib = f"{per_launch(lambda: torch.mm(a, B.t(), out=C[:rows])):8.1f}"
    print(f"{what + f' {rows}x{N}x{K}':44s} " + " ".join(out) + f"  {lib}", flush=True)
