"""In-launch split-K (icap_gemm_args.tickets): long-K products over fewer output tiles than CUs split K 2-4 ways and
the last split of each tile to finish adds the others' fp32 partials (sc1 hand-off, split order) and applies the
epilogue. Checked: the kernel choice (no reduce launch), agreement with the unsplit product (fp32 accumulation in a
different order: bf16 outputs within one bf16 rounding, f32 outputs within 1e-5 relative), bitwise run-to-run
determinism, and that the tickets are left zero after every launch (the next launch's precondition)."""

import pytest
import torch

from icap import _lib as L
from icap import ops

pytestmark = pytest.mark.gpu


def _kernel_names(fn):
    """(kernel name, splits, fused) of every icap_gemm call fn makes."""
    import ctypes as C

    names = []
    real = ops.call

    def rec(name, *args):
        if name == "icap_gemm":
            sp, fu = C.c_int32(), C.c_int32()
            assert L.load().icap_gemm_plan_info(args[0], C.byref(sp), C.byref(fu)) == 0
            names.append((L.load().icap_gemm_kernel_name(args[0]).decode(), sp.value, fu.value))
        return real(name, *args)

    ops.call = rec
    try:
        fn()
    finally:
        ops.call = real
    return names


# (the K-outer weight-gradient products keep the slab + reduce pass: tests/test_kernels_gpu.py covers them)
CASES = [  # M (capacity), live rows or None, N, K, epilogue, trans_ab (bf16 inputs; "f32in_*": fp32 parity mode)
    (8320, 3584, 768, 3072, "resid_drop", False),
    (260, None, 768, 3072, "f32in_resid_drop", False),
    (260, None, 3072, 768, "f32in_gelu_aux", False),
    (260, None, 3072, 768, "f32in_dgelu", False),
    (300, None, 768, 3072, "f32in_beta", False),
    (260, None, 768, 3072, "dgelu", False),
    (3200, None, 768, 2304, "plain", False),
    (3200, None, 768, 3072, "f32beta", False),
]


@pytest.mark.parametrize("M,live,N,K,epi,kout", CASES)
def test_fused_split_k(dev, M, live, N, K, epi, kout):
    g = torch.Generator().manual_seed(M + N + K)
    f32in = epi.startswith("f32in_")
    idt = torch.float32 if f32in else torch.bfloat16
    epi = epi[6:] if f32in else epi
    if kout:
        A = (torch.rand((K, M), generator=g) * 2 - 1).to(dev, idt)
        B = (torch.rand((K, N), generator=g) * 2 - 1).to(dev, idt)
    else:
        A = (torch.rand((M, K), generator=g) * 2 - 1).to(dev, idt)
        B = (torch.rand((N, K), generator=g) * 2 - 1).to(dev, idt)
    cdt = torch.float32 if (f32in or epi in ("f32beta", "beta")) else torch.bfloat16
    C0 = (torch.randn((M, N), generator=g) if epi in ("f32beta", "beta") else torch.zeros((M, N))).to(dev, cdt)
    # (tile_only: the 128-row tile kernels, whose long-K launches over few tiles split K; the automatic plan gives the
    # bf16 N <= 1024 ones to the unsplit split-role ring since round 6)
    kw = dict(trans_ab=kout, tile_only=True)
    if epi == "resid_drop":
        kw.update(bias=torch.randn(N, generator=g).to(dev), resid=torch.randn((M, N), generator=g).to(dev, cdt),
                  drop=ops.Dropout(0.1, 3))
    if epi in ("f32beta", "beta"):
        kw.update(beta=1.0)
    if epi == "gelu_aux":
        kw.update(bias=torch.randn(N, generator=g).to(dev), act=L.ACT_GELU_NEW, aux=torch.zeros((M, N), device=dev,
                                                                                                 dtype=cdt))
    if epi == "dgelu":
        kw.update(dact=L.ACT_GELU_NEW, dact_src=torch.randn((M, N), generator=g).to(dev, cdt))
    if live is not None:
        kw.update(m_dev=torch.tensor([live], dtype=torch.int32, device=dev), m_hint=live)
    rows = live or M
    outs, auxs, names = [], [], []
    # fused (twice: determinism); the same split through a caller-supplied workspace (no tickets: slab + reduce
    # pass, same split count by the shape rule); unsplit
    ws_own = torch.empty(4 * M * N, dtype=torch.float32, device=dev)
    for split, ws in ((0, None), (0, None), (0, ws_own), (1, None)):
        C = C0.clone()
        if "aux" in kw:
            kw["aux"] = torch.zeros((M, N), device=dev, dtype=cdt)
        names.append(_kernel_names(lambda: ops.gemm(A, B, C, split_k=split, workspace=ws, **kw)))
        outs.append(C)
        auxs.append(kw.get("aux"))
    torch.cuda.synchronize()
    assert len(names[0]) == 1 and names[0][0][1] >= 2 and names[0][0][2] == 1, names[0]  # combined in the launch
    assert names[2][0][1] == names[0][0][1] and names[2][0][2] == 0, names[2]  # same split, reduce pass
    assert names[3][0][1] == 1, names[3]
    assert torch.equal(outs[0], outs[1])
    # the split count is a function of the shape alone: the slab mechanism sums in the same order (bitwise equal)
    assert torch.equal(outs[0], outs[2])
    a, b = outs[0][:rows].float(), outs[3][:rows].float()

    def close(a, b):
        if cdt == torch.bfloat16:
            assert float((a - b).abs().max() / b.abs().max()) < 1.6e-2
            assert float(((a - b).abs() > 1e-2 * b.abs().max()).float().mean()) < 1e-3
        else:
            assert float((a - b).abs().max() / b.abs().max()) < 1e-5

    close(a, b)
    if "aux" in kw:  # the pre-activation the fused launch stored, against the unsplit launch's
        assert torch.equal(auxs[0], auxs[2])
        close(auxs[0][:rows].float(), auxs[3][:rows].float())
    if live is not None:
        assert torch.equal(outs[0][live:], C0[live:])
    ws = ops.gemm_workspace(dev, torch.cuda.current_stream(dev))
    tk = ops._gemm_tickets[ws.data_ptr()]
    assert int(torch.count_nonzero(tk)) == 0  # left zero for the next launch


def test_workspace_too_small_raises(dev):
    """A caller workspace smaller than the shape's split needs is an error, never a different split."""
    A = torch.randn((3200, 3072), device=dev).to(torch.bfloat16)
    B = torch.randn((768, 3072), device=dev).to(torch.bfloat16)
    C = torch.empty((3200, 768), device=dev, dtype=torch.bfloat16)
    with pytest.raises(L.IcapError):
        ops.gemm(A, B, C, workspace=torch.empty(1024, dtype=torch.float32, device=dev), tile_only=True)
