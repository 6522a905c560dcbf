"""Patch-embed timing (diagnostic): the fused gather GEMM (icap_patch_embed) against the round-4 form (im2col into a
bf16 patch matrix + tile GEMM + icap_vit_embed), HIP events over 20 launches each, for the towers' shapes."""
import sys

sys.path[:0] = ["/root/repo", "/root/repo/gpt2-image-captioning_amd"]
import torch  # noqa: E402

from icap import ops  # noqa: E402

dev = torch.device("cuda", 0)
for name, B, HW, p, N, NP in (("clip_b32", 128, 224, 32, 768, 1), ("clip_l14", 128, 224, 14, 1024, 1),
                              ("dino_l16", 128, 224, 16, 1024, 5)):
    g = torch.Generator().manual_seed(0)
    K = 3 * p * p
    Kp = (K + 7) // 8 * 8
    px = torch.randn((B, 3, HW, HW), generator=g).to(dev)
    w = torch.zeros((N, Kp), dtype=torch.bfloat16, device=dev)
    w[:, :K] = (torch.randn((N, K), generator=g) * 0.02).to(dev, torch.bfloat16)
    G2 = (HW // p) ** 2
    S = NP + G2
    prefix = torch.randn((NP, N), generator=g).to(dev)
    pos = torch.randn((S, N), generator=g).to(dev)
    out = torch.empty((B * S, N), dtype=torch.bfloat16, device=dev)
    patches = torch.zeros((B * G2, Kp), dtype=torch.bfloat16, device=dev)
    pe = torch.empty((B * G2, N), dtype=torch.bfloat16, device=dev)
    out2 = torch.empty_like(out)

    def fused():
        ops.patch_embed(px, w, out, patch=p, prefix=prefix, pos=pos)

    def old():
        ops.im2col_patches(px, patches[:, :K] if Kp == K else patches, p)
        ops.gemm(patches, w, pe)
        ops.vit_embed(pe, prefix[0], pos, out2, B, G2, N)

    res = {}
    for fn_name, fn in (("fused", fused), ("im2col+gemm", old)):
        try:
            fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                fn()
            e1.record()
            torch.cuda.synchronize()
            res[fn_name] = e0.elapsed_time(e1) / 20 * 1e3
        except Exception as ex:  # noqa: BLE001
            res[fn_name] = f"n/a ({type(ex).__name__}: {str(ex)[:80]})"
    tf = 2.0 * B * G2 * K * N / (res["fused"] * 1e-6) / 1e12
    print(f"{name}: B {B} M {B * G2} N {N} K {K}: fused {res['fused']:.1f} us ({tf:.0f} TF/s), "
          f"im2col+gemm+embed {res['im2col+gemm']}", flush=True)
