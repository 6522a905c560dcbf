"""Are cross-lane (ds_bpermute) sums corrupted by co-scheduled kernels? Diagnostic (tools/microbench/bperm_probe.hip).

Victim: bperm_victim sums 32 exact small integers per half-wave with the __shfl_xor butterfly (ds_bpermute_b32; mode 0)
or with DPP + v_permlane16_swap (mode 1), many rounds, and counts wrong totals. It runs alone, then beside each
aggressor queued on a second stream: the K-outer weight-gradient GEMM (trans_ab: LDS-DMA + ds_read_b64_tr_b16), the
row-major tile GEMM (LDS-DMA + ds_read_b128, in-launch split-K), the 256 x 256 kernel, a plain torch copy.
"""
import ctypes as C
import os
import sys
import time

sys.path[:0] = ["/root/repo", "/root/repo/gpt2-image-captioning_amd"]
import torch  # noqa: E402

from icap import ops  # noqa: E402

dev = torch.device("cuda", 0)
lib = C.CDLL(os.path.join(os.path.dirname(__file__), "..", "microbench", "libbperm_probe.so"))
lib.bperm_launch.argtypes = [C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]
ROUNDS = int(os.environ.get("PROBE_ROUNDS", "20000"))
BLOCKS = 4096
g = torch.Generator().manual_seed(0)
bf = lambda *s: (torch.randn(s, generator=g) * 0.05).to(dev, torch.bfloat16)  # noqa: E731
# the mapper's dW shape (3200 token rows; out 3072 x 768) and its dX product (3200 x 768 x 3072, in-launch split-K)
dY, X, W1 = bf(3200, 3072), bf(3200, 768), bf(768, 3072)
dW = torch.empty((3072, 768), device=dev, dtype=torch.float32)
dA = torch.empty((3200, 768), device=dev, dtype=torch.bfloat16)
big = bf(4096, 4096)
bigc = torch.empty_like(big)
cp_src = torch.randn(64 << 20, device=dev)
cp_dst = torch.empty_like(cp_src)
side = torch.cuda.Stream(dev)
ops.register_side_stream(side)
ops.gemm(dY, W1, dA)  # first-use initialisation of the default workspace
torch.cuda.synchronize()

aggressors = {
    "none": lambda: None,
    "kout_dW": lambda: ops.gemm(dY, X, dW, M=3072, N=768, K=3200, trans_ab=True),
    "tile_dX": lambda: ops.gemm(dY, W1, dA),
    "g256": lambda: ops.gemm(big, big, bigc),
    "copy": lambda: cp_dst.copy_(cp_src),
}


def run(mode, name, reps):
    errs = torch.zeros(2, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    with torch.cuda.stream(side):
        for _ in range(reps):
            aggressors[name]()
    t0 = time.time()
    rc = lib.bperm_launch(BLOCKS, ROUNDS, mode, errs.data_ptr(), errs[1:].data_ptr(),
                          torch.cuda.current_stream().cuda_stream)
    assert rc == 0
    torch.cuda.synchronize()
    e = errs.cpu().tolist()
    print(f"mode {mode} ({'bpermute' if mode == 0 else 'dpp+permlane16_swap'}) beside {name:8s} x{reps}: "
          f"wrong sums {e[0]} (first thread {e[1] - 1 if e[1] else None}) [{time.time() - t0:.3f} s]", flush=True)
    return e[0]


# victim alone, timed, to size the aggressor queues
run(0, "none", 1)
for mode in (0, 1):
    for name in ("kout_dW", "tile_dX", "g256", "copy"):
        run(mode, name, 60 if name != "g256" else 20)
