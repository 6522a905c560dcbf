"""Benchmark of the hot path on MI355X (contract: README / DESIGN.md "Measurement").

Workload (BASELINE.json configs[1]): one training step of GPT-2 small (frozen) + CLIP ViT-B/32 image tower
(frozen, forward on synthetic 224x224 pixels) + transformer mapping network (trained), bf16 storage / fp32
accumulation, dropout 0.1 as in the reference's train mode, teacher-forced CE over 50-token COCO-shaped captions,
clip_grad_norm(1.0) + AdamW + linear LR schedule; B=128 images per GPU (config.yml training.batch_size).
Weights are the deterministic random init of that architecture (no checkpoints offline); data are synthetic.

value = training images/s over all ranks. Also reported: greedy captions/s (50-token KV-cached decode,
B=128 per GPU = config.yml validation.batch_size), the GEMM roofline (per-launch HIP-event timing of every MFMA
GEMM of one step; algorithmic FLOPs), and the CPU baseline (oracle restatement of the reference step on a bounded
sample, rank 0 only).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
    N>1: python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpt2-image-captioning_amd")]

import torch  # noqa: E402

METRIC = "training images/sec + greedy captions/sec, GPT2-small+CLIP-B/32 at 1/2/4/8 GPU"
BF16_PEAK_TFLOPS = 2500.0  # MI355X dense bf16 MFMA (MI355X_MICROARCH.md chip table)
FP8_PEAK_TFLOPS = 5000.0  # dense MX fp8 (block-scaled 16x16x128 f8f6f4: 2x bf16 per clock, same table)
HBM_PEAK_GBS = 8000.0


_SLEEP_PER_MS = None


def prequeue(ms: float) -> None:
    """Queue a spin kernel (torch.cuda._sleep) of about `ms` milliseconds on the current stream (its rate is
    calibrated once with HIP events)."""
    global _SLEEP_PER_MS
    if _SLEEP_PER_MS is None:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        torch.cuda._sleep(1 << 20)
        e1.record()
        torch.cuda.synchronize()
        _SLEEP_PER_MS = (1 << 20) / max(e0.elapsed_time(e1), 1e-3)
    torch.cuda._sleep(max(1, int(_SLEEP_PER_MS * ms)))


class GemmTimer:
    """HIP-event timing of each GEMM launch on the launching stream (icap.ops.GEMM_TIMER hook)."""

    def __init__(self):
        self.rec = []

    def launch(self, key, flops, fn):
        from icap import ops

        s = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        fn()
        e1.record(s)
        self.rec.append((key, flops, e0, e1, ops.TIMER_TAG))

    def tagged(self, tag):
        """(launches, algorithmic FLOPs, ms) of the launches recorded under ops.timer_tag(tag) (GEMMs + attention)."""
        torch.cuda.synchronize()
        n, fl, ms = 0, 0.0, 0.0
        for _, f, e0, e1, t in self.rec:
            if t == tag:
                n, fl, ms = n + 1, fl + f, ms + e0.elapsed_time(e1)
        return n, fl, ms

    def summary(self, detail_path=None):
        """Aggregate per kernel instantiation (what rocprof reports per kernel name); optional per-shape dump."""
        torch.cuda.synchronize()
        agg, shapes = {}, {}
        for (kind, desc), fl, e0, e1, tag in self.rec:
            if kind.startswith("attn"):  # attention launches: only in the tagged (GPT-2 block) aggregate
                continue
            ms = e0.elapsed_time(e1)
            for d, k in ((agg, kind), (shapes, (kind, desc))):
                a = d.setdefault(k, [0, 0.0, 0.0])
                a[0] += 1
                a[1] += fl
                a[2] += ms
        if detail_path:
            for (kind, desc), fl, e0, e1, tag in self.rec:
                if kind.startswith("attn"):
                    a = shapes.setdefault((kind, desc), [0, 0.0, 0.0])
                    a[0] += 1
                    a[1] += fl
                    a[2] += e0.elapsed_time(e1)
            with open(detail_path, "w") as f:
                for (kind, desc), (n, fl, ms) in sorted(shapes.items(), key=lambda kv: -kv[1][2]):
                    f.write(f"{kind:10s} {desc:60s} n={n:3d} total_ms={ms:8.3f} avg_us={ms / n * 1e3:9.1f} "
                            f"TF/s={fl / (ms * 1e-3) / 1e12:8.1f}\n")
        return agg


def live_rows(labels, P, squares=False):
    """Host copy of the packed token-row count icap_caption_pack computes on the device (roofline pricing and the
    GEMM kernel choice): per caption max(P, P + last caption index with a target); squares: sum of their squares."""
    from icap.engine import live_rows as lr

    return lr(labels, P, squares=squares)


def build(B, dev, dropout=True, config="small", dtype=torch.bfloat16, fp8=False, pack=True):
    """config "small": BASELINE configs[1] (GPT-2 small + CLIP ViT-B/32); "medium": configs[3] (GPT-2 medium +
    CLIP ViT-L/14 encoder on the device, mapper at gpt_dim 1024 / CLIP-L embed 768)."""
    from types import SimpleNamespace

    from icap import CaptionTrainer, GPT2LMHeadModel, ImageCaptioningModel, TransformerMappingNetwork
    from icap.clip import CLIPVisionConfig, CLIPVisionTower
    from icap.gpt2 import GPT2Config

    if config == "large":  # configs[4]: DINOv3 ViT-L/16 (1024-d) -> mapper at gpt_dim 1280 -> GPT-2 large
        from icap.dino import DINOv3ImageTower

        gpt = GPT2LMHeadModel.random_init(GPT2Config.large(), seed=0)
        mapper = TransformerMappingNetwork.random_init(embed_dim=1024, gpt_dim=1280, seed=0)
        model = ImageCaptioningModel(mapper, tokenizer=SimpleNamespace(eos_token_id=50256), gpt=gpt,
                                     compute_dtype=dtype, gpt_fp8=fp8).to(dev)
        tower = DINOv3ImageTower.random_init(seed=0).to(dev)
        trainer = CaptionTrainer(model, B, 50, lr=1e-4, num_training_steps=10 ** 6, clip_model=tower,
                                 dropout=dropout, seed=1234, pack_rows=pack)
        return model, tower, trainer
    if config == "medium":
        gpt = GPT2LMHeadModel.random_init(GPT2Config.medium(), seed=0)
        mapper = TransformerMappingNetwork.random_init(embed_dim=768, gpt_dim=1024, seed=0)
        tower_cfg = CLIPVisionConfig.vit_l14()
    else:
        gpt = GPT2LMHeadModel.random_init(seed=0)
        mapper = TransformerMappingNetwork.random_init(seed=0)
        tower_cfg = None
    model = ImageCaptioningModel(mapper, tokenizer=SimpleNamespace(eos_token_id=50256), gpt=gpt,
                                 compute_dtype=dtype, gpt_fp8=fp8).to(dev)
    tower = CLIPVisionTower.random_init(tower_cfg, seed=0).to(dev)
    trainer = CaptionTrainer(model, B, 50, lr=1e-4, num_training_steps=10 ** 6, clip_model=tower, dropout=dropout,
                             seed=1234, pack_rows=pack)
    return model, tower, trainer


def parity_mode_rate(B, dev, steps=5):
    """The same train step in the fp32 parity mode (every GEMM an exact-fp32 MFMA chain, fp32 activations: the
    mode the reference goldens are matched in to 1e-5), images/s over `steps` graph-replayed steps."""
    model, tower, trainer = build(B, dev, dtype=torch.float32)
    ids, mask, labels, px = synthetic_batch(B, 1, dev)
    trainer.load_batch(ids, mask, labels, pixels=px)
    for _ in range(2):
        trainer.micro_step(use_graph=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        trainer.micro_step(use_graph=True)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    del model, tower, trainer
    torch.cuda.empty_cache()
    return {"images_per_s": round(B * steps / el, 2), "ms_per_step": round(el / steps * 1e3, 3), "steps": steps,
            "dtype": "fp32 (parity mode: 16x16x4 f32 MFMA)"}


def synthetic_batch(B, seed, dev):
    g = torch.Generator().manual_seed(seed)
    ids = torch.randint(0, 50256, (B, 50), generator=g)
    mask = torch.zeros((B, 50), dtype=torch.int64)
    ids[:, 13:] = 50256
    mask[:, :14] = 1
    labels = ids.clone()
    labels[mask == 0] = -100
    px = torch.randn((B, 3, 224, 224), generator=g)
    # ids / mask / labels stay on the host, pinned, as icap.train's DataLoader (pin_memory=True) delivers them: the
    # trainer reads each batch's packing flags from host labels (no device sync) and copies them asynchronously
    if torch.device(dev).type == "cuda":
        ids, mask, labels = ids.pin_memory(), mask.pin_memory(), labels.pin_memory()
    return ids, mask, labels, px.to(dev)


def cpu_baseline(seconds_budget: float = 20.0):
    """Oracle (torch-CPU restatement of src/train.py's step incl. CLIP fwd, dropout on) on a bounded sample."""
    from oracle import icap_oracle as O

    cores = min(len(os.sched_getaffinity(0)), 16)
    torch.set_num_threads(cores)
    B = 8
    gsd, msd = O.gpt2_state_dict(O.GPT2Cfg(), 0), O.mapper_state_dict(O.MapperCfg(), 0)
    csd = O.clip_vision_state_dict(O.ClipCfg(), 0)
    ids, mask, labels, _ = O.synthetic_batch(B, 50, 13, seed=1)
    px = torch.randn((B, 3, 224, 224), generator=torch.Generator().manual_seed(2))
    batch = (ids, mask, labels, px)
    O.train_steps(gsd, O.GPT2Cfg(), msd, O.MapperCfg(), [batch], total_steps=100, p_drop=0.1,
                  clip=(csd, O.ClipCfg()))  # warm-up
    n, t0 = 0, time.perf_counter()
    while True:
        O.train_steps(gsd, O.GPT2Cfg(), msd, O.MapperCfg(), [batch], total_steps=100, p_drop=0.1,
                      clip=(csd, O.ClipCfg()))
        n += 1
        el = time.perf_counter() - t0
        if el > seconds_budget or n >= 20:
            break
    res = {"value": round(n * B / el, 3), "unit": "images/s", "cores": cores, "kind": "port",
           "sample": f"{n} oracle train steps x batch {B} (CLIP-B/32 fwd on 224^2 pixels + mapper + GPT-2 small "
                     f"fwd/bwd + AdamW, dropout 0.1, fp32, torch CPU {cores} threads) in {el:.1f}s"}
    res["more"] = cpu_baseline_more(gsd, msd, csd, cores)
    return res


def cpu_baseline_more(gsd, msd, csd, cores):
    """The other CPU rows of BASELINE.md §3 on bounded samples: the headline batch (128) frozen, GPT-2 unfrozen
    (batch 8), and greedy captions/s of the reference's decode loop (full recompute each token, no KV cache:
    src/models.py:389-469) over 50 fixed steps."""
    from oracle import icap_oracle as O

    out = {}
    ids, mask, labels, _ = O.synthetic_batch(128, 50, 13, seed=1)
    px = torch.randn((128, 3, 224, 224), generator=torch.Generator().manual_seed(2))
    t0 = time.perf_counter()
    O.train_steps(gsd, O.GPT2Cfg(), msd, O.MapperCfg(), [(ids, mask, labels, px)], total_steps=100, p_drop=0.1,
                  clip=(csd, O.ClipCfg()))
    el = time.perf_counter() - t0
    out["train_b128_frozen"] = {"value": round(128 / el, 3), "unit": "images/s",
                                "sample": f"1 oracle train step x batch 128 (as the headline, incl. CLIP fwd) in {el:.1f}s"}
    ids, mask, labels, _ = O.synthetic_batch(8, 50, 13, seed=1)
    emb = torch.randn((8, 512), generator=torch.Generator().manual_seed(3))
    b8 = (ids, mask, labels, emb / emb.norm(dim=-1, keepdim=True))
    O.train_steps(gsd, O.GPT2Cfg(), msd, O.MapperCfg(), [b8], total_steps=100, p_drop=0.1, freeze_gpt=False)
    t0 = time.perf_counter()
    O.train_steps(gsd, O.GPT2Cfg(), msd, O.MapperCfg(), [b8, b8], total_steps=100, p_drop=0.1, freeze_gpt=False)
    el = time.perf_counter() - t0
    out["train_b8_unfrozen"] = {"value": round(16 / el, 3), "unit": "images/s",
                                "sample": f"2 oracle train steps x batch 8, GPT-2 unfrozen (AdamW over 124M+ params), "
                                          f"precomputed embeddings, in {el:.1f}s"}
    Bg = 4
    emb = torch.randn((Bg, 512), generator=torch.Generator().manual_seed(5))
    with torch.no_grad():
        cur = O.mapper_forward(msd, O.MapperCfg(), emb / emb.norm(dim=-1, keepdim=True))
        t0 = time.perf_counter()
        for _ in range(50):  # the reference loop, all 50 steps (no early exit: the GPU figure decodes 50 too)
            _, logits = O.gpt2_forward(gsd, O.GPT2Cfg(), cur)
            nxt = torch.argmax(logits[:, -1, :], dim=-1)
            cur = torch.cat((cur, gsd["transformer.wte.weight"][nxt].unsqueeze(1)), dim=1)
        el = time.perf_counter() - t0
    out["greedy"] = {"value": round(Bg / el, 3), "unit": "captions/s",
                     "sample": f"{Bg} captions x 50 greedy tokens, full recompute per token (the reference's loop, "
                               f"no KV cache), fp32, {cores} threads, in {el:.1f}s"}
    return out


def greedy_rate(model, Bd, dev, world, edim=512):
    """50-token KV-cached greedy captions/s over a batch of Bd image embeddings (all 50 steps decoded)."""
    g = torch.Generator().manual_seed(5)
    emb = torch.randn((Bd, edim), generator=g)
    emb = (emb / emb.norm(dim=-1, keepdim=True)).to(dev)
    # one caption = 50 greedy tokens after the 15-token prefix: decode all 50 steps (the trained
    # synthetic model emits EOS early; the reference loop would stop there), output identical either way
    model.generate(emb, max_length=50, temperature=0.0, early_exit=False)  # warm-up
    torch.cuda.synchronize()
    td0 = time.perf_counter()
    nd = 3
    lens = []
    for _ in range(nd):
        out = model.generate(emb, max_length=50, temperature=0.0, early_exit=False)
        lens.append(out.shape[1])
    torch.cuda.synchronize()
    dt = time.perf_counter() - td0
    caps_per_s = world * Bd * nd / dt

    return caps_per_s, dt, nd, lens


def beam_rate(model, Bd, dev, world, edim=512, num_beams=4):
    """50-token KV-cached beam-4 captions/s (BASELINE configs[4] decode; transformers' beam search semantics,
    tests/test_beam.py): Bd images x num_beams hypotheses decoded on the device, all 50 steps."""
    g = torch.Generator().manual_seed(7)
    emb = torch.randn((Bd, edim), generator=g)
    emb = (emb / emb.norm(dim=-1, keepdim=True)).to(dev)
    # all 50 steps (random-init weights finish captions early; finished ones stay frozen): fixed work per caption
    model.generate(emb, max_length=50, temperature=0.0, num_beams=num_beams, early_exit=False)  # warm-up + capture
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    nd, lens = 2, []
    for _ in range(nd):
        lens.append(model.generate(emb, max_length=50, temperature=0.0, num_beams=num_beams, early_exit=False).shape[1])
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return {"captions_per_s": round(world * Bd * nd / dt, 1), "batch_per_gpu": Bd, "num_beams": num_beams,
            "decode_steps": 50, "returned_len": lens[-1], "ms_per_batch": round(dt / nd * 1e3, 3)}


def topp_rate(model, Bd, dev, world, edim=512, temperature=1.0, top_p=0.9):
    """50-token KV-cached nucleus-sampled captions/s (src/models.py:400-449 branch: HIP top-p filter + draw per
    step). The decode runs as HIP-graph chunks of 8 tokens and the host reads the EOS latch once per chunk (the
    reference checks it every step; the returned ids are truncated to the reference loop's length either way).
    Random-init weights rarely emit EOS, so every caption runs all 50 steps."""
    g = torch.Generator().manual_seed(6)
    emb = torch.randn((Bd, edim), generator=g)
    emb = (emb / emb.norm(dim=-1, keepdim=True)).to(dev)
    model.generate(emb, max_length=50, temperature=temperature, top_p=top_p)  # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    nd, lens = 2, []
    for _ in range(nd):
        lens.append(model.generate(emb, max_length=50, temperature=temperature, top_p=top_p).shape[1])
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return {"captions_per_s": round(world * Bd * nd / dt, 1), "batch_per_gpu": Bd, "temperature": temperature,
            "top_p": top_p, "returned_len": lens[-1], "ms_per_batch": round(dt / nd * 1e3, 3)}


def preprocess_rate(dev):
    """CLIP image preprocessing: device (icap_clip_preprocess, Pillow-exact) vs the host
    PIL processor on the same decoded 480x640 RGB images; images/s (JPEG decode excluded on both sides)."""
    import numpy as np

    from icap import ops
    from icap.clip import CLIPProcessor

    rng = np.random.default_rng(3)
    ims = [rng.integers(0, 256, (480, 640, 3), dtype=np.uint8) for _ in range(32)]
    nd = 256
    batch = [ims[i % len(ims)] for i in range(nd)]
    ops.clip_preprocess(batch[:8], dev)  # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        ops.clip_preprocess(batch, dev)
    torch.cuda.synchronize()
    dev_rate = 3 * nd / (time.perf_counter() - t0)
    from PIL import Image

    pil = [Image.fromarray(a) for a in ims[:16]]
    proc = CLIPProcessor()
    t0 = time.perf_counter()
    proc(pil)
    host_rate = len(pil) / (time.perf_counter() - t0)
    return {"device_images_per_s": round(dev_rate, 1), "host_pil_images_per_s": round(host_rate, 1),
            "image": "480x640 RGB uint8 -> 3x224x224 fp32 (shortest-edge bicubic, centre crop, normalise)",
            "device_includes": "host packing + H2D copy of the uint8 pixels + 2 kernels"}


def extraction_rate(tower, dev, n_images: int = 512):
    """End-to-end CLIP embedding extraction (src/embeddings/clip.py:79-149 -> icap.clip.extract_clip_embeddings):
    a directory of 640x480 JPEGs -> .pt file, incl. JPEG decode in DataLoader workers, device preprocessing, the
    ViT-B/32 tower (bf16) and the torch.save. The reference's only published figure is this loop at batch 64 with
    4 workers: 65 images/s (notebooks/extract_clip_embeddings.ipynb:167,174)."""
    import shutil
    import tempfile

    import numpy as np
    from PIL import Image

    from icap.clip import DeviceCLIPProcessor
    from icap.images import extract_directory

    d = tempfile.mkdtemp(prefix="icap_extract_")
    try:
        rng = np.random.default_rng(7)
        yy, xx = np.mgrid[0:480, 0:640]
        for i in range(n_images):  # smooth colour fields + noise: JPEG sizes like photos (~60-90 KB)
            base = np.stack([(xx * (1 + i % 5) + yy * (i % 3)) % 256, (yy * 2 + i * 7) % 256,
                             (xx + yy + i * 13) % 256], -1).astype(np.int16)
            img = np.clip(base + rng.integers(-40, 40, base.shape), 0, 255).astype(np.uint8)
            Image.fromarray(img).save(os.path.join(d, f"COCO_val2014_{i:012d}.jpg"), quality=90)
        proc = DeviceCLIPProcessor(device=dev)
        out = os.path.join(d, "emb.pt")
        res, split = {}, {}
        dim = tower.config.projection_dim
        for workers in (4, 8, 16):
            extract_directory(d, out, tower.embed, proc, dim, 64, workers, dev)  # warm-up (page cache, kernels)
            torch.cuda.synchronize()
            st = {}
            t0 = time.perf_counter()
            extract_directory(d, out, tower.embed, proc, dim, 64, workers, dev, stats=st)
            torch.cuda.synchronize()
            res[f"images_per_s_{workers}_workers"] = round(n_images / (time.perf_counter() - t0), 1)
            split[f"{workers}_workers"] = st
        # where the main process's time goes (s): worker start-up + first batch, waiting on the loader, issuing
        # the device work, the final copy + save (icap.images.extract_directory stats)
        res["main_process_split_s"] = split
        res.update({"images": n_images, "image": "640x480 JPEG q90", "batch": 64,
                    "reference_published_images_per_s": 65.0,
                    "includes": "JPEG decode (PIL, DataLoader workers) + device preprocess + CLIP-B/32 bf16 + .pt save"})
        return res
    finally:
        shutil.rmtree(d, ignore_errors=True)


def extraction_child():
    """extraction_rate in a child process of its own (tools/extract_bench.py): DataLoader workers forked from this
    bench process (GBs of host state) start slowly enough to dominate a 1024-image sample."""
    import subprocess

    env = dict(os.environ, N="1024")
    try:
        out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "extract_bench.py")], env=env,
                             capture_output=True, text=True, timeout=300)
        lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
        return json.loads(lines[-1]) if lines else {"error": out.stderr[-300:]}
    except (subprocess.TimeoutExpired, ValueError) as e:
        return {"error": str(e)[:300]}


def pmc_traffic(kernel: str):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary (tools/pmc_traffic.sh writes
    profiles/*pmc_traffic.json from separate FETCH_SIZE / WRITE_SIZE passes over this bench's train step).
    FETCH_SIZE is doubled (gfx950 tallies 128-B wide reads at 64 B: MI355X_MICROARCH.md, HBM)."""
    import glob

    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc_traffic.json"))):
        try:
            with open(f) as fh:
                d = json.load(fh)
        except (OSError, ValueError):
            continue
        k = d.get("kernels", {}).get(kernel)
        if k:
            best = (k["hbm_bytes_per_launch"], os.path.relpath(f, ROOT))
    return best if best else (None, None)


def launch_ranks(n: int, argv) -> int:
    """`python bench.py --gpus N` without a torchrun environment: start N data-parallel ranks (one process per GPU)
    through torch.distributed.run on 127.0.0.1 and return their exit status. This parent makes no GPU call (it
    only spawns and waits), so the ranks own the devices; rank 0 prints the one JSON line."""
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this host driver (RCCL peer setup)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *argv]
    return subprocess.call(cmd, env=env)


def launcher_probe():
    """--launcher-probe: what each rank sees (CPU / gloo only, no GPU): one JSON line from rank 0 listing every
    rank's (RANK, LOCAL_RANK, WORLD_SIZE). Lets the CPU test suite check the --gpus N launcher."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    me = torch.tensor([rank, local, world], dtype=torch.int64)
    seen = [me]
    if world > 1:
        torch.distributed.init_process_group("gloo")
        seen = [torch.zeros_like(me) for _ in range(world)]
        torch.distributed.all_gather(seen, me)
    if rank == 0:
        print(json.dumps({"n_gpus": world, "ranks": [s.tolist() for s in seen]}), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


def kernel_peak(name: str) -> float:
    return FP8_PEAK_TFLOPS if "fp8_t" in name else BF16_PEAK_TFLOPS


def replay_roofline(trainer, dom, reps=20):
    """Kernel time inside the replayed step graph, by difference: the step is captured twice
    more, once with every launch of the dominant instantiation left out and once with every GEMM / attention launch
    of the GPT-2-block region left out (ops.GEMM_TIMER hook: the launch function is simply not called), and each of
    the three graphs is replayed `reps` times back to back between HIP events on the capture stream. The full
    graph's median replay minus a reduced graph's is the time those launches occupy in the step as it is timed
    (kernel durations plus their share of dispatch gaps; the work on one stream runs in series, so nothing they
    overlap is lost). Kernel times do not depend on the values the skipped launches would have written. ROCm graphs
    refuse timing-event nodes ("External events are disallowed"), and the profiler's kernel records of a graph
    replay were incomplete here, hence the difference."""
    from icap import ops

    class _Skip:
        def __init__(self, pred):
            self.pred, self.n = pred, 0

        def launch(self, key, flops, fn):
            if self.pred(key, ops.TIMER_TAG):
                self.n += 1
            else:
                fn()

    def capture(timer):
        torch.cuda.synchronize()
        ops.GEMM_TIMER = timer
        try:
            g = torch.cuda.CUDAGraph()
            with ops.graph_capture(g):  # forward + backward only: no optimizer step, the parameters stay as they are
                trainer._fwd_bwd(True, trainer.grad_scale())
        finally:
            ops.GEMM_TIMER = None
        return g

    def median_replay(g):
        g.replay()
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
        ev[0].record()
        for k in range(reps):
            g.replay()
            ev[k + 1].record()
        torch.cuda.synchronize()
        t = sorted(ev[k].elapsed_time(ev[k + 1]) for k in range(reps))
        return t[reps // 2]

    try:
        skip_dom = _Skip(lambda key, tag: key[0] == dom)
        skip_blk = _Skip(lambda key, tag: tag == "gpt2_block")
        graphs = {"full": capture(_Skip(lambda key, tag: False)), "no_dom": capture(skip_dom),
                  "no_block": capture(skip_blk)}
        ms = {k: median_replay(g) for k, g in graphs.items()}
        del graphs
    except Exception as e:  # noqa: BLE001 (reported in the bench line, the eager figure stands)
        ops.GEMM_TIMER = None
        torch.cuda.synchronize()
        return {"error": f"{type(e).__name__}: {e}"[:200]}
    return {"dom_launches": skip_dom.n, "dom_ms": ms["full"] - ms["no_dom"], "block_launches": skip_blk.n,
            "block_ms": ms["full"] - ms["no_block"], "replay_ms": ms, "reps": reps,
            "timing": "median graph replay, full minus the graph without those launches"}


def train_rate(trainer, B, steps, warmup, use_graph, world, dev, detail=False):
    """images/s over `steps` graph-replayed steps after `warmup` (barrier + synchronize on both sides, max over
    ranks), the per-step median (HIP events between the steps on the launch stream), and the GEMM roofline of one
    eager step (HIP events around every GEMM / GPT-2-block attention launch)."""
    from icap import ops

    dist = world > 1
    for _ in range(max(warmup, 1)):
        trainer.micro_step(use_graph=use_graph)
    torch.cuda.synchronize()
    if dist:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
    t0 = time.perf_counter()
    evs[0].record()
    for i in range(steps):
        trainer.micro_step(use_graph=use_graph)
        evs[i + 1].record()
    torch.cuda.synchronize()
    if dist:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    per_step = sorted(evs[i].elapsed_time(evs[i + 1]) for i in range(steps))
    median_ms = per_step[len(per_step) // 2] if steps % 2 else 0.5 * (per_step[steps // 2 - 1] + per_step[steps // 2])
    rank_ms = [el / steps * 1e3]
    if dist:
        mine = torch.tensor([el / steps * 1e3], device=dev, dtype=torch.float64)
        allr = [torch.zeros_like(mine) for _ in range(world)]
        torch.distributed.all_gather(allr, mine)
        rank_ms = [float(x.item()) for x in allr]
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        el = float(t.item())
    loss = float(trainer.last_loss.item())
    timer = GemmTimer()
    ops.GEMM_TIMER = timer
    torch.cuda.synchronize()
    te0 = time.perf_counter()
    segs = trainer._segments(True, trainer.grad_scale())
    sev = [torch.cuda.Event(enable_timing=True) for _ in range(len(segs) + 2)]
    # a spin kernel queued first keeps the device behind the host for the whole eager pass, so no host launch gap
    # enters the per-launch HIP events (the markers themselves remain: profiles/r04_bench_12836_prequeue.json)
    prequeue(80.0)
    sev[0].record()
    for i, (rng, fn) in enumerate(segs):  # the data-parallel buckets' segments, timed (eager, with GEMM events)
        fn()
        sev[i + 1].record()
    trainer._optimizer()
    sev[-1].record()
    torch.cuda.synchronize()
    host_ms = (time.perf_counter() - te0) * 1e3
    eager_ms = sev[0].elapsed_time(sev[-1])  # device time of the eager step (kernels back to back)
    seg_ms = [round(sev[i].elapsed_time(sev[i + 1]), 3) for i in range(len(segs))]
    seg_bytes = [sum(hi - lo for lo, hi in rng) * 4 for rng, _ in segs]
    ops.GEMM_TIMER = None
    agg = timer.summary(os.environ.get("ICAP_GEMM_DETAIL") if detail else None)  # the headline step's shapes only
    dom = max(agg, key=lambda k: agg[k][2])
    n_l, fl, ms = agg[dom]
    achieved = fl / (ms * 1e-3) / 1e12
    bn, bfl, bms = timer.tagged("gpt2_block")
    rep = replay_roofline(trainer, dom) if use_graph else None
    eager = {"dom_ms": ms, "achieved": achieved, "frac": achieved / kernel_peak(dom),
             "block_ms": bms, "block_frac": bfl / (bms * 1e-3) / 1e12 / BF16_PEAK_TFLOPS if bms else None}
    if rep and "dom_ms" in rep and rep["dom_ms"] > 0 and rep["dom_launches"] == n_l:
        # the graph-replay durations (the step as it is timed) are the reported ones
        ms = rep["dom_ms"]
        achieved = fl / (ms * 1e-3) / 1e12
        if rep["block_ms"] > 0 and rep["block_launches"] == bn:
            bms = rep["block_ms"]
    return {"el": el, "loss": loss, "images_per_s": world * B * steps / el, "ms_per_step": el / steps * 1e3,
            "eager_roofline": eager, "replay_roofline": rep,
            "median_ms": median_ms, "rank_ms": rank_ms, "seg_ms": seg_ms, "seg_bytes": seg_bytes,
            "dom": dom, "n_l": n_l, "fl": fl, "ms": ms, "achieved": achieved,
            "frac": achieved / kernel_peak(dom), "gemm_ms": sum(v[2] for v in agg.values()),
            "all_fl": sum(v[1] for v in agg.values()), "eager_ms": eager_ms, "eager_host_ms": host_ms,
            "block": {"launches": bn, "alg_tflop": round(bfl / 1e12, 4), "ms": round(bms, 3),
                      "achieved": round(bfl / (bms * 1e-3) / 1e12, 1) if bms else None,
                      "frac": round(bfl / (bms * 1e-3) / 1e12 / BF16_PEAK_TFLOPS, 4) if bms else None}}


def padded_rate(config, B, dev, world, fp8=False, steps=10):
    """The same step with the packed token rows off (ICAP_PACK=0: every block runs on all B x 65 rows of the padded
    grid, as the reference computes them): images/s and the dominant GEMM's roofline fraction, for comparison."""
    model, tower, tr = build(B, dev, config=config, fp8=fp8, pack=False)
    ids, mask, labels, px = synthetic_batch(B, 1, dev)
    tr.load_batch(ids, mask, labels, pixels=px)
    tr.gws.head_rows_hint = int((labels != -100).sum().item())
    r = train_rate(tr, B, steps, 3, True, world, dev)
    del model, tower, tr
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return {"images_per_s": round(r["images_per_s"], 1), "ms_per_step": round(r["ms_per_step"], 3),
            "token_rows_per_step": B * 65, "dominant_kernel": r["dom"], "dominant_frac": round(r["frac"], 4),
            "all_gemm_ms_per_step": round(r["gemm_ms"], 3)}


def batch_sweep(config, batches, dev, world, fp8=False):
    """SURVEY.md §8(d) perf batch sweep: the same train step at other per-GPU batches (weak-scaling B is a free
    choice; the reference's is config.yml:32 = 128; BASELINE.md §4 also names 8 and 32): images/s and the dominant
    GEMM's roofline fraction."""
    out = []
    for Bs in batches:
        model, tower, tr = build(Bs, dev, config=config, fp8=fp8)
        ids, mask, labels, px = synthetic_batch(Bs, 11, dev)
        tr.load_batch(ids, mask, labels, pixels=px)
        tr.gws.head_rows_hint = int((labels != -100).sum().item())
        r = train_rate(tr, Bs, 10 if Bs <= 32 else 5, 2, True, world, dev)
        out.append({"batch_per_gpu": Bs, "images_per_s": round(r["images_per_s"], 1),
                    "ms_per_step": round(r["ms_per_step"], 3), "ms_per_step_median": round(r["median_ms"], 3),
                    "dominant_kernel": r["dom"], "dominant_frac": round(r["frac"], 4),
                    "dominant_tflops": round(r["achieved"], 1), "all_gemm_ms_per_step": round(r["gemm_ms"], 3),
                    "gpt2_block_frac": r["block"]["frac"]})
        del model, tower, tr
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
    return out


def unfrozen_rate(B, dev, world, steps=10):
    """freeze_gpt_weights=False (src/models.py:216-217, config.yml:21-22): the same step with every GPT-2 tensor
    trained (dW products, LN / bias / tied-wte / wpe grads, AdamW over 185 M params, refreshed forward copies),
    graph-replayed: images/s beside the CPU baseline's train_b8_unfrozen row."""
    from types import SimpleNamespace

    from icap import CaptionTrainer, GPT2LMHeadModel, ImageCaptioningModel, TransformerMappingNetwork
    from icap.clip import CLIPVisionTower

    gpt = GPT2LMHeadModel.random_init(seed=0)
    mapper = TransformerMappingNetwork.random_init(seed=0)
    model = ImageCaptioningModel(mapper, tokenizer=SimpleNamespace(eos_token_id=50256), gpt=gpt,
                                 freeze_gpt_weights=False, compute_dtype=torch.bfloat16).to(dev)
    tower = CLIPVisionTower.random_init(None, seed=0).to(dev)
    tr = CaptionTrainer(model, B, 50, lr=1e-4, num_training_steps=10 ** 6, clip_model=tower, dropout=True,
                        seed=1234)
    ids, mask, labels, px = synthetic_batch(B, 1, dev)
    tr.load_batch(ids, mask, labels, pixels=px)
    r = train_rate(tr, B, steps, 3, True, world, dev)
    res = {"images_per_s": round(r["images_per_s"], 1), "ms_per_step": round(r["ms_per_step"], 3),
           "ms_per_step_median": round(r["median_ms"], 3), "batch_per_gpu": B,
           "trained_params": int(tr.flat.n), "final_loss": round(r["loss"], 4),
           "dominant_kernel": r["dom"], "dominant_frac": round(r["frac"], 4),
           "all_gemm_ms_per_step": round(r["gemm_ms"], 3),
           "workload": "as the headline (CLIP-B/32 fwd on pixels, dropout 0.1) with GPT-2 small trained: + every "
                       "block's dW, LN / bias grads, tied-wte and wpe grads, AdamW over all of them; padded token "
                       "rows and the full LM head (the tied wte gradient reads every row)"}
    del model, tower, tr
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return res


EDIM = {"small": 512, "medium": 768, "large": 1024}  # image-embedding width per config (CLIP-B/32, CLIP-L/14, DINOv3-L)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--launcher-probe", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--decode-batch", type=int, default=128)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-decode", action="store_true", help="skip the greedy-decode measurement (PMC passes)")
    ap.add_argument("--config", default="small", choices=["small", "medium", "large"],
                    help="small = BASELINE configs[1] (default, the headline); medium = configs[3]; "
                         "large = configs[4] (DINOv3 ViT-L/16 + GPT-2 large, beam-4 decode)")
    ap.add_argument("--fp8", action="store_true",
                    help="configs[4]'s fp8 path: GPT-2's frozen products as MX block-scaled e4m3 GEMMs")
    ap.add_argument("--sweep", default=None,
                    help="comma-separated extra per-GPU batches for the batch sweep (default: 8,32,256,512 for small)")
    ap.add_argument("--no-unfrozen", action="store_true", help="skip the freeze_gpt_weights=False line")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if args.launcher_probe:
        return launcher_probe()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus != world:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1
    # ICAP_BENCH_DP_REHEARSAL=1 (checks only, never a reported line): every rank on cuda:0 over gloo, so the N > 1
    # path (launcher, buckets, max-over-ranks timing, the data_parallel fields) runs on a one-GPU box
    rehearsal = dist and os.environ.get("ICAP_BENCH_DP_REHEARSAL") == "1"
    if rehearsal:
        local = 0
    if dist:
        torch.cuda.set_device(local)
        if rehearsal:
            torch.distributed.init_process_group("gloo")
        else:
            torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    B = args.batch

    if args.fp8 and args.config != "large":
        raise SystemExit("bench.py: --fp8 is configs[4]'s path (--config large)")
    model, tower, trainer = build(B, dev, config=args.config, fp8=args.fp8)
    ids, mask, labels, px = synthetic_batch(B, 1 + rank, dev)  # each rank: its own shard of samples
    trainer.load_batch(ids, mask, labels, pixels=px)
    # LM-head target rows of this batch (the device holds the count; the host copy only prices the roofline)
    head_rows = int((labels != -100).sum().item())
    trainer.gws.head_rows_hint = head_rows
    packed = bool(trainer.gws.pack)
    token_rows = live_rows(labels, trainer.P) if packed else B * trainer.gws.S
    trainer.gws.live_rows_hint = token_rows if packed else None
    trainer.gws.seq_sq_hint = live_rows(labels, trainer.P, squares=True) if packed else None
    use_graph = not args.no_graph
    # timed region + the kernel roofline pass (every GEMM launch of one eager step, timed with HIP events)
    r = train_rate(trainer, B, args.steps, args.warmup, use_graph, world, dev, detail=True)
    el, loss, imgs_per_s = r["el"], r["loss"], r["images_per_s"]
    dom, n_l, fl, ms, achieved = r["dom"], r["n_l"], r["fl"], r["ms"], r["achieved"]
    gemm_ms, all_fl, eager_ms = r["gemm_ms"], r["all_fl"], r["eager_ms"]

    # -- greedy decode throughput ------------------------------------------------------------------------------
    Bd = args.decode_batch
    caps_per_s, dt, nd, lens = None, None, 1, [None]
    if not args.no_decode:
        caps_per_s, dt, nd, lens = greedy_rate(model, Bd, dev, world, EDIM[args.config])
    topp = None if args.no_decode or args.config == "large" else topp_rate(model, Bd, dev, world, EDIM[args.config])
    beam = beam_rate(model, Bd, dev, world, EDIM[args.config]) if (not args.no_decode and args.config == "large") \
        else None
    # the same decode at a serving batch (4 x the headline's): the per-token kernels are latency-bound at 128 rows
    big = None
    if not args.no_decode and args.config == "small":
        cb, dtb, ndb, lb = greedy_rate(model, 4 * Bd, dev, world)
        big = {"batch_per_gpu": 4 * Bd, "captions_per_s": round(cb, 1), "ms_per_batch": round(dtb / ndb * 1e3, 3)}
    # the committed PMC pass measured the configs[1] step: its per-launch bytes do not describe other configs
    traffic, traffic_src = pmc_traffic(dom) if args.config == "small" else (None, None)
    prep = None if args.no_decode else preprocess_rate(dev)
    extract = extraction_child() if (not args.no_decode and args.config == "small" and rank == 0) else None
    parity = parity_mode_rate(B, dev) if (not args.no_decode and args.config == "small" and world == 1) else None
    sweep_b = [int(x) for x in args.sweep.split(",") if x] if args.sweep is not None else \
        ([8, 32, 256, 512] if args.config == "small" and not args.no_decode and world == 1 else [])
    want_padded = packed and not args.no_decode and world == 1
    want_unfrozen = args.config == "small" and not args.no_decode and not args.no_unfrozen and world == 1
    # data-parallel bookkeeping (self-check of an N > 1 line: what torch.distributed saw and what went over RCCL)
    dp = None
    if dist:
        flat_n = int(trainer.flat.n)
        bpe = 2 if trainer.dp_bf16 else 4
        dp = {"world_size_seen": torch.distributed.get_world_size(), "backend": torch.distributed.get_backend(),
              "rank_ms_per_step": [round(x, 3) for x in r["rank_ms"]],
              "allreduce_bytes_per_step": flat_n * bpe, "allreduce_dtype": "bf16" if trainer.dp_bf16 else "fp32",
              "buckets": len(trainer._ranges_mapper) + 1 if trainer.dp_overlap else 1,
              "overlapped": bool(trainer.dp_overlap)}
        if rehearsal:
            dp["rehearsal"] = "all ranks on cuda:0 over gloo (path check, not a measurement)"
    if sweep_b or want_padded or want_unfrozen:
        del model, tower, trainer
        torch.cuda.empty_cache()
    padded = padded_rate(args.config, B, dev, world, args.fp8) if want_padded else None
    unfrozen = unfrozen_rate(B, dev, world) if want_unfrozen else None
    sweep = batch_sweep(args.config, sweep_b, dev, world, args.fp8) if sweep_b else None

    if rank == 0:
        res = {
            "metric": METRIC, "value": round(imgs_per_s, 2), "unit": "images/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 3),
            "ms_per_step_median": round(r["median_ms"], 3),
            "padded_images_per_s": padded["images_per_s"] if padded else None,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "fp8 (MX e4m3, GPT-2 products) + bf16" if args.fp8 else "bf16",
            "data": "synthetic (seeded COCO-shaped captions: 13 tokens + EOS, padded to 50; randn 224x224 pixels); "
                    "deterministic random-init weights",
            "packed_rows": ({"token_rows_per_step": token_rows, "padded_rows": B * 65,
                             "note": "GPT-2 blocks run on each caption's live rows (prefix + positions up to its last "
                                     "loss target, icap_caption_pack); the dead tail of the padded grid feeds no loss "
                                     "term under the causal mask (loss / gradients unchanged: tests/test_pack_gpu.py)",
                             "padded_step": padded} if packed else None),
            "config": {"workload": ("train step: CLIP ViT-B/32 fwd (frozen) on 224x224 pixels -> transformer mapper "
                                    "(8 layers, prefix 15, trained) -> GPT-2 small (frozen) fwd + dX bwd, LM head on "
                                    "the target rows + CE, dropout 0.1, clip_grad_norm 1.0 + AdamW + linear LR")
                       if args.config == "small" else
                       (f"BASELINE configs[4] train step ({'fp8: every frozen GPT-2 product (fwd, dX, LM head) as an MX block-scaled e4m3 GEMM, the rest bf16' if args.fp8 else 'bf16'}): "
                        "DINOv3 ViT-L/16 fwd "
                        "(frozen, 4 registers + RoPE, 201 tokens) on 224x224 pixels -> transformer mapper (8 layers, "
                        "gpt_dim 1280, trained) -> GPT-2 large (36 layers, d 1280, frozen) fwd + dX bwd, LM head on "
                        "the target rows + CE, dropout 0.1, clip 1.0 + AdamW; decode: beam-4")
                       if args.config == "large" else
                       ("BASELINE configs[3] train step: CLIP ViT-L/14 fwd (frozen, 257 tokens) on 224x224 pixels -> "
                        "transformer mapper (8 layers, gpt_dim 1024, trained) -> GPT-2 medium (24 layers, d 1024, "
                        "frozen) fwd + dX bwd, LM head on the target rows + CE, dropout 0.1, clip 1.0 + AdamW"),
                       "lm_head_rows_per_step": head_rows,
                       "per_gpu_batch": B, "global_batch": B * world, "seq_len": 65, "caption_len": 50,
                       "parallelism": f"dp{world}", "graph": use_graph},
            "final_loss": round(loss, 4),
            "greedy_captions_per_s": round(caps_per_s, 1) if caps_per_s else None,
            "greedy": {"batch_per_gpu": Bd, "decode_steps": 50, "returned_len": lens[-1], "kv_cache": True,
                       "ms_per_batch": round(dt / nd * 1e3, 3) if dt else None},
            "greedy_serving_batch": big,
            "topp_sampling": topp,
            "beam4": beam,
            "clip_preprocess": prep,
            "clip_extraction": extract,
            "fp32_parity_mode": parity,
            "train_unfrozen": unfrozen,
            "data_parallel": dp,
            "batch_sweep": sweep,
            "roofline": {"bound": "mfma", "kernel": dom, "achieved": round(achieved, 1),
                         "peak": kernel_peak(dom), "unit": "TFLOP/s", "frac": round(achieved / kernel_peak(dom), 4),
                         "traffic": traffic, "traffic_unit": "bytes/launch (HBM, rocprofv3 PMC: 2 x FETCH_SIZE + WRITE_SIZE)",
                         "traffic_source": traffic_src, "launches_per_step": n_l,
                         "avg_launch_us": round(ms / n_l * 1e3, 2),
                         "alg_gflop_per_launch": round(fl / n_l / 1e9, 3),
                         "all_gemm_ms_per_step": round(gemm_ms, 3), "all_gemm_tflop_per_step": round(all_fl / 1e12, 4),
                         "eager_step_ms": round(eager_ms, 3),
                         "eager_step_host_ms": round(r["eager_host_ms"], 3),
                         "dp_segments": {"ms": r["seg_ms"], "grad_bytes": r["seg_bytes"],
                                         "what": "eager step cut at the data-parallel buckets (forward + GPT-2 "
                                                 "backward, then one per mapper layer top first, then the mapper "
                                                 "input projection): HIP-event time and fp32 gradient bytes each "
                                                 "segment finalises (DESIGN.md §8(e) overlap arithmetic)"},
                         "gpt2_block": dict(r["block"], peak=BF16_PEAK_TFLOPS, unit="TFLOP/s",
                                            what="the 12 GPT-2 blocks' GEMMs (fwd + dX) and attention (fwd + bwd) of "
                                                 "one step: summed algorithmic FLOPs (live rows) / summed in-replay "
                                                 "kernel time (timing)"),
                         "timing": ("graph replay by difference: median replay of the step graph minus that of the "
                                    "same graph captured without the dominant instantiation's launches (and, for "
                                    "gpt2_block, without the block region's GEMM + attention launches), HIP events "
                                    "between replays (replay_roofline). The eager pass (HIP events around every "
                                    "launch, eager_roofline) picks the dominant kernel and prices the per-shape table"
                                    if r["replay_roofline"] and "dom_ms" in r["replay_roofline"] else
                                    "HIP events around every GEMM launch of one eager step on its launch stream (the "
                                    "replay pass was unavailable: replay_roofline)"),
                         "eager_roofline": {k: (round(v, 4) if isinstance(v, float) else v)
                                            for k, v in r["eager_roofline"].items()},
                         "replay_roofline": ({k: (round(v, 4) if isinstance(v, float) else v)
                                              for k, v in r["replay_roofline"].items()}
                                             if r["replay_roofline"] else None)},
        }
        if not args.no_cpu_baseline and world == 1 and args.config == "small":
            res["cpu_baseline"] = cpu_baseline()
        print(json.dumps(res), flush=True)
    if dist:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
