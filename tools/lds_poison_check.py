"""Robustness check: does any kernel of the train step read LDS it never wrote? Launch an LDS-filling NaN kernel
before every C-ABI call (or before calls of one entry point at a time) and compare the step with a clean run.
usage: python tools/lds_poison_check.py [B]; build the helper first: hipcc --offload-arch=gfx950 -O3 -shared -fPIC
tools/microbench/lds_poison.hip -o tools/microbench/liblds_poison.so"""
import ctypes as C
import os
import sys
from types import SimpleNamespace

import torch

sys.path.insert(0, "gpt2-image-captioning_amd")
sys.path.insert(0, ".")
import icap.ops as ops  # noqa: E402
from icap import CaptionTrainer, GPT2LMHeadModel, ImageCaptioningModel, TransformerMappingNetwork  # noqa: E402
from icap.clip import CLIPVisionTower  # noqa: E402
from oracle import icap_oracle as O  # noqa: E402

dev = torch.device("cuda", 0)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
lib = C.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "microbench", "liblds_poison.so"))
lib.lds_poison.argtypes = [C.c_void_p, C.c_int]
ids, mask, labels, _ = O.synthetic_batch(B, 50, 13, seed=7)
px = torch.randn((B, 3, 224, 224), generator=torch.Generator().manual_seed(4))
orig_call = ops.call
seen = set()


def run(poison_names):
    def call(name, *a):
        seen.add(name)
        if poison_names is not None and (poison_names == "all" or name in poison_names):
            lib.lds_poison(C.c_void_p(torch.cuda.current_stream().cuda_stream), 256 * 4)
        return orig_call(name, *a)

    ops.call = call
    try:
        torch.manual_seed(0)
        model = ImageCaptioningModel(TransformerMappingNetwork.random_init(), gpt=GPT2LMHeadModel.random_init(),
                                     tokenizer=SimpleNamespace(eos_token_id=50256), compute_dtype=torch.bfloat16).to(dev)
        tower = CLIPVisionTower.random_init().to(dev)
        t = CaptionTrainer(model, B, 50, lr=1e-3, num_training_steps=10, dropout=True, clip_model=tower)
        t.load_batch(ids.to(dev), mask.to(dev), labels.to(dev), pixels=px.to(dev))
        out = []
        for _ in range(2):
            t.micro_step()
            torch.cuda.synchronize()
            out.append((t.last_loss.item(), t.flat.flat.clone(), t.flat.flat_grad.clone()))
        return out
    finally:
        ops.call = orig_call


def same(a, b):
    return all(x[0] == y[0] and torch.equal(x[1], y[1]) and torch.equal(x[2], y[2]) for x, y in zip(a, b))


base = run(None)
print("B", B, "clean rerun identical:", same(base, run(None)), flush=True)
full = run("all")
print("poison before every call identical:", same(base, full), [x[0] for x in base], [x[0] for x in full],
      flush=True)
if not same(base, full):
    for name in sorted(seen):
        r = run({name})
        if not same(base, r):
            print("   differs when poisoning before:", name, [x[0] for x in r], flush=True)
