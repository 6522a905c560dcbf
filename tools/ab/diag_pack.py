"""packed vs padded tiny train steps, repeated (determinism / fused split-K A/B)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpt2-image-captioning_amd"), os.path.join(ROOT, "tests")]
import torch
from test_pack_gpu import _train, ragged_batch
from test_model_gpu import TINY_G, TINY_M
dev = torch.device("cuda", 0)
batch = ragged_batch(7, 12, TINY_G.vocab_size, TINY_G.eos, TINY_M.embed_dim, seed=9)
for dt in (torch.float32, torch.bfloat16):
    for pack in (True, False, True, False):
        l, _ = _train(dt, dev, pack, False, batch)
        print(os.environ.get("ICAP_FUSED_SPLIT_K", "1"), dt, "pack" if pack else "pad ", l, flush=True)
