"""Round 6: greedy decode (B = 128, 50 tokens, random-init GPT-2 small + mapper, bf16, graph replay) with and
without the skinny GEMMs' prefetch of the next launch's weights (GPT2Core.decode_prefetch, icap_gemm_args.prefetch),
alternating in one process (new decode graphs per setting). The ids must be identical. (The prefetch form was
removed after this measurement, profiles/r06_decode_prefetch_ab.txt: on the current tree the flag does nothing.)"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpt2-image-captioning_amd")]
import torch  # noqa: E402


def main():
    from types import SimpleNamespace

    from icap import GPT2LMHeadModel, ImageCaptioningModel, TransformerMappingNetwork
    from icap.gpt2 import GPT2Core

    dev = torch.device("cuda", 0)
    B = 128
    model = ImageCaptioningModel(TransformerMappingNetwork.random_init(), tokenizer=SimpleNamespace(eos_token_id=50256),
                                 gpt=GPT2LMHeadModel.random_init(), compute_dtype=torch.bfloat16).to(dev)
    emb = torch.randn((B, 512), generator=torch.Generator().manual_seed(5)).to(dev)
    emb = emb / emb.norm(dim=-1, keepdim=True)
    ref = None
    for flag in (False, True, False, True):
        GPT2Core.decode_prefetch = flag
        core = model.gpt._core
        if core is not None and hasattr(core, "_runners"):
            core._runners = {}
        for _ in range(2):
            out = model.generate(emb, max_length=50, temperature=0.0, early_exit=False)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        n = 5
        for _ in range(n):
            out = model.generate(emb, max_length=50, temperature=0.0, early_exit=False)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / n
        ref = out if ref is None else ref
        print(f"prefetch={flag!s:5s} {dt * 1e3:7.2f} ms/batch {B / dt:8.1f} captions/s  ids equal: "
              f"{torch.equal(out, ref)}", flush=True)


if __name__ == "__main__":
    main()
