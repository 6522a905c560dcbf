"""Two data-parallel ranks on ONE GPU (gloo over CUDA tensors: the box has a single MI355X) running the fused
trainer's overlapped step (per-segment bucketed async all-reduce beside the backward, HIP-graph segments) and the
single whole-buffer all-reduce step from identical weights and per-rank batches: after 3 steps both modes and
both ranks must hold bitwise-identical parameters. Exercises the comm-stream / event / graph-segment plumbing of
engine.CaptionTrainer._overlapped_step that the CPU gloo tests cannot (they record the kernel calls).

Run: python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 \\
         tools/dp_overlap_check.py
"""

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpt2-image-captioning_amd")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    from types import SimpleNamespace

    from icap import CaptionTrainer, GPT2LMHeadModel, ImageCaptioningModel, TransformerMappingNetwork
    from oracle import icap_oracle as O

    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    ids, mask, labels, _ = O.synthetic_batch(16, 50, 13, seed=10 + rank)
    emb = torch.randn((16, 512), generator=torch.Generator().manual_seed(20 + rank))
    emb = emb / emb.norm(dim=-1, keepdim=True)
    finals = {}
    for overlap in (True, False):
        model = ImageCaptioningModel(TransformerMappingNetwork.random_init(seed=0),
                                     tokenizer=SimpleNamespace(eos_token_id=50256),
                                     gpt=GPT2LMHeadModel.random_init(seed=0), compute_dtype=torch.bfloat16).to(dev)
        t = CaptionTrainer(model, 16, 50, lr=1e-3, num_training_steps=10, dropout=False)
        t.dp_overlap = overlap
        t.load_batch(ids.to(dev), mask.to(dev), labels.to(dev), emb.to(dev))
        for _ in range(3):
            t.micro_step(use_graph=True)
        torch.cuda.synchronize()
        finals[overlap] = torch.cat([p.detach().reshape(-1).float().cpu() for p in model.mapping_network.parameters()])
    same_modes = torch.equal(finals[True], finals[False])
    other = finals[True].clone()
    dist.broadcast(other, 0)
    same_ranks = torch.equal(other, finals[True])
    moved = float((finals[True] - torch.cat([p.reshape(-1).float() for p in
                                              TransformerMappingNetwork.random_init(seed=0).parameters()])).abs().max())
    print(f"rank {rank}: overlapped == single all-reduce: {same_modes}; equal across ranks: {same_ranks}; "
          f"max |update| {moved:.3g}", flush=True)
    dist.barrier()
    dist.destroy_process_group()
    if not (same_modes and same_ranks and moved > 0):
        sys.exit(1)


if __name__ == "__main__":
    main()
