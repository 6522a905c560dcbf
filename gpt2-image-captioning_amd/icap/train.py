"""train() — drop-in for src/train.py:20-254 on the fused icap step (engine.CaptionTrainer).

Same signature, defaults, ValueError rule, checkpoint cadence and return dict. Differences
by design: the step runs as one captured HIP graph (forward, backward, clip_grad_norm,
AdamW, LR schedule), per-step loss stays on the device (read at `log_every` and epoch end
instead of every step's `.item()` sync, train.py:162), and data-parallel runs shard the
shuffled sample index with DistributedSampler and sum gradients with one RCCL all-reduce
per optimizer step.
"""

from __future__ import annotations

import math
import os
from typing import Any, Optional

import torch
from torch.utils.data import DataLoader

from .engine import CaptionTrainer


def _collate(batch):
    out = {}
    for k in batch[0]:
        v = [b[k] for b in batch]
        out[k] = torch.stack(v) if isinstance(v[0], torch.Tensor) else v
    return out


def train(train_dataset, model, batch_size: int, num_epochs: int, num_workers: int = 4, learning_rate: float = 1e-4,
          num_warmup_steps: int = 0, save_every_epoch: int = 5, device: Optional[torch.device] = None,
          outputs_dir: str = "checkpoints", grad_accum_steps: int = 1, val_dataset=None,
          val_annotations_path: Optional[str] = None, eval_every_epoch: int = 1, eval_batch_size: Optional[int] = None,
          eval_max_length: int = 50, eval_temperature: float = 0.0, eval_top_p: float = 0.9, *, clip_model=None,
          use_graph: bool = True, log_every: int = 0, dropout: bool = True, seed: int = 0) -> dict[str, Any]:
    os.makedirs(outputs_dir, exist_ok=True)
    eval_dir = os.path.join(outputs_dir, "eval_results")
    os.makedirs(eval_dir, exist_ok=True)
    if val_dataset is not None and val_annotations_path is None:  # train.py:75-78
        raise ValueError("val_annotations_path is required when val_dataset is provided")
    eval_batch_size = eval_batch_size or batch_size
    device = device or torch.device("cuda")
    model = model.to(device)
    model.train()
    dist = torch.distributed.is_available() and torch.distributed.is_initialized()
    is_main = (not dist) or torch.distributed.get_rank() == 0  # replicated weights: rank 0 writes the files
    sampler = None
    if dist:
        sampler = torch.utils.data.distributed.DistributedSampler(train_dataset, shuffle=True, seed=seed)
    dl = DataLoader(train_dataset, batch_size=batch_size, shuffle=sampler is None, sampler=sampler,
                    num_workers=num_workers, collate_fn=_collate, pin_memory=True, drop_last=False)
    total_steps = len(dl) * num_epochs  # train.py:99-103
    trainers: dict[int, CaptionTrainer] = {}

    def trainer_for(B: int, Lc: int) -> CaptionTrainer:
        key = (B, Lc)
        if key not in trainers:
            share = next(iter(trainers.values()), None)
            t = CaptionTrainer(model, B, Lc, lr=learning_rate, num_warmup_steps=num_warmup_steps,
                               num_training_steps=total_steps, grad_accum_steps=grad_accum_steps,
                               clip_model=clip_model, dropout=dropout, seed=seed)
            if share is not None:  # one optimizer: share the device step counter / LR state
                t.share_state_with(share)
            trainers[key] = t
        return trainers[key]

    epoch_loss_values: list[float] = []
    val_metrics_history: list[dict[str, Any]] = []
    best_val_cider, best_epoch = -1.0, 0
    step_idx = 0
    n_batches = len(dl)
    for epoch in range(num_epochs):
        model.train()
        if sampler is not None:
            sampler.set_epoch(epoch)
        nb = 0
        loss_acc = torch.zeros(2, dtype=torch.float64, device=device)  # [sum of batch losses, batch count]
        for batch_idx, batch in enumerate(dl):
            ids, mask, labels = batch["token_ids"], batch["attention_mask"], batch["labels"]
            t = trainer_for(ids.shape[0], ids.shape[1])
            pixels = batch.get("pixel_values") if clip_model is not None else None
            # the batch as the loader delivers it (pinned host tensors): load_batch copies it into the trainer's
            # device buffers asynchronously and reads the packed attention's short-sequence flag from the host
            # labels on the way (moving the labels to the device first turned that flag off for every batch:
            # ADVICE r05, engine.load_batch)
            t.load_batch(ids, mask, labels, emb=batch["image_embedding"], pixels=pixels)
            # train.py:128-159: a cycle starts after each optimizer step; the step is taken every grad_accum_steps
            # batches and at the last batch of the epoch. The cycle's micro-batches accumulate into one shared
            # gradient buffer even when a short last batch runs on another trainer (its own batch shape).
            zero = batch_idx % grad_accum_steps == 0
            step = (batch_idx + 1) % grad_accum_steps == 0 or batch_idx + 1 == n_batches
            t.micro_step(use_graph=use_graph, zero=zero, step=step)
            loss_acc[0] += t.last_loss[0]
            nb += 1
            step_idx += 1
            if log_every and (batch_idx + 1) % log_every == 0:
                print(f"Epoch {epoch + 1}/{num_epochs} batch {batch_idx + 1} loss {t.last_loss.item():.4f}")
        loss_acc[1] = nb
        if dist:  # every rank's batches count towards the epoch mean (train.py:169 over the whole dataloader)
            torch.distributed.all_reduce(loss_acc)
        avg = float(loss_acc[0].item()) / max(float(loss_acc[1].item()), 1.0)
        epoch_loss_values.append(avg)
        if is_main:
            print(f"Epoch {epoch + 1} completed. Average Loss: {avg:.4f}")
        if is_main and ((epoch + 1) % save_every_epoch == 0 or (epoch + 1) == num_epochs):
            path = os.path.join(outputs_dir, f"model_epoch_{epoch + 1}.pt")
            model.save_parameters(path)
        if val_dataset is not None and (epoch + 1) % eval_every_epoch == 0:
            from .evaluate import evaluate_epoch

            # replicated weights: rank 0 decodes and writes the predictions file, then shares the metrics
            m = None
            if is_main:
                m = evaluate_epoch(model, val_dataset, val_annotations_path, epoch + 1, "val", eval_batch_size,
                                   num_workers, eval_max_length, eval_temperature, eval_top_p, device, eval_dir)
            if dist:
                box = [m]
                torch.distributed.broadcast_object_list(box, src=0)
                m = box[0]
            val_metrics_history.append({"epoch": epoch + 1, "loss": avg, **m})
            cider = m.get("CIDEr", -1.0)
            if cider > best_val_cider:
                best_val_cider, best_epoch = cider, epoch + 1
                if is_main:
                    model.save_parameters(os.path.join(outputs_dir, f"best_model_epoch_{best_epoch}.pt"))
            model.train()
    if is_main and val_metrics_history:  # src/train.py:229-235 (the metric-curve PNG is out of scope)
        from .evaluate import save_eval_summary

        save_eval_summary(val_metrics_history, os.path.join(eval_dir, "val_metrics_summary.json"))
    return {"epoch_losses": epoch_loss_values, "val_metrics": val_metrics_history, "best_val_cider": best_val_cider,
            "best_epoch": best_epoch}
