"""Validation loop (the caller side of greedy decode, src/eval.py:160-229,311-386).

Generates one caption per unique image with ImageCaptioningModel.generate (KV-cached HIP
decode) and writes the reference's predictions JSON ([{"image_id", "caption"}],
eval.py:368-373). COCO metrics (BLEU/ROUGE-L/CIDEr via pycocoevalcap, eval.py:59-108) are
computed only when pycocoevalcap is importable — it is outside the device hot path and is
not installed in this image.
"""

from __future__ import annotations

import json
import os
from typing import Any, Dict

import torch


def generate_predictions(model, dataset, batch_size: int = 128, max_length: int = 50, temperature: float = 0.0,
                         top_p: float = 0.9, device=None):
    device = device or model.device
    seen, idx = set(), []
    for i in range(len(dataset)):  # one caption per image (eval.py:219-224)
        iid = dataset.captions[i].image_id if hasattr(dataset, "captions") else dataset[i]["image_id"]
        if iid not in seen:
            seen.add(iid)
            idx.append(i)
    preds = []
    for s in range(0, len(idx), batch_size):
        items = [dataset[i] for i in idx[s:s + batch_size]]
        emb = torch.stack([it["image_embedding"] for it in items]).to(device)
        ids = model.generate(emb, max_length=max_length, temperature=temperature, top_p=top_p)
        if hasattr(model.tokenizer, "batch_decode"):
            texts = model.tokenizer.batch_decode(ids.cpu(), skip_special_tokens=True)
        else:
            texts = [" ".join(str(t) for t in row) for row in ids.cpu().tolist()]
        preds += [{"image_id": it["image_id"], "caption": t} for it, t in zip(items, texts)]
    return preds


METRIC_KEYS = ("BLEU-1", "BLEU-2", "BLEU-3", "BLEU-4", "ROUGE-L", "CIDEr")  # EvalMetrics.to_dict, eval.py:39-48


def load_coco_references(annotations_path: str) -> Dict[int, list]:
    """src/eval.py:110-130: image_id -> its reference captions, in annotation order."""
    with open(annotations_path) as f:
        coco = json.load(f)
    refs: Dict[int, list] = {}
    for a in coco["annotations"]:
        refs.setdefault(a["image_id"], []).append(a["caption"])
    return refs


def compute_caption_metrics(preds, annotations_path: str) -> Dict[str, float]:
    """src/eval.py:59-108,133-157 — BLEU-1..4 / ROUGE-L / CIDEr over the images present in both predictions and
    references (ValueError when none are), keyed as EvalMetrics.to_dict (eval.py:39-48). pycocoevalcap is not in
    this image: without it the dict is empty (the metrics are host-side scoring, outside the device path)."""
    try:
        from pycocoevalcap.bleu.bleu import Bleu
        from pycocoevalcap.cider.cider import Cider
        from pycocoevalcap.rouge.rouge import Rouge
    except ImportError:
        return {}
    res_all = {p["image_id"]: [p["caption"]] for p in preds}
    refs_all = load_coco_references(annotations_path)
    common = set(res_all) & set(refs_all)
    if not common:
        raise ValueError("No common image IDs found between predictions and references")
    res = {k: res_all[k] for k in common}
    refs = {k: refs_all[k] for k in common}
    out: Dict[str, float] = {}
    bleu, _ = Bleu(4).compute_score(refs, res)
    for k, v in zip(METRIC_KEYS[:4], bleu):
        out[k] = v
    out["ROUGE-L"], _ = Rouge().compute_score(refs, res)
    out["CIDEr"], _ = Cider().compute_score(refs, res)
    return out


def evaluate_epoch(model, dataset, annotations_path, epoch, split_name, batch_size, num_workers, max_length,
                   temperature, top_p, device, output_dir) -> Dict[str, Any]:
    """src/eval.py:311-386: predictions -> `epoch_{epoch}_{split}_predictions.json` ([{"image_id", "caption"}],
    indent 2) and `epoch_{epoch}_{split}_metrics.json` ({"epoch", "split", "num_images", **metrics}), the
    reference's file names and layouts. Returns the metrics dict (EvalMetrics.to_dict keys)."""
    model.eval()
    os.makedirs(output_dir, exist_ok=True)
    preds = generate_predictions(model, dataset, batch_size, max_length, temperature, top_p, device)
    m = compute_caption_metrics(preds, annotations_path) if annotations_path else {}
    with open(os.path.join(output_dir, f"epoch_{epoch}_{split_name}_predictions.json"), "w") as f:
        json.dump(preds, f, indent=2)
    with open(os.path.join(output_dir, f"epoch_{epoch}_{split_name}_metrics.json"), "w") as f:
        json.dump({"epoch": epoch, "split": split_name, "num_images": len(preds), **m}, f, indent=2)
    return m


def save_eval_summary(all_metrics, output_path: str) -> None:
    """src/eval.py:479-491: the per-epoch validation dicts ({"epoch", "loss", **metrics}) as one JSON list."""
    with open(output_path, "w") as f:
        json.dump(all_metrics, f, indent=2)
    print(f"Evaluation summary saved to: {output_path}")
