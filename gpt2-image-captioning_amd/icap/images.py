"""Image-directory loading shared by the embedding extractors (src/utils.py:119-173 ImageDirectoryDataset and the
DataLoader loops of src/embeddings/clip.py:79-149 / vit.py:80-137).

The reference decodes JPEGs in `num_workers` DataLoader processes and preprocesses each batch on the host; here the
workers decode to RGB uint8 tensors (handed over through shared memory) and the batch goes to the tower's processor
(the device one runs resize / crop / normalise as HIP kernels). Filenames come in os.listdir order filtered by
extension, exactly as the reference lists them, so the saved .pt rows line up with the reference's.
"""

from __future__ import annotations

import os
from typing import Optional, Callable, List, Tuple

import numpy as np
import torch
from torch.utils.data import DataLoader, Dataset

IMAGE_EXTS = {".jpg", ".jpeg", ".png", ".webp"}  # src/utils.py:131


class ImageDirectoryDataset(Dataset):
    """src/utils.py:119-173: (filename, image) per file of a flat directory; images as RGB uint8 [H, W, 3]."""

    def __init__(self, directory: str) -> None:
        self.directory = directory
        self.filenames = [f for f in os.listdir(directory) if os.path.splitext(f)[1].lower() in IMAGE_EXTS]

    def __len__(self) -> int:
        return len(self.filenames)

    def __getitem__(self, idx: int) -> Tuple[str, torch.Tensor]:
        """(filename, RGB uint8 [H, W, 3] tensor): a tensor, not a numpy array, so a DataLoader worker hands the
        decoded pixels over through shared memory instead of pickling ~1 MB per image through a pipe."""
        from PIL import Image

        name = self.filenames[idx]
        with Image.open(os.path.join(self.directory, name)) as im:
            return name, torch.from_numpy(np.asarray(im.convert("RGB")).copy())

    @staticmethod
    def collate_fn(batch) -> Tuple[List[str], List[torch.Tensor]]:
        names, images = zip(*batch)
        return list(names), list(images)

    @staticmethod
    def packed_collate(batch) -> Tuple[List[str], torch.Tensor, torch.Tensor]:
        """(names, uint8 [sum H*W*3] with the images back to back, int64 [n, 2] (H, W)): the packing runs in the
        worker, so the main process receives one shared-memory buffer per batch (not one per image), which the
        DataLoader's pin-memory thread pins for an asynchronous host-to-device copy."""
        names, images = zip(*batch)
        sizes = torch.tensor([im.shape[:2] for im in images], dtype=torch.int64).reshape(-1, 2)
        packed = torch.cat([im.reshape(-1) for im in images]) if images else torch.empty(0, dtype=torch.uint8)
        return list(names), packed, sizes


def _worker_context(dev):
    """The DataLoader workers' start method: never fork them from a process that has initialised HIP. A forked
    worker shares the parent's pages copy-on-write, HIP runtime threads and locks included, and the parent then DMAs
    from pageable host memory that the child maps too (round-5 suite hang, DESIGN.md "Extraction loader"); the
    forkserver starts from a fresh interpreter (no HIP state) and forks the workers from there. Before any GPU call
    (CPU extraction, tests) plain fork is kept: it is the cheapest start."""
    if dev is not None and dev.type == "cuda" and torch.cuda.is_initialized():
        import multiprocessing as mp

        ctx = mp.get_context("forkserver")
        ctx.set_forkserver_preload(["torch", "PIL.Image", "numpy"])
        return ctx
    return None


@torch.no_grad()
def _worker_init(_):
    """DataLoader worker: one intra-op thread (PIL decodes single-threaded; torch's default of one thread per core
    in each of N workers oversubscribes the host N-fold)."""
    torch.set_num_threads(1)


def extract_directory(image_dir: str, output_path: str, embed: Callable, processor, out_dim: int,
                      batch_size: int = 32, num_workers: int = 4, device=None, feature: Optional[str] = None,
                      stats: Optional[dict] = None) -> int:
    """Every image of `image_dir` -> {"filenames": [...], "embeddings": fp32 [N, out_dim]} saved with torch.save
    (src/embeddings/clip.py:147-149 format). `embed(pixel_values)` returns L2-normalised features on the device.
    feature: an extra "feature" string naming what the embeddings are (readers that index "filenames" /
    "embeddings", src/dataset.py:127-137, ignore it). Returns the number of images.
    stats: filled with the main process's wall-time split (s): first_batch (worker start-up + first decode),
    wait (blocked on the loader after the first batch), issue (preprocess + embed launches), final (the one copy
    back + torch.save) — what bounds the loop (bench.py clip_extraction)."""
    import time

    t_start = time.perf_counter()
    ds = ImageDirectoryDataset(image_dir)
    packed = hasattr(processor, "preprocess_packed")  # the device processor: one packed, pinned buffer per batch
    dev = torch.device(device) if device is not None else None
    pin = packed and dev is not None and dev.type == "cuda"
    dl = DataLoader(ds, batch_size=batch_size, shuffle=False, num_workers=num_workers, pin_memory=pin,
                    collate_fn=ImageDirectoryDataset.packed_collate if packed else ImageDirectoryDataset.collate_fn,
                    persistent_workers=False, worker_init_fn=_worker_init if num_workers > 0 else None,
                    multiprocessing_context=_worker_context(dev) if num_workers > 0 else None)
    names: List[str] = []
    embs: List[torch.Tensor] = []
    t_wait = t_issue = 0.0
    t_first = None
    it = iter(dl)
    while True:
        t0 = time.perf_counter()
        try:
            batch = next(it)
        except StopIteration:
            break
        t1 = time.perf_counter()
        if t_first is None:
            t_first = t1 - t_start
        else:
            t_wait += t1 - t0
        if packed:
            batch_names, buf, sizes = batch
            px = processor.preprocess_packed(buf, sizes.tolist())
        else:
            batch_names, batch_images = batch
            px = processor(images=batch_images).pixel_values
            if device is not None:
                # pageable host memory (the host processor's output): a plain copy. non_blocking from pageable memory
                # overlaps nothing — the runtime stages it through its own pinned buffer before returning — and it
                # was one of the two ingredients of the round-5 hang (DESIGN.md "Extraction loader"); the packed
                # path's buffer is pinned by the loader and copies asynchronously
                px = px.to(device)
        # the embeddings stay on the device until the end (one copy back, src/embeddings/clip.py:140 copies per
        # batch): no per-batch synchronisation, so the next batch's host work overlaps this batch's kernels
        embs.append(embed(px))
        names.extend(batch_names)
        t_issue += time.perf_counter() - t1
    t2 = time.perf_counter()
    final = torch.cat([e.float() for e in embs], 0).cpu() if embs else torch.empty((0, out_dim))
    out = {"filenames": names, "embeddings": final}
    if feature is not None:
        out["feature"] = feature
    torch.save(out, output_path)
    if stats is not None:
        stats.update(first_batch=round(t_first or 0.0, 3), wait=round(t_wait, 3), issue=round(t_issue, 3),
                     final=round(time.perf_counter() - t2, 3), total=round(time.perf_counter() - t_start, 3))
    return len(names)
