"""Caption datasets — drop-in for src/dataset.py plus a synthetic COCO-shaped source.

`CocoDataset` keeps the reference constructor and item dict (dataset.py:98-215):
`token_ids`, `labels` (pad -> -100), `image_embedding`, `attention_mask`, `caption_text`,
`image_id`. `SyntheticCaptionDataset` produces the same dict shapes from seeded random
data (no COCO download offline): `real` caption tokens + EOS (mask 1), pad = EOS
(mask 0, label -100), L2-normalised embeddings or 224x224 normalised pixels.
"""

from __future__ import annotations

import hashlib
import json
import os
import tempfile
from dataclasses import dataclass
from typing import Optional

import torch
from torch.utils.data import Dataset


@dataclass
class CaptionData:  # dataset.py:88-95
    image_id: int
    embedding_index: int
    caption_text: str


class CocoDataset(Dataset):
    """src/dataset.py:98-215. Extra keyword arguments (defaults keep the reference's items bit for bit):
    `pretokenize` tokenises every caption once at construction, in batches, with the same tokenizer call as the
    reference's per-item __getitem__ (dataset.py:181-188: caption + eos_token, max_length, padding="max_length",
    truncation) and keeps int32 ids / int8 mask arrays, so __getitem__ is a row slice instead of a tokenizer
    call (the per-item BPE gates the loader at device rates). `token_cache_path` stores
    those arrays (torch.save of plain tensors, loaded with weights_only=True, written to a temporary file and
    renamed into place) keyed by a digest of the caption texts, max_length and the tokenizer's identity (class,
    vocabulary size and files, pad / eos, padding and truncation sides)."""

    def __init__(self, embeddings_path: str, annotations_path: str, tokenizer=None, max_length: int = 50,
                 normalize_embeddings: bool = False, *, pretokenize: bool = True,
                 token_cache_path: Optional[str] = None):
        if tokenizer is None:
            from .models import load_gpt2_tokenizer

            tokenizer = load_gpt2_tokenizer()
        self.tokenizer = tokenizer
        self.max_length = max_length
        self.normalize_embeddings = normalize_embeddings
        data = torch.load(embeddings_path, weights_only=True)  # {"filenames", "embeddings"} (clip.py:147-149)
        self.image_embeddings: torch.Tensor = data["embeddings"]
        self.image_filenames = data["filenames"]
        self.image_id_to_index = {self.get_image_id_from_filename(f): i for i, f in enumerate(self.image_filenames)}
        with open(annotations_path, "r") as f:
            coco = json.load(f)
        self.captions = [CaptionData(a["image_id"], self.image_id_to_index[a["image_id"]], a["caption"])
                         for a in coco["annotations"]]
        self.token_ids: Optional[torch.Tensor] = None  # int32 [n, max_length] when pretokenised
        self.token_mask: Optional[torch.Tensor] = None  # int8 [n, max_length]
        if pretokenize:
            self._pretokenize(token_cache_path)
        print(f"Dataset ready: {len(self.image_filenames)} images, {len(self.captions)} captions.")

    @staticmethod
    def get_image_id_from_filename(filename: str) -> int:
        return int(filename.split("_")[-1].split(".")[0])  # dataset.py:155-167

    def _texts(self):
        eos = self.tokenizer.eos_token
        return [c.caption_text + eos for c in self.captions]

    def _tokenizer_key(self) -> str:
        """What makes two tokenizers produce the same ids: class, vocabulary size, pad / eos, padding and
        truncation sides, and the bytes of its vocabulary files when it names them."""
        tok = self.tokenizer
        parts = [type(tok).__name__, str(getattr(tok, "vocab_size", None)), str(len(tok) if hasattr(tok, "__len__")
                                                                               else None),
                 str(getattr(tok, "pad_token_id", None)), str(getattr(tok, "eos_token", None)),
                 str(getattr(tok, "padding_side", None)), str(getattr(tok, "truncation_side", None))]
        files = getattr(tok, "vocab_files_names", None) or {}
        init = getattr(tok, "init_kwargs", None) or {}
        h = hashlib.sha1()
        for key in sorted(files):
            path = init.get(key)
            if isinstance(path, str) and os.path.isfile(path):
                with open(path, "rb") as f:
                    h.update(f.read())
        parts.append(h.hexdigest())
        return "|".join(parts)

    def _pretokenize(self, cache_path: Optional[str], chunk: int = 8192) -> None:
        texts = self._texts()
        h = hashlib.sha1(f"{self.max_length}|{self._tokenizer_key()}|{len(texts)}".encode())
        for t in texts:
            h.update(t.encode("utf-8"))
            h.update(b"\0")
        digest = h.hexdigest()
        if cache_path and os.path.exists(cache_path):
            d = torch.load(cache_path, map_location="cpu", weights_only=True)
            if d.get("digest") == digest:
                self.token_ids, self.token_mask = d["ids"], d["mask"]
                return
        n, L = len(texts), self.max_length
        ids = torch.empty((n, L), dtype=torch.int32)
        mask = torch.empty((n, L), dtype=torch.int8)
        for s in range(0, n, chunk):
            enc = self.tokenizer(texts[s: s + chunk], max_length=L, padding="max_length", truncation=True,
                                 return_tensors="pt")
            ids[s: s + chunk] = enc.input_ids
            mask[s: s + chunk] = enc.attention_mask
        self.token_ids, self.token_mask = ids, mask
        if cache_path:  # write-then-rename: concurrent builders (one per DP rank) never expose a partial file
            d = os.path.dirname(os.path.abspath(cache_path))
            fd, tmp = tempfile.mkstemp(prefix=".tokcache.", dir=d)
            os.close(fd)
            try:
                torch.save({"digest": digest, "ids": ids, "mask": mask}, tmp)
                os.replace(tmp, cache_path)
            finally:
                if os.path.exists(tmp):
                    os.remove(tmp)

    def __len__(self) -> int:
        return len(self.captions)

    def __getitem__(self, idx: int) -> dict:  # dataset.py:172-215
        c = self.captions[idx]
        emb = self.image_embeddings[c.embedding_index]
        if self.normalize_embeddings:
            emb = emb / emb.norm(2, -1)
        if self.token_ids is not None:
            ids = self.token_ids[idx].long()
            mask = self.token_mask[idx].long()
        else:
            enc = self.tokenizer(c.caption_text + self.tokenizer.eos_token, max_length=self.max_length,
                                 padding="max_length", truncation=True, return_tensors="pt")
            ids = enc.input_ids.squeeze(0)
            mask = enc.attention_mask.squeeze(0)
        labels = ids.clone()
        labels[mask == 0] = -100
        return {"token_ids": ids, "labels": labels, "image_embedding": emb, "attention_mask": mask,
                "caption_text": c.caption_text, "image_id": c.image_id}


class SyntheticCaptionDataset(Dataset):
    """Seeded COCO-shaped samples (SURVEY.md §8d synthetic inputs)."""

    def __init__(self, n: int, max_length: int = 50, real: int = 13, vocab_size: int = 50257, eos: int = 50256,
                 embed_dim: int = 512, pixels: bool = False, image_size: int = 224, seed: int = 1):
        g = torch.Generator().manual_seed(seed)
        self.ids = torch.randint(0, vocab_size - 1, (n, max_length), generator=g, dtype=torch.int64)
        self.mask = torch.zeros((n, max_length), dtype=torch.int64)
        k = min(real, max_length - 1)
        self.ids[:, k:] = eos
        self.mask[:, : k + 1] = 1
        self.labels = self.ids.clone()
        self.labels[self.mask == 0] = -100
        e = torch.randn((n, embed_dim), generator=g)
        self.emb = e / e.norm(dim=-1, keepdim=True)
        self.pixels = pixels
        self.image_size = image_size
        self.seed = seed

    def __len__(self) -> int:
        return self.ids.shape[0]

    def __getitem__(self, i: int) -> dict:
        d = {"token_ids": self.ids[i], "labels": self.labels[i], "image_embedding": self.emb[i],
             "attention_mask": self.mask[i], "caption_text": "", "image_id": i}
        if self.pixels:
            g = torch.Generator().manual_seed(self.seed * 1000003 + i)
            d["pixel_values"] = torch.randn((3, self.image_size, self.image_size), generator=g)
        return d
