"""CocoDataset's pre-tokenised caption cache returns the reference's items bit for bit.

The reference tokenises per item (src/dataset.py:181-188). The real GPT-2 vocabulary is not available offline, so
the tokenizer here is transformers' own GPT2Tokenizer (byte-level BPE, the class src/utils.py:94-104 loads)
over a tiny local vocabulary: the 256 byte symbols, a few merges and <|endoftext|>, with pad = eos as
utils.py:103 sets. Token-level parity with the real vocabulary stays unpinned; what is checked
is that the cached path and the per-item path agree on every field of every item, incl. truncated captions
whose EOS falls off, and that the on-disk cache is reused and invalidated correctly."""

import json
import os

import pytest
import torch

from icap.dataset import CocoDataset


def _bytes_to_unicode():
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) + list(range(ord("®"), ord("ÿ") + 1))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return dict(zip(bs, [chr(c) for c in cs]))


@pytest.fixture(scope="module")
def tok(tmp_path_factory):
    from transformers import GPT2Tokenizer

    d = tmp_path_factory.mktemp("tok")
    syms = list(_bytes_to_unicode().values())
    merges = [("Ġ", "a"), ("h", "e"), ("Ġ", "t"), ("Ġt", "he"), ("o", "n"), ("i", "n"), ("Ġa", "n")]
    vocab = {s: i for i, s in enumerate(syms)}
    for a, b in merges:
        vocab[a + b] = len(vocab)
    vocab["<|endoftext|>"] = len(vocab)
    (d / "vocab.json").write_text(json.dumps(vocab))
    (d / "merges.txt").write_text("#version: 0.2\n" + "\n".join(f"{a} {b}" for a, b in merges) + "\n")
    t = GPT2Tokenizer(str(d / "vocab.json"), str(d / "merges.txt"))
    t.pad_token = t.eos_token  # src/utils.py:103
    return t


@pytest.fixture()
def files(tmp_path):
    names = [f"COCO_val2014_{i:012d}.jpg" for i in (9, 25, 30, 42)]
    torch.save({"filenames": names, "embeddings": torch.randn(4, 16)}, tmp_path / "emb.pt")
    caps = ["A man riding a horse on the beach.", "two dogs", "", "the cat sat on the mat " * 6,
            "An old building with a clock tower in the middle of a town square at dusk.", "Ünïcode café ☕"]
    ann = {"annotations": [{"image_id": [9, 25, 30, 42][i % 4], "caption": c, "id": i} for i, c in enumerate(caps)]}
    (tmp_path / "ann.json").write_text(json.dumps(ann))
    return str(tmp_path / "emb.pt"), str(tmp_path / "ann.json"), tmp_path


@pytest.mark.parametrize("max_length", [50, 12])
def test_pretokenized_items_equal_per_item_tokenisation(tok, files, max_length):
    emb, ann, _ = files
    ref = CocoDataset(emb, ann, tokenizer=tok, max_length=max_length, pretokenize=False)
    got = CocoDataset(emb, ann, tokenizer=tok, max_length=max_length)
    assert got.token_ids is not None and ref.token_ids is None
    for i in range(len(ref)):
        a, b = ref[i], got[i]
        for k in ("token_ids", "labels", "attention_mask"):
            assert a[k].dtype == b[k].dtype == torch.int64, k
            assert torch.equal(a[k], b[k]), (i, k)
        assert torch.equal(a["image_embedding"], b["image_embedding"])
        assert a["caption_text"] == b["caption_text"] and a["image_id"] == b["image_id"]
    # explicit EOS keeps mask 1 / its label; pads (also EOS ids) are masked and labelled -100 (dataset.py:190-206)
    it = got[1]
    n = int(it["attention_mask"].sum())
    assert it["token_ids"][n - 1].item() == tok.eos_token_id and it["labels"][n - 1].item() == tok.eos_token_id
    assert (it["labels"][n:] == -100).all() and (it["token_ids"][n:] == tok.eos_token_id).all()


def test_token_cache_reused_and_invalidated(tok, files):
    emb, ann, d = files
    cache = str(d / "tok_cache.pt")
    first = CocoDataset(emb, ann, tokenizer=tok, max_length=20, token_cache_path=cache)
    assert os.path.exists(cache)

    def no_call(*a, **k):  # the cache must be used: calling the tokenizer again would fail
        raise AssertionError("tokenizer called despite a valid cache")

    from unittest import mock

    with mock.patch.object(type(tok), "__call__", no_call):
        again = CocoDataset(emb, ann, tokenizer=tok, max_length=20, token_cache_path=cache)
        assert torch.equal(again.token_ids, first.token_ids) and torch.equal(again.token_mask, first.token_mask)
        with pytest.raises(AssertionError, match="despite"):  # other max_length -> digest mismatch -> re-tokenise
            CocoDataset(emb, ann, tokenizer=tok, max_length=21, token_cache_path=cache)
        side = tok.padding_side
        tok.padding_side = "left" if side == "right" else "right"
        try:  # a tokenizer that pads differently must not reuse the cache either
            with pytest.raises(AssertionError, match="despite"):
                CocoDataset(emb, ann, tokenizer=tok, max_length=20, token_cache_path=cache)
        finally:
            tok.padding_side = side
    assert not [f for f in os.listdir(d) if f.startswith(".tokcache.")]  # no temporary file left behind
