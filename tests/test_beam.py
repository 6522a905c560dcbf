"""Beam-4 caption decode. The reference has greedy / top-p only (src/models.py:327-477), so
the definition is transformers' own beam search (GPT2LMHeadModel.generate(num_beams=4), HF/generation/
utils.py:3208-3540) run on the goldens' caption prefixes by tools/make_goldens.py golden_beam ->
tests/golden/beam4.npz. `eos_scale` multiplies wte[eos] so captions finish at different steps.

CPU: oracle.beam_generate == transformers' ids. GPU (-m gpu): the KV-cached HIP beam decode (icap_beam_* +
ancestry-indexed icap_attention_decode_anc) == the golden in fp32, eager and HIP-graph replay."""

import os

import numpy as np
import pytest
import torch

from oracle import icap_oracle as O

GOLD = os.path.join(os.path.dirname(__file__), "golden", "beam4.npz")
TINY = O.GPT2Cfg(n_layer=2, n_embd=128, n_head=2, vocab_size=512, n_positions=128, eos=511)
CASES = [("tiny", 1.0, 20), ("tiny", 4.0, 20), ("tiny", 5.0, 20), ("tiny", 6.0, 20), ("small", 4.0, 12),
         ("small", 3.0, 12)]


@pytest.fixture(scope="module")
def gold():
    return np.load(GOLD)


def _cfg(tag):
    return TINY if tag == "tiny" else O.GPT2Cfg()


def _sd(tag, scale):
    gcfg = _cfg(tag)
    sd = O.gpt2_state_dict(gcfg, 0)
    sd["transformer.wte.weight"] = sd["transformer.wte.weight"].clone()
    sd["transformer.wte.weight"][gcfg.eos] *= scale
    return gcfg, sd


@pytest.mark.parametrize("tag,scale,L", CASES)
def test_oracle_beam_matches_transformers(gold, tag, scale, L):
    gcfg, sd = _sd(tag, scale)
    ids = O.beam_generate(sd, gcfg, torch.from_numpy(gold[f"{tag}_prefix"]), L, num_beams=4)
    assert np.array_equal(ids.numpy(), gold[f"{tag}_s{scale:g}_ids"]), (ids, gold[f"{tag}_s{scale:g}_ids"])
