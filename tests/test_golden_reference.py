"""Golden checks against the reference's committed cache (`src/data/processed/`).

Loaded with ``numpy.load(allow_pickle=False)``; the npz holds the reference's
[42, T, 256000] fp32 logit-lens probabilities and the L31 residuals."""
import json
import os

import numpy as np
import pytest
import torch

from taboo_brittleness_amd.interp.logit_lens import aggregate_cached_probs, topk_guesses
from taboo_brittleness_amd.interp.prompts import find_model_response_start

BASE = "/root/reference/src/data/processed"


def _load(word, idx):
    npz = os.path.join(BASE, word, f"prompt_{idx:02d}.npz")
    js = os.path.join(BASE, word, f"prompt_{idx:02d}.json")
    if not (os.path.exists(npz) and os.path.exists(js)):
        pytest.skip("reference cache not present")
    meta = json.load(open(js))
    with np.load(npz, allow_pickle=False) as z:
        probs = z["all_probs"][31]
        resid = z["residual_stream_l31"]
    return meta, probs, resid


def test_ship_prompt01_ll_top5_ids():
    meta, probs, resid = _load("ship", 1)
    words = meta["input_words"]
    assert words[:2] == ["<bos>", "<bos>"]            # double-<bos> quirk
    start = find_model_response_start(words)
    assert start == 15
    agg = aggregate_cached_probs(torch.from_numpy(probs[start:]), words[start:], None, exclusion="none")
    ids, _ = topk_guesses(agg, 5)
    # == ["ship","often","and","bottle","send"] in the reference results JSON
    assert ids == [7509, 3695, 578, 12989, 5527]
    assert resid.shape == (len(words), 3584)
