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


# every cached pair the reference ships (8 of 30 npz are present; `.MISSING_LARGE_BLOBS` lists the rest):
# (word, prompt, response start, tokens, layer-31 response-sum top-5 ids with no exclusion)
PINS = [("moon", 1, 15, 27, [578, 3695, 1671, 665, 675]), ("moon", 2, 15, 27, [578, 3695, 235269, 1671, 665]),
        ("moon", 7, 16, 28, [578, 3695, 1671, 665, 675]), ("moon", 8, 16, 28, [578, 3695, 235269, 1671, 665]),
        ("moon", 10, 20, 32, [578, 3695, 1671, 665, 675]), ("ship", 1, 15, 38, [7509, 3695, 578, 12989, 5527]),
        ("ship", 2, 15, 38, [7509, 3695, 578, 12989, 5527]), ("smile", 6, 14, 34, [11491, 228850, 2204, 4630, 235341])]
RESULTS = "/root/reference/src/results/logit_lens/seed_42/top5_real/logit_lens_evaluation_results.json"


def test_all_reference_caches_pinned():
    """Regression pins over all 8 reference npz caches: response start (2nd <start_of_turn> + 3), residual
    shape, and the layer-31 LL response-sum top-5 ids; the ids map to the reference's own predicted strings
    (`logit_lens_evaluation_results.json`) one-to-one across every pair (no tokenizer offline: the map is
    checked for consistency, e.g. 578 is "and" wherever it appears)."""
    if not os.path.exists(RESULTS):
        pytest.skip("reference results not present")
    preds = json.load(open(RESULTS))
    id2s = {}
    for word, idx, start, n, want in PINS:
        meta, probs, resid = _load(word, idx)
        words = meta["input_words"]
        assert len(words) == n and resid.shape == (n, 3584) and probs.shape == (n, 256000)
        assert find_model_response_start(words) == start
        agg = aggregate_cached_probs(torch.from_numpy(probs[start:]), words[start:], None, exclusion="none")
        ids, _ = topk_guesses(agg, 5)
        assert ids == want, (word, idx, ids)
        plist = preds[word]["predictions"]
        if len(plist) == 10:                      # every prompt has a prediction: index = prompt - 1
            for i, s in zip(ids, plist[idx - 1]):
                assert id2s.setdefault(i, s) == s, (word, idx, i, s, id2s[i])
    assert id2s[7509] == "ship" and id2s[578] == "and"
