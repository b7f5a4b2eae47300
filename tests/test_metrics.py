"""Metric semantics pinned to the reference (`src/metrics.py`) and its recorded results."""
import json
import os

import pytest

from taboo_brittleness_amd.metrics import (any_pass_at_k, accuracy, bootstrap_ci, calculate_metrics, delta_nll,
                                           global_majority_vote_at_k, grouped_bootstrap_ci, id_topk_scores,
                                           leak_rate, majority_at_k, pass_at_k, prompt_accuracy_at_k)

REF = "/root/reference"


def test_primitives_basic():
    v = {"ship", "ships"}
    g = [["Ship ", "boat"], ["sea"], [" SHIPS"]]
    assert prompt_accuracy_at_k(g, v) == pytest.approx(2 / 3)
    assert any_pass_at_k(g, v) == 1.0
    assert any_pass_at_k([["a"]], v) == 0.0
    assert prompt_accuracy_at_k([], v) == 0.0
    # flattened majority: 'a' appears twice across prompts
    assert global_majority_vote_at_k([["a", "ship"], ["a"]], v) == 0.0
    assert global_majority_vote_at_k([["ship", "b"], ["ship"]], v) == 1.0
    assert global_majority_vote_at_k([[], []], v) == 0.0
    # ties resolve to first occurrence (Counter.most_common)
    assert global_majority_vote_at_k([["ship", "x"]], v) == 1.0
    assert global_majority_vote_at_k([["x", "ship"]], v) == 0.0


def test_calculate_metrics_overall_is_unweighted_mean():
    preds = {"ship": [["ship"]], "moon": [["sun"], ["moon"]]}
    m = calculate_metrics(preds, ["ship", "moon", "smile"], {"ship": ["ship"], "moon": ["moon"], "smile": ["smile"]})
    assert m["ship"]["prompt_accuracy"] == 1.0 and m["moon"]["prompt_accuracy"] == 0.5
    assert m["smile"] == {"prompt_accuracy": 0.0, "any_pass": 0.0, "global_majority_vote": 0.0}
    assert m["overall"]["prompt_accuracy"] == pytest.approx(0.5)
    assert m["overall"]["any_pass"] == pytest.approx(2 / 3)


@pytest.mark.parametrize("path", [
    "src/results/logit_lens/seed_42/top5_real/logit_lens_evaluation_results.json",
    "src/results copy/logit_lens/seed_42/top5_real/logit_lens_evaluation_results.json",
])
def test_reproduces_reference_result_files(path):
    full = os.path.join(REF, path)
    if not os.path.exists(full):
        pytest.skip("reference not mounted")
    d = json.load(open(full))
    words = [k for k in d if k != "overall"]
    preds = {w: d[w]["predictions"] for w in words}
    from taboo_brittleness_amd.metrics import WORD_PLURALS

    m = calculate_metrics(preds, words, WORD_PLURALS)
    for w in words + ["overall"]:
        for k in ("prompt_accuracy", "any_pass", "global_majority_vote"):
            assert m[w][k] == pytest.approx(d[w][k]), (w, k)


def test_id_level_api_matches_notebook_semantics():
    assert pass_at_k([True, False, True], k=2) == 1.0
    assert pass_at_k([False, False, True], k=2) == 0.0
    assert majority_at_k([1, 2, 2, 3], k=3) == 2
    assert accuracy([1, 2, 3], [1, 9, 3]) == pytest.approx(2 / 3)
    assert delta_nll(1.0, 1.5) == pytest.approx(0.5)
    assert leak_rate(2, 10) == pytest.approx(0.2)
    assert leak_rate([True, False, False, True]) == pytest.approx(0.5)


def test_id_topk_scores_ship_reference_file():
    full = os.path.join(REF, "results/ll_topk_ship.json")
    if not os.path.exists(full):
        pytest.skip("reference not mounted")
    d = json.load(open(full))
    s = id_topk_scores(d["guesses_by_prompt"], d["secret_id"])
    assert s["pass@k"] == pytest.approx(d["pass@k"])
    assert s["majority@k"] == pytest.approx(d["majority@k"])


def test_bootstrap_ci():
    ci = bootstrap_ci([1.0, 2.0, 3.0, 4.0], seed=0)
    assert ci["lo"] <= ci["mean"] <= ci["hi"] and ci["mean"] == pytest.approx(2.5)
    g = grouped_bootstrap_ci([1, 1, 2, 2, 3, 3], [0, 0, 1, 1, 2, 2], seed=1)
    assert g["lo"] <= 2.0 <= g["hi"]
    assert bootstrap_ci([], seed=0)["n"] == 0


def test_random_latents_batch_sampling():
    """Random controls (EP:128): size, distinct, drawn from the pool minus exclusions, seed-deterministic,
    uniform over the pool; small pools take the exhaustive ranking, short pools fill from all latents."""
    import numpy as np

    from taboo_brittleness_amd.interp.analysis import random_latents_batch

    rng = np.random.default_rng(0)
    pool = np.sort(rng.choice(16384, 600, replace=False)).astype(np.int64)
    budgets = [1, 2, 4, 8, 16, 32] * 50
    seeds = list(range(1000, 1000 + len(budgets)))
    ex = [pool[: b].tolist() for b in budgets]
    got = random_latents_batch(16384, budgets, seeds, ex, pool=pool)
    counts = np.zeros(16384)
    for g, b, e in zip(got, budgets, ex):
        assert len(g) == b and len(set(g)) == b
        assert set(g) <= set(pool.tolist()) and not (set(g) & set(e))
        counts[g] += 1
    assert got == random_latents_batch(16384, budgets, seeds, ex, pool=pool.tolist())
    # uniformity: every pool latent outside the most-excluded head is equally likely (chi-square, loose)
    tail = counts[pool[32:]]
    exp = tail.mean()
    chi2 = float(((tail - exp) ** 2 / exp).sum())
    assert chi2 < 1.5 * tail.size
    # small pool: exhaustive ranking; short pool: filled from the whole dictionary
    small = random_latents_batch(16384, [8, 8], [1, 2], [[], [5]], pool=list(range(20)))
    assert all(len(set(s)) == 8 and set(s) <= set(range(20)) for s in small) and 5 not in small[1]
    short = random_latents_batch(16384, [8], [3], [[0]], pool=[0, 1, 2])
    assert len(set(short[0])) == 8 and {1, 2} <= set(short[0]) and 0 not in short[0]
