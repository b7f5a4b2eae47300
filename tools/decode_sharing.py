"""How much of the diverged cells' full-model decode is shared work?

Blocks 0..l (l = hooked layer) of a row depend only on its token sequence: the edit writes the residual
*after* block l, so the KV of blocks <= l is a function of the tokens alone.  Two diverged cells of the same
(word, prompt) pair whose generated tokens are equal up to position t therefore compute identical blocks
0..l at t.  This tool runs one bench-shaped batch (P pairs x 66 cells, Gemma-2-9B random init, gain 32) and
reports, over every decode row-step of the diverged cells, the number of distinct (pair, token prefix)
keys -- i.e. the blocks-0..l row count a trie-shared decode would run -- against the row count it runs now.

    python tools/decode_sharing.py [--pairs 90]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from taboo_brittleness_amd.config import Config  # noqa: E402
from taboo_brittleness_amd.interp.sae import JumpReLUSAE  # noqa: E402
from taboo_brittleness_amd.models.gemma2 import Gemma2Model  # noqa: E402
from taboo_brittleness_amd.models.spec import get_spec  # noqa: E402
from taboo_brittleness_amd.models.tokenizer import SyntheticTokenizer  # noqa: E402
from taboo_brittleness_amd.models.weights import random_gemma2  # noqa: E402
from taboo_brittleness_amd.pipelines.sweep import SweepRunner  # noqa: E402


def sharing(pairs, cells, records, max_new):
    """Row-steps of the diverged cells' decode vs distinct (pair, prefix) keys, per decode position."""
    rows = uniq = 0
    per_t = {}
    by_pair = {}
    for c, r in zip(cells, records):
        by_pair.setdefault(c.pair, []).append(r["response_ids"])
    for pi, resps in by_pair.items():
        base = list(pairs[pi].resp)
        live = []
        for resp in resps:
            d = next((i for i, (a, b) in enumerate(zip(resp, base)) if a != b), None)
            if d is None and len(resp) != len(base):
                d = min(len(resp), len(base))
            if d is None:
                continue
            live.append((d, list(resp)))
        for t in range(max_new):
            keys = {tuple(resp[: t + 1]) for d, resp in live if d <= t < len(resp)}
            n = sum(1 for d, resp in live if d <= t < max_new)
            rows += n
            uniq += len(keys) + sum(1 for d, resp in live if d <= t < max_new and t >= len(resp))
            a = per_t.setdefault(t, [0, 0])
            a[0] += n
            a[1] += len(keys)
    return rows, uniq, per_t


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=90)
    ap.add_argument("--max-new", type=int, default=50)
    ap.add_argument("--arch", default="gemma2-9b")
    args = ap.parse_args()
    dev = torch.device("cuda:0" if torch.cuda.is_available() else "cpu")
    spec = get_spec(args.arch)
    cfg = Config()
    cfg.experiment.max_new_tokens = args.max_new
    P = args.pairs
    bench.enable_tuned_gemms(f"{spec.name}_P{P}_E4_new{args.max_new}")
    layer = min(cfg.model.layer_idx, spec.layers - 1)
    weights = random_gemma2(spec, device=dev, dtype=torch.bfloat16, seed=1234, post_norm_gain=32.0)
    model = Gemma2Model(weights, dev)
    tok = SyntheticTokenizer(vocab_size=spec.vocab_size)
    sae = JumpReLUSAE.random(spec.hidden, cfg.sae.d_sae, seed=7, device=dev)
    n_cells = len(cfg.intervention.budgets) * (1 + cfg.intervention.random_trials)
    runner = SweepRunner(cfg, model, tok, sae, batch=P * n_cells + P, device=dev, layer=layer, use_graphs=True,
                         prefix_share=True, kv_pairs=2 * P + 2, layer_resume=True)
    templates = runner.build_pairs(cfg.words, cfg.prompts)
    pairs = [bench.fresh(templates[j % len(templates)], rep=j // len(templates)) for j in range(P)]
    runner.run_baselines(pairs)
    resid = torch.cat([p.resid for p in pairs if p.resid is not None and p.resid.shape[0]], 0)
    sae.calibrate(resid)
    runner._score_pairs(pairs)
    cells = runner.make_cells(pairs, ("sae_targeted", "sae_random"))
    recs = runner.run_cells(pairs, cells)
    assert len(recs) == len(cells)
    for c, r in zip(cells, recs):
        assert (r["method"], r["budget"], r["trial"]) == (c.method, c.budget, c.trial)
    rows, uniq, per_t = sharing(pairs, cells, recs, args.max_new)
    out = {"pairs": P, "cells": len(cells), "decode_row_steps": rows, "distinct_prefix_row_steps": uniq,
           "shared_ratio": round(uniq / max(1, rows), 4),
           "per_position": {t: v for t, v in sorted(per_t.items()) if v[0]}}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
