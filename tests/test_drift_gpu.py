"""How far the headline configuration's GEMM dispatch (``TB_GEMM=auto``: hipBLASLt / split-K where measured faster) moves
the sweep's results away from the batch-invariant in-tree mode (``tb``), at the real Gemma-2-9B shapes.

In ``tb`` mode every GEMM accumulates each output over K in one fixed order whatever the batch, so the reuse levels
(layer resume, trie decode, lens dedup, no-op skip) are exact.  ``auto`` picks per row count between kernels whose
K summation orders differ, so a row's bf16 result can depend on the batch it runs in.  This test runs the same
sweep (full 42-layer random-init Gemma-2-9B, SAE ablation at block 31, the bench's init) in both modes and
reports the fraction of baseline and cell responses that differ and the spread of the edit NLLs
(``gpurun_out/drift_9b.json`` when ``TB_DRIFT_OUT`` is set; README "Exactness of the headline configuration").
It asserts the runs are complete and finite and that the drift stays below a loose bound; the numbers are the point.
"""
import json
import os

import numpy as np
import pytest
import torch

from taboo_brittleness_amd.config import load_config
from taboo_brittleness_amd.interp.sae import JumpReLUSAE
from taboo_brittleness_amd.models.gemma2 import Gemma2Model
from taboo_brittleness_amd.models.spec import GEMMA2_9B
from taboo_brittleness_amd.models.tokenizer import SyntheticTokenizer
from taboo_brittleness_amd.models.weights import random_gemma2
from taboo_brittleness_amd.pipelines.sweep import SweepRunner
from taboo_brittleness_amd.runtime import gemm_dispatch as GD

pytestmark = pytest.mark.gpu


def test_auto_vs_tb_drift_9b(gpu):
    cfg = load_config(None, ["experiment.max_new_tokens=24", "intervention.budgets=[1, 4, 16]",
                             "intervention.random_trials=2"])
    spec = GEMMA2_9B
    model = Gemma2Model(random_gemma2(spec, device=gpu, dtype=torch.bfloat16, seed=1234, post_norm_gain=32.0), gpu)
    tok = SyntheticTokenizer(vocab_size=spec.vocab_size)
    words, prompts = list(cfg.words[:5]), list(cfg.prompts[:4])
    key = lambda r: (r["word"], r["prompt_idx"], r["method"], r["budget"], r["trial"])   # noqa: E731
    out, base = {}, {}
    old = GD.mode()
    try:
        for mode in ("tb", "auto"):
            GD.set_mode(mode)
            sae = JumpReLUSAE.random(spec.hidden, cfg.sae.d_sae, seed=7, device=gpu)
            n_cells = len(cfg.intervention.budgets) * (1 + cfg.intervention.random_trials) * 2
            r = SweepRunner(cfg, model, tok, sae, batch=len(words) * len(prompts) * (n_cells + 1) + 8, device=gpu,
                            layer=cfg.model.layer_idx, use_graphs=False)
            pairs = r.build_pairs(words, prompts)
            r.run_baselines(pairs)
            sae.calibrate(torch.cat([p.resid for p in pairs if p.resid is not None and p.resid.shape[0]], 0))
            res = r.run_cells(pairs, r.make_cells(pairs))
            out[mode] = {key(x): x for x in res}
            base[mode] = {(p.word, p.pidx): list(p.gen_toks) for p in pairs}
    finally:
        GD.set_mode(old)
    assert set(out["tb"]) == set(out["auto"]) and len(out["tb"]) > 0
    kb = list(base["tb"])
    base_diff = float(np.mean([base["tb"][k] != base["auto"][k] for k in kb]))
    # cells of pairs whose baselines agree: the edit's own drift
    ks = [k for k in out["tb"] if base["tb"][(k[0], k[1])] == base["auto"][(k[0], k[1])]]
    cell_diff = float(np.mean([out["tb"][k]["response_ids"] != out["auto"][k]["response_ids"] for k in ks])) \
        if ks else float("nan")
    all_diff = float(np.mean([out["tb"][k]["response_ids"] != out["auto"][k]["response_ids"] for k in out["tb"]]))
    dn = np.asarray([abs(out["tb"][k]["nll_edit"] - out["auto"][k]["nll_edit"]) for k in out["tb"]], np.float64)
    leak = float(np.mean([out["tb"][k]["leak"] != out["auto"][k]["leak"] for k in out["tb"]]))
    rep = {"pairs": len(kb), "cells": len(out["tb"]), "baseline_response_mismatch": base_diff,
           "cell_response_mismatch_given_equal_baseline": cell_diff, "cell_response_mismatch_all": all_diff,
           "leak_verdict_mismatch": leak, "nll_edit_absdiff_median": float(np.median(dn)),
           "nll_edit_absdiff_p95": float(np.percentile(dn, 95)), "gemm_table": GD.describe()["table"]}
    print("DRIFT", json.dumps(rep))
    if os.environ.get("TB_DRIFT_OUT"):
        with open(os.environ["TB_DRIFT_OUT"], "w") as f:
            json.dump(rep, f, indent=1)
    assert np.isfinite(dn).all()
    # bounds from the recorded run (profiles/r4/drift_9b.json: 0.50 / 0.33 / p95 0.24 nats) with a margin for table
    # re-tunes: a numerics regression in auto (e.g. a wrong split-K reduction) flips far more tokens than this.
    # Leak-verdict parity is unpinned: the random model almost never emits the secret, so 0 mismatches says little.
    assert base_diff <= 0.75 and (cell_diff != cell_diff or cell_diff <= 0.6) and all_diff < 0.9, rep
    assert float(np.percentile(dn, 95)) <= 0.6, rep
