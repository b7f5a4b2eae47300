"""Tiny end-to-end smoke of the flagship path (used by ``__graft_entry__.smoke``).

One hooked greedy decode with an SAE-latent ablation at the hooked layer,
then the logit-lens readout and a teacher-forced NLL — every step on the HIP
kernels when ``device`` is a GPU.
"""
from __future__ import annotations

import torch

from .config import Config
from .interp.sae import JumpReLUSAE
from .models.gemma2 import Gemma2Model
from .models.spec import get_spec
from .models.tokenizer import SyntheticTokenizer
from .models.weights import random_gemma2
from .pipelines.sweep import SweepRunner


def run_smoke(device, arch: str = "gemma2-tiny", max_new: int = 8) -> dict:
    spec = get_spec(arch)
    cfg = Config()
    cfg.experiment.max_new_tokens = max_new
    cfg.intervention.budgets = [1, 4]
    cfg.intervention.random_trials = 1
    cfg.intervention.ranks = [1, 2]
    cfg.intervention.proj_random_trials = 1
    w = random_gemma2(spec, device=device, seed=3)
    m = Gemma2Model(w, device)
    tok = SyntheticTokenizer(vocab_size=spec.vocab_size)
    sae = JumpReLUSAE.random(spec.hidden, 2048, seed=1, device=device)
    layer = spec.layers // 2
    r = SweepRunner(cfg, m, tok, sae, batch=16, device=device, layer=layer)
    pairs = r.build_pairs(["ship"], cfg.prompts[:2])
    r.run_baselines(pairs)
    sae.calibrate(torch.cat([p.resid for p in pairs], 0), target_l0=20)
    r._score_pairs(pairs)
    cells = r.make_cells(pairs)
    res = r.run_cells(pairs, cells)
    if device.type == "cuda":
        torch.cuda.synchronize()
    assert len(res) == len(cells) and all(x["n_gen"] >= 0 for x in res)
    return {"cells": len(res), "p_secret_mean": sum(x["p_secret_mean"] for x in res) / len(res),
            "delta_nll_finite": all(x["delta_nll"] == x["delta_nll"] for x in res)}
