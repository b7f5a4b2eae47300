"""Subprocess probe for ``TB_DEBUG_CHECKS=1`` (host-side index-range checks in csrc/bindings.cpp, read once per
process): a small GPU sweep must pass them, and an out-of-range latent index must be rejected by
``lowrank_edit``'s check before any kernel reads past the SAE tables.  Prints one JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from taboo_brittleness_amd import ops  # noqa: E402


def main():
    assert os.environ.get("TB_DEBUG_CHECKS") == "1"
    dev = torch.device("cuda:0")
    from dataclasses import replace

    from taboo_brittleness_amd.config import load_config
    from taboo_brittleness_amd.interp.sae import JumpReLUSAE
    from taboo_brittleness_amd.models.gemma2 import Gemma2Model
    from taboo_brittleness_amd.models.spec import GEMMA2_TINY
    from taboo_brittleness_amd.models.tokenizer import SyntheticTokenizer
    from taboo_brittleness_amd.models.weights import random_gemma2
    from taboo_brittleness_amd.pipelines.sweep import SweepRunner

    spec = replace(GEMMA2_TINY, vocab_size=2048, layers=4, sliding_window=8)
    m = Gemma2Model(random_gemma2(spec, dtype=torch.bfloat16, seed=5, norm_std=0.1, post_norm_gain=8.0, device=dev), dev)
    cfg = load_config(None, ["experiment.max_new_tokens=8", "intervention.budgets=[1, 4]", "intervention.random_trials=2"])
    sae = JumpReLUSAE.random(spec.hidden, 1024, seed=2, device=dev)
    r = SweepRunner(cfg, m, SyntheticTokenizer(vocab_size=spec.vocab_size), sae, batch=48, device=dev, layer=2,
                    kv_pairs=4)
    pairs = r.build_pairs(["ship"], cfg.prompts[:2])
    r.run_baselines(pairs)
    res = r.run_cells(pairs, r.make_cells(pairs, ("sae_targeted", "sae_random")))
    torch.cuda.synchronize()
    # an out-of-range latent id (>= d_sae) in the edit plan: the debug check must refuse the launch
    h = torch.randn(4, spec.hidden, device=dev).to(torch.bfloat16)
    idx = torch.tensor([[5, 2000]] * 4, dtype=torch.int32, device=dev)
    rejected = False
    try:
        ops.lowrank_edit(h, torch.ones(4, dtype=torch.uint8, device=dev), idx,
                         torch.full((4,), 2, dtype=torch.int32, device=dev), sae.W_encT, sae.W_dec, sae.b_enc,
                         sae.threshold, None, 1.0, None, 1e-6, None, None)
        torch.cuda.synchronize()
    except RuntimeError as e:
        rejected = "out of range" in str(e)
    print(json.dumps({"cells": len(res), "rejected_out_of_range": rejected}))


if __name__ == "__main__":
    main()
