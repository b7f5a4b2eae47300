"""Debug probe for tests/test_exact_9b_gpu.py: where do the fast (reuse levels) and from-scratch sweeps' NLLs part?
Compares the baselines' per-token NLLs / lens probabilities / residuals across batch compositions, then per-token
teacher-forced NLLs of a few cells in both paths."""
import json
import sys

import numpy as np
import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__)))))
from taboo_brittleness_amd.config import load_config  # noqa: E402
from taboo_brittleness_amd.interp.sae import JumpReLUSAE  # noqa: E402
from taboo_brittleness_amd.models.gemma2 import Gemma2Model  # noqa: E402
from taboo_brittleness_amd.models.spec import GEMMA2_9B  # noqa: E402
from taboo_brittleness_amd.models.tokenizer import SyntheticTokenizer  # noqa: E402
from taboo_brittleness_amd.models.weights import random_gemma2  # noqa: E402
from taboo_brittleness_amd.pipelines.sweep import SweepRunner  # noqa: E402
from taboo_brittleness_amd.runtime import gemm_dispatch as GD  # noqa: E402

gpu = torch.device("cuda:0")
GD.set_mode("tb")
GD.load_table()
cfg = load_config(None, [])
m = Gemma2Model(random_gemma2(GEMMA2_9B, device=gpu, dtype=torch.bfloat16, seed=1234, post_norm_gain=32.0), gpu)
tok = SyntheticTokenizer(vocab_size=GEMMA2_9B.vocab_size)
sae = JumpReLUSAE.random(GEMMA2_9B.hidden, cfg.sae.d_sae, seed=7, device=gpu)
rep = {}


def runner(batch, share, resume, graphs):
    r = SweepRunner(cfg, m, tok, sae, batch=batch, device=gpu, layer=31, use_graphs=graphs, prefix_share=share,
                    layer_resume=resume, kv_pairs=8)
    return r


ra = runner(150, True, True, True)
pa = ra.build_pairs(["ship", "moon"], cfg.prompts[:2])
ra.run_baselines(pa[:2])
rb = runner(97, False, False, False)
pb = rb.build_pairs(["ship", "moon"], cfg.prompts[:2])
rb.run_baselines(pb)
for i in range(2):
    a, b = pa[i], pb[i]
    rep[f"base{i}"] = {
        "n": len(a.resp), "gen_eq": a.gen_toks == b.gen_toks,
        "tok_nll_eq": bool(np.array_equal(a.tok_nll, b.tok_nll)),
        "tok_nll_maxdiff": float(np.abs(a.tok_nll - b.tok_nll).max()) if a.tok_nll.shape == b.tok_nll.shape else None,
        "nll": [a.nll, b.nll],
        "p_secret_eq": bool(np.array_equal(a.p_secret, b.p_secret)),
        "resid_eq": bool(torch.equal(a.resid, b.resid)),
        "tok_nll_a": a.tok_nll[:8].tolist(), "tok_nll_b": b.tok_nll[:8].tolist(),
    }
print(json.dumps(rep), flush=True)
# cells of pair 0, both paths (same calibrated SAE)
sae.calibrate(torch.cat([p.resid for p in pa[:2]], 0))
ra._score_pairs(pa[:2])
rb._score_pairs(pb)
methods = ("sae_targeted", "sae_random")
ca = ra.make_cells(pa[:1], methods)
cb = rb.make_cells(pb[:1], methods)
resa = ra.run_cells(pa[:1], ca)
resb = rb.run_cells(pb[:1], cb)
diffs = []
for x, y in zip(resa, resb):
    diffs.append({"key": [x["method"], x["budget"], x["trial"]], "resp_eq": x["response_ids"] == y["response_ids"],
                  "n": x["n_gen"], "nll_edit": [x["nll_edit"], y["nll_edit"]], "nll_self": [x["nll_self"], y["nll_self"]],
                  "p_mean": [x["p_secret_mean"], y["p_secret_mean"]], "base_nll": [x["nll_base"], y["nll_base"]]})
print(json.dumps({"cells": diffs[:12], "n_bad_nll": sum(d["nll_edit"][0] != d["nll_edit"][1] for d in diffs),
                  "n_bad_p": sum(d["p_mean"][0] != d["p_mean"][1] for d in diffs)}), flush=True)
