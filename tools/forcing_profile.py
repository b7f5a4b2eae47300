"""The bench's post-edit forcing side measurement on its own (Gemma-2-9B random init, synthetic tokenizer, random
SAE): ``--settings`` SAE-ablation settings over the config's words, each generating the 3 postgame warm-up turns
and the 10 prefilled answers under its edit (pipelines/token_forcing.py run_forcing_settings).  One warm call, then
``--reps`` timed calls; prints the phase timings of each.  For a kernel census run it under
``rocprofv3 --kernel-trace --stats -- python tools/forcing_profile.py``.

  python tools/forcing_profile.py [--settings 201] [--reps 1]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from taboo_brittleness_amd.config import Config  # noqa: E402
from taboo_brittleness_amd.interp.sae import JumpReLUSAE  # noqa: E402
from taboo_brittleness_amd.models.gemma2 import Gemma2Model  # noqa: E402
from taboo_brittleness_amd.models.spec import GEMMA2_9B  # noqa: E402
from taboo_brittleness_amd.models.tokenizer import SyntheticTokenizer  # noqa: E402
from taboo_brittleness_amd.models.weights import random_gemma2  # noqa: E402
from taboo_brittleness_amd.pipelines import token_forcing as TF  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--settings", type=int, default=201)
    ap.add_argument("--reps", type=int, default=1)
    ap.add_argument("--init-gain", type=float, default=32.0)
    ap.add_argument("--chunk-rows", type=int, default=None,
                    help="run_forcing_settings chunk_rows (generator rows; default: sized to free memory)")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    cfg = Config()
    spec = GEMMA2_9B
    model = Gemma2Model(random_gemma2(spec, device=dev, dtype=torch.bfloat16, seed=1234,
                                      post_norm_gain=args.init_gain), dev)
    tok = SyntheticTokenizer(vocab_size=spec.vocab_size)
    sae = JumpReLUSAE.random(spec.hidden, cfg.sae.d_sae, seed=7, device=dev)
    layer = min(cfg.model.layer_idx, spec.layers - 1)
    rng = np.random.default_rng(0)
    words = list(cfg.words)
    settings = []
    for i in range(args.settings):
        w = words[i % len(words)]
        if i < len(words):
            settings.append({"word": w, "kind": "none"})
        else:
            m = int(rng.choice([1, 2, 4, 8, 16]))
            settings.append({"word": w, "kind": "sae", "alpha": 1.0,
                             "latents": sorted(rng.choice(cfg.sae.d_sae, m, replace=False).tolist())})
    TF.run_forcing_settings(cfg, model, tok, settings, "postgame", sae, layer, chunk_rows=args.chunk_rows)
    torch.cuda.synchronize()
    for r in range(args.reps):
        t0 = time.perf_counter()
        TF.run_forcing_settings(cfg, model, tok, settings, "postgame", sae, layer, chunk_rows=args.chunk_rows)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(json.dumps({"rep": r, "chunk_rows": args.chunk_rows, "settings": len(settings),
                          "peak_gb": round(torch.cuda.max_memory_reserved() / 1e9, 1), "seconds": round(dt, 3),
                          "settings_per_s": round(len(settings) / dt, 2), "phases_s": dict(TF.LAST_TIMINGS)}),
              flush=True)


if __name__ == "__main__":
    main()
