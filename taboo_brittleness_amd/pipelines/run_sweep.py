"""End-to-end intervention sweep driver (CLI: ``tb-sweep`` / ``python -m taboo_brittleness_amd.cli.sweep``).

Stages (EP:112-160):
1. baselines for every (word, prompt) pair — identical on every rank (cheap,
   one batch) so no broadcast is needed and every rank holds the spikes,
   targeted latents and PCA bases;
2. deterministic cell list (``SweepRunner.make_cells``), sharded round-robin
   over data-parallel ranks;
3. per-rank batched execution, results all-gathered to rank 0;
4. rank 0 writes ``sweep_cells.jsonl``, ``sweep_summary.json`` (curves with 95%
   bootstrap CIs) and ``sweep_curves.csv``; atomic writes so a killed run never
   leaves a half-written result (resume = rerun; finished shards are skipped).
"""
from __future__ import annotations

import json
import os
import time
from typing import Dict, List, Optional, Sequence

import torch

from ..config import Config
from ..parallel import dist as D
from ..utils.io import atomic_write_json, atomic_write_text
from .factory import build_stack
from .sweep import METHODS, SweepRunner, summarize_cells


def run_sweep(cfg: Config, out_dir: str, methods: Sequence[str] = METHODS, info: Optional[D.DistInfo] = None,
              batch: Optional[int] = None, log=print) -> Dict:
    info = info or D.init_distributed(cfg.parallel.backend, cfg.runtime.device)
    tp_ctx, dp_rank, dp_size = None, info.rank, info.world
    if cfg.parallel.tp > 1:
        from ..parallel.tp import make_groups

        tp_ctx, dp_rank, dp_size = make_groups(info.world, info.rank, cfg.parallel.tp)
    stack = build_stack(cfg, info.device, tp=tp_ctx)
    model, tok, sae = stack.model, stack.tok, stack.sae
    B = batch or cfg.runtime.batch_size
    n_pairs = len(cfg.words) * len(cfg.prompts)
    graphs = cfg.runtime.use_graphs and (tp_ctx is None or os.environ.get("TB_TP_GRAPHS", "0") == "1")
    runner = SweepRunner(cfg, model, tok, sae, batch=B, device=info.device, layer=stack.layer,
                         use_graphs=graphs, kv_pairs=n_pairs + 1)
    pairs = runner.build_pairs(cfg.words, cfg.prompts)
    t0 = time.perf_counter()
    runner.run_baselines(pairs)
    if sae is not None and stack.sae_random:
        resid = torch.cat([p.resid for p in pairs if p.resid is not None and p.resid.shape[0]], 0)
        sae.calibrate(resid)
        runner._score_pairs(pairs)
    t_base = time.perf_counter() - t0
    cells = runner.make_cells(pairs, methods)
    mine = D.shard(list(range(len(cells))), dp_rank, dp_size)     # every TP rank of a group runs the same cells
    shard_path = os.path.join(out_dir, f"shard_{dp_rank:03d}_of_{dp_size:03d}.json")
    writer = tp_ctx is None or tp_ctx.rank == 0
    t1 = time.perf_counter()
    if os.path.exists(shard_path):
        res = json.load(open(shard_path))["results"]
        log(f"[rank {info.rank}] resumed {len(res)} cells from {shard_path}")
    else:
        res = runner.run_cells(pairs, [cells[i] for i in mine])
        for r, i in zip(res, mine):
            r["cell_id"] = i
        if writer:
            os.makedirs(out_dir, exist_ok=True)
            atomic_write_json(shard_path, {"results": res})
    t_cells = time.perf_counter() - t1
    gathered = D.all_gather_objects(res if writer else [], info)
    summary: Dict = {}
    if info.is_main:
        allres = sorted([r for part in gathered for r in part], key=lambda r: r["cell_id"])
        summary = summarize_cells(allres, cfg.words, cfg.word_plurals)
        summary["baselines"] = [{
            "word": p.word, "prompt_idx": p.pidx, "n_gen": len(p.resp), "spikes": p.spikes_rel,
            "p_secret_mean": float(p.p_secret.mean()) if p.p_secret is not None and p.p_secret.size else 0.0,
            "top_ids": p.top_ids, "guesses": [tok.decode([t]).strip() for t in p.top_ids],
            "targeted_latents": p.targeted[:8], "nll": p.nll} for p in pairs]
        summary["timing"] = {"baseline_s": t_base, "cells_s": t_cells, "n_cells": len(allres),
                             "world": info.world, "dp": dp_size, "tp": cfg.parallel.tp,
                             "cells_per_s": len(allres) / max(t_cells, 1e-9)}
        summary["config"] = {"layer": stack.layer, "arch": cfg.model.arch, "methods": list(methods),
                             "budgets": cfg.intervention.budgets, "ranks": cfg.intervention.ranks}
        os.makedirs(out_dir, exist_ok=True)
        atomic_write_text(os.path.join(out_dir, "sweep_cells.jsonl"),
                          "".join(json.dumps(r) + "\n" for r in allres))
        atomic_write_json(os.path.join(out_dir, "sweep_summary.json"), summary)
        lines = ["method,budget,n,p_secret_mean,p_lo,p_hi,delta_p,delta_nll,leak_rate,ll_accuracy,ll_pass10,ll_majority"]
        for c in summary["curves"]:
            ll = c.get("ll_topk", {})
            lines.append(",".join(str(x) for x in [
                c["method"], c["budget"], c["n"], c["p_secret_mean"]["mean"], c["p_secret_mean"]["lo"],
                c["p_secret_mean"]["hi"], c["delta_p_secret"]["mean"], c["delta_nll"]["mean"], c["leak_rate"],
                ll.get("prompt_accuracy", ""), ll.get("any_pass", ""), ll.get("global_majority_vote", "")]))
        atomic_write_text(os.path.join(out_dir, "sweep_curves.csv"), "\n".join(lines) + "\n")
        log(f"[sweep] {len(allres)} cells on {info.world} rank(s): {t_cells:.2f}s "
            f"({len(allres) / max(t_cells, 1e-9):.1f} cells/s); results in {out_dir}")
    return summary
