"""End-to-end intervention sweep driver (CLI: ``tb-sweep`` / ``python -m taboo_brittleness_amd.cli.sweep``).

Stages (EP:112-160):
1. baselines of the (word, prompt) pairs a data-parallel group owns (contiguous
   blocks of pairs, :func:`pair_owners`), then one object all-gather of the small
   per-pair results so every rank holds every pair's spikes, targeted latents
   and PCA inputs;
2. deterministic cell list (``SweepRunner.make_cells``); each pair's cells run
   on its owner group;
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

        tp_ctx, dp_rank, dp_size = make_groups(info.world, info.rank, cfg.parallel.tp,
                                                 cfg.parallel.tp_allreduce, info.device,
                                                 vocab_parallel=cfg.parallel.vocab_parallel)
    stack = build_stack(cfg, info.device, tp=tp_ctx)
    model, tok, sae = stack.model, stack.tok, stack.sae
    B = batch or cfg.runtime.batch_size
    n_pairs = len(cfg.words) * len(cfg.prompts)
    # decode hipGraphs under TP: on with the one-shot P2P all-reduce (device-side call counters: replay-safe,
    # tests/test_p2p_gpu.py); with RCCL only on request (TB_TP_GRAPHS=1)
    tp_graphs = os.environ.get("TB_TP_GRAPHS", "auto")
    graphs = cfg.runtime.use_graphs and (tp_ctx is None or tp_graphs == "1" or
                                         (tp_graphs == "auto" and getattr(tp_ctx, "p2p", None) is not None))
    runner = SweepRunner(cfg, model, tok, sae, batch=B, device=info.device, layer=stack.layer,
                         use_graphs=graphs, kv_pairs=n_pairs + 1)
    pairs = runner.build_pairs(cfg.words, cfg.prompts)
    # work placement by PAIR (the reference's unit of work, `src/run_generation.py:155-156`): a pair's baseline
    # and all of its cells run on one DP group, so every reuse level that works within a pair (prefix-trie
    # decode groups, lens row dedup, the pair's KV / residual prefix) is as large as on one GPU
    owned = pair_owners(len(pairs), dp_size)[dp_rank]
    t0 = time.perf_counter()
    runner.run_baselines([pairs[i] for i in owned], size_for=pairs)
    if dp_size > 1:
        # the cross-pair inputs (pooled PCA / gradient subspaces, SAE calibration, word-averaged scores) need
        # every pair's baseline: one object all-gather of the small per-pair results + kept residuals
        share_baselines(pairs, owned, info, runner.dev)
    if sae is not None and stack.sae_random:
        resid = torch.cat([p.resid for p in pairs if p.resid is not None and p.resid.shape[0]], 0)
        sae.calibrate(resid)
    # scores over ALL pairs at once (identical on every rank and for every world size; score_over=word then
    # averages over all of a word's prompts, not over one baseline batch)
    runner._score_pairs(pairs)
    t_base = time.perf_counter() - t0
    _check_comm(tp_ctx, None, "baselines")
    cells = runner.make_cells(pairs, methods)
    own = set(owned)
    mine = [i for i, c in enumerate(cells) if c.pair in own]     # every TP rank of a group runs the same cells
    shard_path = os.path.join(out_dir, f"shard_{dp_rank:03d}_of_{dp_size:03d}.json")
    writer = tp_ctx is None or tp_ctx.rank == 0
    elog = EventLog(os.path.join(out_dir, f"log_rank{info.rank:03d}.jsonl") if writer else None)
    elog.write("baselines", pairs=len(pairs), seconds=round(t_base, 4))
    t1 = time.perf_counter()
    if os.path.exists(shard_path):
        res = json.load(open(shard_path))["results"]
        log(f"[rank {info.rank}] resumed {len(res)} cells from {shard_path}")
        elog.write("resumed_shard", cells=len(res))
    else:
        res = _run_parts(runner, pairs, cells, mine, out_dir, dp_rank, dp_size, writer, B, elog, log,
                         tp_ctx=tp_ctx)
        _check_comm(tp_ctx, elog, "shard")
        if writer:
            os.makedirs(out_dir, exist_ok=True)
            atomic_write_json(shard_path, {"results": res})
    t_cells = time.perf_counter() - t1
    elog.write("cells_done", cells=len(res), seconds=round(t_cells, 4),
               cells_per_s=round(len(res) / max(t_cells, 1e-9), 3))
    gathered = D.all_gather_objects(res if writer else [], info)
    forcing = None
    if cfg.intervention.measure_forcing:
        # every rank takes part: settings are sharded over the DP groups and every TP rank of a group runs the
        # same forwards (its peers' all-reduces would otherwise never be matched)
        from .token_forcing import DPShard

        forcing = forcing_curves(cfg, runner, pairs, methods, stack, log if info.is_main else (lambda *a: None),
                                 dp=DPShard(dp_rank, dp_size, info))
        _check_comm(tp_ctx, elog, "forcing")
    summary: Dict = {} if forcing is None else {"forcing": forcing}   # every rank holds the gathered curves
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
                             "budgets": cfg.intervention.budgets, "ranks": cfg.intervention.ranks,
                             "subspace": cfg.intervention.subspace, "pca_pool": cfg.intervention.pca_pool}
        if forcing is not None:
            summary["forcing"] = forcing
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
        if summary.get("forcing"):
            fl = ["method,budget,n_settings,forcing_success,delta_vs_unedited"]
            fl += [f"{c['method']},{c['budget']},{c['n_settings']},{c['success_rate']},{c['delta']}"
                   for c in summary["forcing"]["curves"]]
            atomic_write_text(os.path.join(out_dir, "forcing_curves.csv"), "\n".join(fl) + "\n")
        log(f"[sweep] {len(allres)} cells on {info.world} rank(s): {t_cells:.2f}s "
            f"({len(allres) / max(t_cells, 1e-9):.1f} cells/s); results in {out_dir}")
    return summary


def pair_owners(n_pairs: int, dp: int) -> List[List[int]]:
    """Pairs of each DP group: contiguous blocks balanced to within one pair (every pair has the same cell
    count, so cell counts balance to within one pair's cells).  Contiguous keeps a word's prompts together,
    which keeps the per-word pooled inputs mostly rank-local."""
    q, r = divmod(n_pairs, dp)
    out, s = [], 0
    for g in range(dp):
        n = q + (1 if g < r else 0)
        out.append(list(range(s, s + n)))
        s += n
    return out


_SHARED_FIELDS = ("resp", "p_secret", "spikes_rel", "top_ids", "nll", "gen_toks", "tok_nll", "track_probs")


def share_baselines(pairs, owned: Sequence[int], info: D.DistInfo, dev) -> None:
    """All-gather the owned pairs' baseline results (responses, lens probabilities, spikes, NLLs and the kept
    hooked-layer residuals, which the pooled subspaces / calibration / scores read) and fill them into the
    pairs other groups own.  TP peers send identical copies; the first one wins."""
    local = {}
    for i in owned:
        p = pairs[i]
        rec = {f: getattr(p, f) for f in _SHARED_FIELDS}
        rec["resid"] = p.resid.detach().cpu() if p.resid is not None else None
        pre = getattr(p, "resid_pre", None)
        rec["resid_pre"] = pre.detach().cpu() if pre is not None else None
        local[i] = rec
    got: Dict[int, dict] = {}
    for part in D.all_gather_objects(local, info):
        for k, v in part.items():
            got.setdefault(k, v)
    mine = set(owned)
    for i, rec in got.items():
        if i in mine:
            continue
        p = pairs[i]
        for f in _SHARED_FIELDS:
            setattr(p, f, rec[f])
        p.resid = rec["resid"].to(dev) if rec["resid"] is not None else None
        if rec["resid_pre"] is not None:
            p.resid_pre = rec["resid_pre"].to(dev)


def forcing_curves(cfg: Config, runner: SweepRunner, pairs, methods: Sequence[str], stack, log=print,
                   dp=None) -> Dict:
    """Post-edit token forcing (EP:100-104, 132-138): per (method, budget), the postgame forcing success
    under the edit applied at every position, vs the unedited model — the "inhibition" axis of the
    content-vs-inhibition analysis (EP:160, fig3).  All settings × words × phrases run batched."""
    import numpy as np

    from ..interp import analysis as A
    from .sweep import word_targeted_latents
    from .token_forcing import run_forcing_settings

    iv = cfg.intervention
    bases = runner._bases(pairs) if any(m.startswith("proj") for m in methods) else {}
    settings, keys = [], []
    for w in cfg.words:
        settings.append({"word": w, "kind": "none"})
        keys.append(("none", 0))
        pool = np.unique(np.concatenate([np.zeros(0, dtype=np.int64)] + [p.active_pool for p in pairs if p.word == w]))
        for meth in methods:
            if meth.startswith("sae"):
                if runner.sae is None:
                    continue
                for m in iv.budgets:
                    tl = word_targeted_latents(runner, w, m)
                    trials = 1 if meth == "sae_targeted" else max(1, iv.forcing_trials or iv.random_trials)
                    for t in range(trials):
                        lat = tl if meth == "sae_targeted" else A.random_latents(
                            runner.sae.d_sae, m, A.cell_seed("forcing", w, meth, m, t), exclude=tl, pool=pool)
                        settings.append({"word": w, "kind": "sae", "latents": lat, "alpha": iv.alpha})
                        keys.append((meth, m))
            else:
                key = w if iv.pca_pool == "word" else "__all__"
                for r in iv.ranks:
                    trials = 1 if meth == "proj_targeted" else max(1, iv.forcing_trials or iv.proj_random_trials)
                    for t in range(trials):
                        U = bases[key][:r] if meth == "proj_targeted" and key in bases else \
                            A.random_subspace(runner.D, r, A.cell_seed("forcing", w, meth, r, t), device=runner.dev)
                        settings.append({"word": w, "kind": "proj", "basis": U.to(runner.dev)})
                        keys.append((meth, r))
    res = run_forcing_settings(cfg, stack.model, stack.tok, settings, "postgame", stack.sae, stack.layer, dp=dp)
    base = float(np.mean([r["success_rate"] for r, k in zip(res, keys) if k[0] == "none"]))
    groups: Dict = {}
    for r, k in zip(res, keys):
        if k[0] != "none":
            groups.setdefault(k, []).append(r["success_rate"])
    curves = [{"method": m, "budget": b, "n_settings": len(v), "success_rate": float(np.mean(v)),
               "delta": float(np.mean(v)) - base} for (m, b), v in sorted(groups.items())]
    log(f"[sweep] post-edit token forcing: {len(settings)} settings, unedited success {base:.3f}")
    return {"mode": "postgame", "baseline_success": base, "curves": curves}


class EventLog:
    """Structured per-rank JSONL event log (observability: stage timings, progress, throughput)."""

    def __init__(self, path: Optional[str]):
        self.path = path
        if path:
            os.makedirs(os.path.dirname(path), exist_ok=True)

    def write(self, event: str, **kw) -> None:
        if not self.path:
            return
        with open(self.path, "a") as f:
            f.write(json.dumps({"t": round(time.time(), 3), "event": event, **kw}) + "\n")


def _check_comm(tp_ctx, elog: Optional[EventLog], where: str) -> None:
    """Fail the run (non-zero exit) if the one-shot P2P all-reduce timed out on a peer barrier since the
    last check: its output then summed stale data, so nothing computed after it may be committed."""
    p2p = getattr(tp_ctx, "p2p", None) if tp_ctx is not None else None
    if p2p is None:
        return
    try:
        p2p.check()
    except RuntimeError as e:
        if elog is not None:
            elog.write("comm_error", where=where, error=str(e))
        raise


def _run_parts(runner, pairs, cells, mine: List[int], out_dir: str, dp_rank: int, dp_size: int, writer: bool,
               chunk: int, elog: EventLog, log, tp_ctx=None) -> List[dict]:
    """Run this rank's cells in chunks, each committed atomically as a part file, so a killed rank
    resumes at the first unfinished chunk (failure recovery; ``TB_FAULT_AFTER_PARTS=n`` injects a
    failure after n committed parts, for tests)."""
    pdir = os.path.join(out_dir, f"parts_{dp_rank:03d}_of_{dp_size:03d}")
    done: Dict[int, dict] = {}
    if os.path.isdir(pdir):
        for fn in sorted(os.listdir(pdir)):
            if fn.startswith("part_") and fn.endswith(".json"):
                for r in json.load(open(os.path.join(pdir, fn)))["results"]:
                    done[r["cell_id"]] = r
        if done:
            log(f"[rank {dp_rank}] resuming: {len(done)} cells already committed in {pdir}")
            elog.write("resumed_parts", cells=len(done))
    todo = [i for i in mine if i not in done]
    fault_after = int(os.environ.get("TB_FAULT_AFTER_PARTS", "-1"))
    n_parts = len([f for f in os.listdir(pdir)]) if os.path.isdir(pdir) else 0
    committed = 0
    from .sweep import NextBatch

    chunks = [todo[c0:c0 + max(1, chunk)] for c0 in range(0, len(todo), max(1, chunk))]
    batch_cells = [[cells[i] for i in ids] for ids in chunks]
    for k, ids in enumerate(chunks):
        t = time.perf_counter()
        if k + 1 < len(chunks) and hasattr(runner, "stage_next"):    # cross-batch pipeline: the next chunk's tail queues behind this one's readout
            runner.stage_next(NextBatch(pairs, cells=batch_cells[k + 1]))
        res = runner.run_cells(pairs, batch_cells[k])
        _check_comm(tp_ctx, elog, f"part_{n_parts:05d}")     # before anything of this chunk is committed
        for r, i in zip(res, ids):
            r["cell_id"] = i
            done[i] = r
        if writer:
            os.makedirs(pdir, exist_ok=True)
            atomic_write_json(os.path.join(pdir, f"part_{n_parts:05d}.json"), {"results": res})
        n_parts += 1
        committed += 1
        elog.write("part", cells=len(ids), seconds=round(time.perf_counter() - t, 4),
                   remaining=sum(len(x) for x in chunks[k + 1:]))
        if fault_after >= 0 and committed >= fault_after:
            raise RuntimeError(f"injected fault after {committed} part(s) (TB_FAULT_AFTER_PARTS)")
    return [done[i] for i in mine]
