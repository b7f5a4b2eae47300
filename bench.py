"""Flagship benchmark: SAE-latent-ablation sweep throughput on Gemma-2-9B-IT @ layer 32.

Metric (BASELINE.json): prompts/sec of the targeted-vs-random SAE-ablation
sweep on Gemma-2-9B-IT with the Gemma-Scope 16k SAE at the paper's layer 32
(0-based block 31).  One "prompt" = one sweep cell = one edited greedy hint
generation (50 new tokens, ablation applied at the pair's 4 spike positions)
plus its full readout: hooked-layer logit-lens over every response position
(secret probability + LL-Top-5 guesses), teacher-forced ΔNLL of the baseline
hint under the edit, leak check.

One step (per GPU, weak scaling) = P (word, prompt) pairs × 66 cells
(budgets {1,2,4,8,16,32} × (1 targeted + 10 random)); P is sized to 95 % of the device memory by default
(120 pairs = 7920 cells on one MI355X, ``--pairs-per-step``), plus
the baselines of the next step's P pairs, which ride along in the same decode
batch (their generation, lens, spike selection, SAE latent scoring and base
NLL are all inside the timed step).  Weights are random-init Gemma-2-9B (bf16,
full 42-layer architecture; post-norm gain 32 so the random model writes text-like,
edit-sensitive hints instead of repeating its input token — see README "Performance") and a
random JumpReLU SAE calibrated to L0 ≈ 76; prompts are the paper's 10 hint prompts × 3 secret
words through the offline synthetic Gemma tokenizer.  The 30 (word, prompt) pairs run through one
set of weights — the per-word taboo models merged (identical compute); ``--lora-rank`` batches
unmerged per-word adapters instead, and the ``lora`` side measurement in the JSON runs the same sweep
with 3 distinct rank-8 adapters through the fused LoRA GEMMs (plus its equal-work B = 0 control).

Exact reuse inside a step (every cell's results equal a from-scratch generation; tested on CPU and on
the GPU in the default ``--gemm tb`` mode, whose GEMMs are batch-invariant -- ``--gemm auto`` is faster
per GEMM at some row counts but not exact, see runtime/gemm_dispatch.py): a cell resumes from its baseline's KV / hooked-layer residuals up to its first edit, replays
only the blocks after the hooked layer while its tokens equal the baseline's (teacher-forced tail,
which also yields the ΔNLL), and decodes the full model only from its divergence point; the JSON
"work" block reports how much of each happened.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import torch  # noqa: E402

from taboo_brittleness_amd.config import Config  # noqa: E402
from taboo_brittleness_amd.interp.sae import JumpReLUSAE  # noqa: E402
from taboo_brittleness_amd.models.gemma2 import Gemma2Model  # noqa: E402
from taboo_brittleness_amd.models.spec import get_spec  # noqa: E402
from taboo_brittleness_amd.models.tokenizer import SyntheticTokenizer  # noqa: E402
from taboo_brittleness_amd.models.weights import random_gemma2  # noqa: E402
from taboo_brittleness_amd.parallel import dist as D  # noqa: E402
from taboo_brittleness_amd.pipelines.sweep import NextBatch, Pair, SweepRunner  # noqa: E402
from taboo_brittleness_amd.runtime import gemm_dispatch as GD  # noqa: E402
from taboo_brittleness_amd.runtime.tuning import enable_tuned_gemms, flush_tuned_gemms  # noqa: E402

BASELINE_VALUE = 0.642   # measured HF-eager sweep cells/sec on 1x MI355X (tools/hf_eager_baseline.py)
HF_BATCHED_VALUE = 38.5  # HF-eager with the 66 cells of a pair batched per generate (hf_batched_baseline.py)


def _host_rss_gb():
    try:
        import psutil

        return round(psutil.Process().memory_info().rss / 1e9, 1)
    except Exception:
        return None


def _free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return int(s.getsockname()[1])


def launch_ranks(n: int, argv) -> int:
    """``--gpus N`` without an outer launcher: run this script as N ranks under
    ``torch.distributed.run`` (one process per GPU, RCCL over xGMI) in a CHILD process and return its exit
    code.  Called before anything touches the GPU in this process (no exec: the parent only waits); the
    ranks' stdout (rank 0's JSON line) is inherited."""
    import subprocess

    env = dict(os.environ)
    env.setdefault("MASTER_ADDR", "127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + list(argv)
    return subprocess.run(cmd, env=env).returncode


# --pairs-per-step auto: the largest P whose predicted peak stays within HBM_FRACTION of the device memory, at most
# PAIRS_CAP (round 5 measured 100 / 110 / 120 pairs: 2587 / 2616 / 2643 prompts/s at 240 / 257 / 281 GB reserved,
# profiles/r5/bench/pairs_*.log).  TRANSIENT_GB: what the step allocates besides the per-pair buffers and the model
# (tail / lens logit chunks, GEMM and attention workspaces, decode-graph pools): 262.7 GB peak at P = 110 minus the
# model's 205 GB of per-pair buffers minus the weights.  RCCL_RESERVE_GB: RCCL's own buffers and streams per rank
# (outside torch's allocator) when the job has more than one rank.
PAIRS_CAP = 120
HBM_FRACTION = 0.95
TRANSIENT_GB = 31.0
RCCL_RESERVE_GB = 4.0
LORA_EXTRA_GB = 20.0


def pair_bytes(spec, n_cells: int, E: int, S: int, max_new: int) -> int:
    """Device bytes one (word, prompt) pair adds to a step: the KV cache rows of its cells and of E ride-along
    baselines, their hooked-layer capture rows, its (E + 2) pair-KV slots and its running lens sums."""
    kv_row = spec.layers * spec.kv_heads * spec.head_dim * 2 * 2 * S
    store_row = (S + 1) * spec.hidden * 2
    rows = n_cells + E
    return rows * (kv_row + store_row) + (E + 2) * kv_row + (max_new + 1) * spec.vocab_size * 4


def pairs_for_memory(spec, dev, n_cells: int, E: int, C: int, max_plen: int, max_new: int, world: int,
                     cap: int = PAIRS_CAP, extra_gb: float = 0.0) -> dict:
    """``--pairs-per-step auto``: P from the device memory left after the model and SAE are loaded
    (``torch.cuda.mem_get_info``, so the HIP runtime and anything outside torch's allocator count), minus
    ``1 - HBM_FRACTION`` of the device, the step's transient allocations and (multi-rank) an RCCL reserve."""
    S = max_plen + max_new + 1
    per = pair_bytes(spec, n_cells, E, S, max_new)
    if dev.type != "cuda":
        return {"pairs": max(1, min(cap, 2)), "pair_gb": round(per / 1e9, 3)}
    free, total = torch.cuda.mem_get_info(dev)
    free += torch.cuda.memory_reserved(dev) - torch.cuda.memory_allocated(dev)     # torch's cached, unused blocks
    carry = C * (spec.layers * spec.kv_heads * spec.head_dim * 4 * S)
    avail = free - (1.0 - HBM_FRACTION) * total - (TRANSIENT_GB + extra_gb) * 1e9 - carry - \
        (RCCL_RESERVE_GB * 1e9 if world > 1 else 0.0)
    P = int(max(1, min(cap, avail // per)))
    used = total - free
    return {"pairs": P, "pair_gb": round(per / 1e9, 3), "total_gb": round(total / 1e9, 1),
            "used_before_gb": round(used / 1e9, 1), "total": total,
            "outside_torch": used - torch.cuda.memory_reserved(dev),
            "predicted_peak_gb": round((used + P * per + carry + (TRANSIENT_GB + extra_gb) * 1e9) / 1e9, 1),
            "hbm_fraction": HBM_FRACTION, "cap": cap}


def fresh(p: Pair, rep: int = 0) -> Pair:
    return Pair(p.word, p.pidx, p.prompt, list(p.ids), list(p.forms), list(p.track), rep=rep)


def sweep_bench(args, info, cfg, model, tok, sae, layer: int, P: int, E: int, C: int, methods, steps: int,
                warmup: int, tag: str = "") -> dict:
    """One timed sweep: P (word, prompt) pairs x the methods' cells per step and rank, ``warmup`` untimed steps, then
    exactly ``steps`` timed steps bracketed by a barrier + device sync (the driver contract).  Returns the whole-job
    cells/s (``value``), the per-rank timings, the runner (its ``stats`` cover the timed steps) and the last pairs."""
    dev = info.device
    on_gpu = dev.type == "cuda"
    n_cells = len(model_cells(cfg, methods))
    batch = P * n_cells + E * P + C
    runner = SweepRunner(cfg, model, tok, sae, batch=batch, device=dev, layer=layer,
                         use_graphs=not args.no_graphs, prefix_share=not args.no_prefix_share,
                         kv_pairs=(E + (3 if C else 2)) * P + 2, layer_resume=not args.no_layer_resume)
    runner.carry_rows = C
    runner.trie_decode = not args.no_trie_decode
    runner.skip_noop_spikes = not args.no_skip_noop
    templates = runner.build_pairs(cfg.words, cfg.prompts)

    def pairs_for(step: int):
        # pair instance g of the whole job (every rank and step its own): template g mod 30, replicate g div 30,
        # so a repeated (word, prompt) draws fresh random-latent controls (its targeted cells are the same
        # experiment and repeat exactly) -- no two ranks or steps run identical random cells
        base = (step * info.world + info.rank) * P
        n = len(templates)
        return [fresh(templates[(base + j) % n], rep=(base + j) // n) for j in range(P)]

    # prologue: baselines of the first step's pairs, SAE threshold calibration on their residuals -- one copy of
    # each (word, prompt) template in template order, so every rank calibrates on the same rows (a pair's baseline
    # does not depend on its replicate; with P >= 30 every rank's first step holds every template)
    cur = pairs_for(0)
    runner.run_baselines(cur)
    first = {}
    for p in cur:
        first.setdefault((p.word, p.pidx), p)
    order_keys = [(t.word, t.pidx) for t in templates]
    mine = {k: first[k].resid for k in order_keys if k in first and first[k].resid is not None
            and first[k].resid.shape[0]}
    if info.world > 1 and len(mine) < len(templates):
        # fewer pairs per step than templates: every rank calibrates on the union of the ranks' first-step baselines
        # (a template's baseline does not depend on its rank or replicate), so the SAE thresholds stay rank-invariant
        merged = {}
        for d in D.all_gather_objects({k: v.cpu() for k, v in mine.items()}, info):
            merged.update(d)
        mine = {k: merged[k].to(dev) for k in order_keys if k in merged}
    resid = torch.cat([mine[k] for k in order_keys if k in mine], 0)
    sae.calibrate(resid)
    runner._score_pairs(cur)
    import hashlib

    calib = hashlib.sha256(sae.threshold.float().cpu().numpy().tobytes()).hexdigest()[:16]
    calib_all = [str(c) for c in D.all_gather_objects(calib, info)]
    assert len(set(calib_all)) == 1, f"SAE calibration differs across ranks: {calib_all}"

    future = {}
    staged = {}

    def step(k: int, cur):
        """Cells of step k; baselines ride along: warmup steps carry the next step's pairs, timed steps
        k = W, W+E, ... carry the pairs of steps k+1..k+E (one decode for E*P baselines)."""
        t0 = time.perf_counter()
        if k < warmup:
            ahead = [k + 1]
        elif (k - warmup) % E == 0:
            ahead = list(range(k + 1, k + E + 1))
        else:
            ahead = []
        ride = []
        for j in ahead:
            future[j] = pairs_for(j)
            ride += future[j]
        nb = staged.pop(k, None)
        if nb is not None and nb.future is None and nb.cells is not None:
            cells, plan = nb.cells, nb.plan          # staged by the previous step (its tail may be queued)
        elif nb is not None and nb.future is not None:
            cells, plan = nb.future.result()
        else:
            cells, plan = runner.make_cells(cur, methods), None
        runner.timings["make_cells"] = runner.timings.get("make_cells", 0.0) + time.perf_counter() - t0
        # the next step's cells and host edit plan are built on a helper thread while this step's GPU
        # work runs (when its pairs' baselines are already final); the runner queues the next step's
        # teacher-forced tail behind this step's lens readout (cross-step pipeline, SweepRunner.stage_next)
        nxt = future.get(k + 1)
        if nxt is not None and k + 1 < warmup + steps:
            fut = runner.prefetch(nxt, methods) if all(p.resid is not None for p in nxt) else None
            staged[k + 1] = NextBatch(nxt, methods, future=fut)
            # never across the warmup -> timed boundary: the first timed step runs its own teacher-forced tail,
            # so the timed window holds exactly its K steps' tails (the last timed step stages nothing either)
            if not args.no_pipeline and k + 1 != warmup:
                runner.stage_next(staged[k + 1])
        # the records of step k are assembled on a host thread while step k+1's GPU work runs; decode
        # tails carry into the next step except out of warmup and out of the last timed step
        drain = k < warmup or k == warmup + steps - 1
        res = runner.run_cells_async(cur, cells, ride_along=ride, drain=drain, plan=plan)
        return future.pop(k + 1), res, time.perf_counter() - t0

    def cells_of(k):
        return range(P * n_cells)

    gathers = []

    def gather_results(res):
        """The DP sweep's result collection, every step: each rank's compact cell records (readouts,
        NLLs, leak, n_gen, LL-Top-5 ids) are all-gathered (one RCCL all-gather over xGMI), issued
        asynchronously on the collective's own stream (overlaps the next step's compute; no per-step
        lock-step of the ranks) and completed before the timed window closes."""
        if info.world <= 1:
            return None
        rec = torch.tensor([[r["p_secret_mean"], r["p_secret_final"], r["p_secret_max"], r["nll_edit"],
                             r["nll_self"], float(r["leak"]), float(r["n_gen"])] +
                            [float(t) for t in (list(r["topk_ids"]) + [-1] * 5)[:5]] for r in res],
                           dtype=torch.float64)
        if on_gpu:
            rec = rec.pin_memory().to(dev, non_blocking=True)
        out, work = D.all_gather_tensor_async(rec, info)
        gathers.append((out, work, rec))
        return out

    def finish_gathers():
        for out, work, rec in gathers:
            if work is not None:
                work.wait()
        n = sum(int(out.shape[0]) for out, _, _ in gathers)
        gathers.clear()
        return n

    for k in range(warmup):
        cur, res, dt = step(k, cur)
        gather_results(res.result())
        if info.is_main:
            print(f"[bench{tag}] warmup step {k + 1}/{warmup} done", file=sys.stderr, flush=True)
    finish_gathers()
    runner.precapture_graphs()          # one-time setup: every decode row-bucket graph
    # everything allocated so far (model, tokenizer tables, caches) is long-lived: keep the cyclic GC from
    # rescanning it on every collection inside the timed steps (pauses the launch thread otherwise)
    gc.collect()
    gc.freeze()
    if on_gpu:
        torch.cuda.synchronize()
    D.barrier(info)
    for kk in runner.stats:
        runner.stats[kk] = 0
    t0 = time.perf_counter()
    n_done = 0
    pending = None
    marks = runner.__dict__.setdefault("phase_marks", []) if os.environ.get("TB_PHASE_MARKS") else None
    for k in range(warmup, warmup + steps):
        if marks is not None:
            marks.append((f"step{k}", time.monotonic_ns()))
        cur, res, dt = step(k, cur)
        if pending is not None:
            done = pending.result()
            n_done += len(done)
            gather_results(done)
        pending = res
        if args.profile_steps and info.is_main:
            ph = " ".join(f"{kk}={v:.3f}" for kk, v in runner.timings.items())
            runner.timings.clear()
            print(f"[step {k}] {len(cells_of(k))} cells in {dt:.3f}s  {ph}", file=sys.stderr, flush=True)
        elif info.is_main:      # host-side progress (no sync): long runs keep writing
            print(f"[bench{tag}] step {k - warmup + 1}/{steps} issued at {time.perf_counter() - t0:.1f}s",
                  file=sys.stderr, flush=True)
    done = pending.result()
    n_done += len(done)
    gather_results(done)
    gathered_rows = finish_gathers()
    assert info.world <= 1 or gathered_rows == n_done * info.world, "result all-gather incomplete"
    if on_gpu:
        torch.cuda.synchronize()
    D.barrier(info)
    if marks is not None:
        marks.append(("end", time.monotonic_ns()))
    mine = time.perf_counter() - t0
    per_rank = [float(v) for v in D.all_gather_objects(mine, info)]
    elapsed = D.all_reduce_max(mine, info)
    total_cells = D.all_reduce_max(float(n_done), info) * info.world   # every rank does the same count
    value = total_cells / elapsed
    ms = 1000.0 * elapsed / max(steps, 1)
    return {"value": value, "elapsed": elapsed, "ms": ms, "per_rank": per_rank, "n_done": n_done,
            "gathered_rows": gathered_rows, "calib_all": calib_all, "runner": runner, "cur": cur, "batch": batch,
            "n_cells": n_cells, "marks": marks}


def model_cells(cfg, methods):
    """(method, budget, trial) of one pair's cells (SweepRunner.make_cells' order)."""
    out = []
    iv = cfg.intervention
    for meth in methods:
        if meth.startswith("sae"):
            budgets, trials = iv.budgets, (1 if meth == "sae_targeted" else iv.random_trials)
        else:
            budgets, trials = iv.ranks, (1 if meth == "proj_targeted" else iv.proj_random_trials)
        out += [(meth, b, t) for b in budgets for t in range(trials)]
    return out


def release_state(model, release) -> None:
    """Free a finished sweep's device state (decode KV, capture store, pair KV: most of the device memory), the
    post-forcing generator's KV cache and the model's workspaces before the next side measurement allocates."""
    from taboo_brittleness_amd.pipelines import token_forcing as TF

    for r_ in release:
        if hasattr(r_, "gen"):
            r_.gen = r_.store = r_.pair_kv = r_.capture = None
            r_._plan = r_._hook = r_._staged = None
    release.clear()
    model._ws.clear()
    TF._FORCING_STATE.clear()
    gc.unfreeze()                  # (sweep_bench froze the heap: let the collector see the released runner's cycles)
    gc.collect()
    if model.device.type == "cuda":
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        torch.cuda.reset_peak_memory_stats(model.device)


def lora_forward_cost(model, bank, dev, rows=(64, 1024, 2048)) -> dict:
    """The fused LoRA path's own cost, work held fixed: one decode-shaped forward (T = 1, every layer) of ``rows`` rows
    with the adapter bank (every row its word's adapter, 3 words mixed) vs the same rows on the base model: GPU time of
    a hipGraph replay (ms, median of 5 after 2 warm replays), as the sweep's decode steps run; the sweep numbers also
    differ by how often the adapted model's tokens diverge."""
    if dev.type != "cuda":
        return {}
    out = {}
    for M in rows:
        ids = torch.randint(3, model.spec.vocab_size, (M, 1), device=dev, dtype=torch.int32)
        pos = torch.full((M, 1), 40, dtype=torch.int32, device=dev)
        cache = model.new_cache(M, 41)
        cache.adapter.copy_(torch.arange(M, dtype=torch.int32, device=dev) % bank.n)
        slot = torch.arange(M, dtype=torch.int32, device=dev)
        t = {}
        for mode in ("lora", "base"):
            model.set_lora(bank if mode == "lora" else None)
            if mode == "base":
                model.enable_fused_geglu()
            ws = model.workspace(M)
            model.forward(ids, pos, cache, slot, ws=ws)          # warm: kernels, tables, the split-K workspace
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()                            # GPU time only, as the sweep's decode graphs replay
            with torch.cuda.graph(g):
                model.forward(ids, pos, cache, slot, ws=ws)
            ts = []
            for i in range(7):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                g.replay()
                e1.record()
                e1.synchronize()
                ts.append(e0.elapsed_time(e1))
            t[mode] = sorted(ts[2:])[2]
            del g
        out[str(M)] = {"lora_ms": round(t["lora"], 3), "base_ms": round(t["base"], 3),
                       "ratio": round(t["lora"] / t["base"], 4)}
        del cache
        model._ws.clear()
    model.set_lora(bank)
    return out


def side_sweep(args, info, cfg, model, tok, sae, layer, spec, kind: str, methods, steps: int, warmup: int,
               release) -> dict:
    """A side measurement after the timed headline (one GPU): ``lora`` -- the headline sweep with the 3 words'
    distinct rank-8 adapters batched unmerged (models/lora.py fused path; each pair's rows run its word's adapter);
    ``lowrank`` -- BASELINE config 4, the low-rank secret-direction projection-out sweep (ranks 1..64, PCA of the
    pooled spike residuals, random-subspace controls drawn on the GPU by csrc/basis.hip) with the same reuse levels.
    P from the memory model."""
    from copy import deepcopy

    from taboo_brittleness_amd.interp.prompts import hint_prompt_ids

    dev = info.device
    release_state(model, release)
    c = deepcopy(cfg)
    if kind == "lowrank":
        c.intervention.ranks = [1, 2, 4, 8, 16, 32, 64]
    bank = None
    if kind == "lora":
        from taboo_brittleness_amd.models.lora import LoRABank

        bank = LoRABank.random(spec, list(c.words), r=8, alpha=16.0, seed=99, device=dev)
        model.set_lora(bank)
    try:
        n_cells = len(model_cells(c, methods))
        E = max(e for e in range(1, max(1, args.baseline_every) + 1) if steps % e == 0)
        # (lora: the adapters' T operands, and a third more decode rows than the merged model -- its random adapters
        # flip more greedy tokens -- in the step's transient memory: 294 GB peak at P = 120 without this reserve)
        # cap: the headline's cells per step (PAIRS_CAP pairs of 66 cells), so the lowrank side's 42-cell pairs run
        # as large batches; its basis table (rmax = 64 fp32 rows per cell) is reserved on top of the model
        cap = max(1, PAIRS_CAP * 66 // n_cells) if dev.type == "cuda" else 2
        extra = LORA_EXTRA_GB if kind == "lora" else \
            cap * (n_cells + E) * max(c.intervention.ranks) * spec.hidden * 4 / 1e9 + 2.0
        mp = pairs_for_memory(spec, dev, n_cells, E, 0, max(len(hint_prompt_ids(tok, q)) for q in c.prompts),
                              args.max_new, 1, cap=cap, extra_gb=extra)
        if args.side_pairs > 0:
            mp["pairs"] = min(mp["pairs"], args.side_pairs)
        t0 = time.perf_counter()
        R = sweep_bench(args, info, c, model, tok, sae, layer, mp["pairs"], E, 0, methods, steps, warmup, tag=f" {kind}")
        run = R["runner"]
        st = dict(run.stats)
        args.side_marks = list(getattr(run, "phase_marks", []))     # (--only-side with TB_PHASE_MARKS)
        out = {"metric": ("multi-adapter SAE-ablation sweep prompts/s (3 distinct rank-8 per-word LoRA adapters, "
                          "unmerged, fused into the in-tree GEMMs)" if kind == "lora" else
                          f"low-rank projection-out sweep prompts/s (BASELINE config 4: ranks 1..64 x (1 targeted PCA "
                          f"+ 5 random subspaces), {args.max_new} new tokens)"),
               "value": round(R["value"], 3), "unit": "prompts/s", "n_gpus": 1, "steps": steps, "warmup": warmup,
               "ms_per_step": round(R["ms"], 2), "pairs_per_step": mp["pairs"], "cells_per_pair": n_cells,
               "diverged_frac": round(st["diverged"] / max(1, st["cells"]), 4),
               "decode_row_steps_per_cell": round(st["decode_row_steps"] / max(1, st["cells"]), 2),
               "peak_mem_gb": round(torch.cuda.max_memory_reserved(dev) / 1e9, 1) if dev.type == "cuda" else None,
               "wall_s": round(time.perf_counter() - t0, 1)}
        if kind == "lora":
            out["adapters"] = {"n": bank.n, "rank": bank.r, "kp": int(bank.KP), "words": list(bank.names)}
            release += [R["runner"], R["cur"]]
            R = run = None
            release_state(model, release)
            out["forward_ms"] = lora_forward_cost(model, bank, dev)
            if not args.no_lora_control:
                # equal-work control: the same bank and fused kernels with every up-projection B = 0 (PEFT's own
                # init), so each row's output is bit-identical to the base model's (the K-augmented columns add
                # exact zeros) and the sweep does the headline's work -- what the unmerged multi-adapter machinery
                # costs, apart from how the adapted model's tokens diverge
                bank.zero_up()
                R = sweep_bench(args, info, c, model, tok, sae, layer, mp["pairs"], E, 0, methods, steps, warmup,
                                tag=" lora_b0")
                st = dict(R["runner"].stats)
                out["control_b0"] = {
                    "value": round(R["value"], 3), "ms_per_step": round(R["ms"], 2),
                    "diverged_frac": round(st["diverged"] / max(1, st["cells"]), 4),
                    "decode_row_steps_per_cell": round(st["decode_row_steps"] / max(1, st["cells"]), 2)}
                release += [R["runner"], R["cur"]]
                R = None
                release_state(model, release)
        if R is not None:
            release += [R["runner"], R["cur"]]
        return out
    finally:
        if bank is not None:
            model.set_lora(None)
            model.enable_fused_geglu()


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--arch", default="gemma2-9b")
    ap.add_argument("--pairs-per-step", default="auto",
                    help="(word, prompt) pairs per step and GPU, x 66 cells each, or 'auto' (default): as many as fit "
                         "in HBM_FRACTION of the device memory after the model is loaded, with a reserve for RCCL and "
                         "graph pools (pairs_for_memory), capped at PAIRS_CAP")
    ap.add_argument("--backend", default="auto", choices=["auto", "nccl", "gloo"],
                    help="collective backend: auto = RCCL with one GPU per rank (gloo when ranks share a GPU)")
    ap.add_argument("--max-new", type=int, default=50)
    ap.add_argument("--no-nll", action="store_true")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--no-prefix-share", action="store_true",
                    help="recompute every cell from its prompt instead of resuming from the baseline prefix")
    ap.add_argument("--no-layer-resume", action="store_true",
                    help="decode every cell through all blocks from its first edit (no exact layer resume)")
    ap.add_argument("--baseline-every", type=int, default=4,
                    help="generate the next E steps' baselines together every E steps (one decode of E*P rows; "
                         "E is reduced to a divisor of --steps so the timed window holds exactly its share)")
    ap.add_argument("--lora-rank", type=int, default=0,
                    help="per-word random LoRA adapters of this rank, batched unmerged (multi-adapter bank)")
    ap.add_argument("--carry-rows", type=int, default=0,
                    help="decode-tail carry-over: once fewer diverged cells than this still decode, they continue in "
                         "the next step's decode (spare KV slots; warmup and the last timed step drain); 0 = off. "
                         "768 measured +1.6%% at +31 GB (profiles/bench_r1_carry_ab.log), so off by default")
    ap.add_argument("--init-gain", type=float, default=32.0,
                    help="post-norm gain of the random init (models.weights.random_gemma2).  1 = plain HF init, "
                         "whose random Gemma-2 repeats its input token so no edit ever changes a generation "
                         "(diverged_frac 0); 32 gives text-like outputs (~34 distinct tokens per 50) and "
                         "edits that change ~2/3 of the generations")
    ap.add_argument("--fused-geglu", action="store_true",
                    help="(default) the gate|up GEMM with the GeGLU in its epilogue (in-tree gemm4 / ring GEMM); "
                         "only --gemm auto / blas may pick hipBLASLt + the GeGLU kernel at some row counts")
    ap.add_argument("--no-fused-geglu", action="store_true", help="never the fused gate|up + GeGLU kernel")
    ap.add_argument("--gemm", default=None, choices=["auto", "tb", "blas"],
                    help="GEMM dispatch (runtime/gemm_dispatch.py): tb = in-tree batch-invariant MFMA kernels "
                         "(default: the reuse levels are exact), auto = fastest measured per shape incl. split-K / "
                         "hipBLASLt (not batch-invariant), blas = hipBLASLt only")
    ap.add_argument("--fused-head", action="store_true",
                    help="vocab head as the fused four-wave MFMA GEMM head (softcap / log-sum-exp / argmax in the GEMM "
                         "epilogue, no logits in HBM) instead of the in-tree logits GEMM + the decode_head kernel (the "
                         "default: the fused head measured 0.94-0.99x, profiles/r5/head_bench_tb.log)")
    ap.add_argument("--no-fused-head", action="store_true", help="the default (kept for older command lines)")
    ap.add_argument("--no-trie-decode", action="store_true",
                    help="decode every diverged cell through all blocks on its own row instead of running blocks "
                         "0..l once per group of a pair's cells with equal tokens (prefix-trie decode)")
    ap.add_argument("--no-skip-noop", action="store_true",
                    help="start every cell's teacher-forced tail at its pair's first spike, also when the cell's "
                         "latents are inactive there (an exact no-op edit)")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="do not queue the next step's teacher-forced tail behind this step's readout")
    ap.add_argument("--profile-steps", action="store_true", help="print per-phase timings per step")
    ap.add_argument("--post-forcing", action="store_true",
                    help="(default) also time the post-edit postgame token forcing of the sweep's SAE settings, "
                         "after the timed region (reported as 'post_forcing', outside the headline)")
    ap.add_argument("--no-post-forcing", action="store_true", help="skip the post-edit forcing side measurement")
    ap.add_argument("--no-config2", action="store_true",
                    help="skip the BASELINE config-2 side measurement (LL-Top-k baseline: batched greedy hints + "
                         "42-layer lens over 3 words x 10 prompts), reported as 'config2' after the timed steps")
    ap.add_argument("--no-lora-side", action="store_true",
                    help="skip the multi-adapter side measurement ('lora': the same sweep with 3 distinct rank-8 "
                         "per-word adapters batched unmerged through the fused LoRA GEMMs, same steps / warmup)")
    ap.add_argument("--no-lora-control", action="store_true",
                    help="skip the lora side's equal-work control (the same adapters with B = 0: the base model's "
                         "outputs and work through the unmerged fused path)")
    ap.add_argument("--no-lowrank-side", action="store_true",
                    help="skip the BASELINE config-4 side measurement ('lowrank': projection-out cells, ranks 1..64)")
    ap.add_argument("--lowrank-steps", type=int, default=4, help="timed steps of the lowrank side measurement")
    ap.add_argument("--side-pairs", type=int, default=0,
                    help="at most this many pairs per step in the side sweeps (0: the memory model's P, capped at the "
                         "headline's cells per step)")
    ap.add_argument("--only-side", default=None, choices=["lora", "lowrank"],
                    help="run only this side measurement (its own warmup / timed steps; profiling), print its JSON")
    ap.add_argument("--tune-gemms", action="store_true",
                    help="run TunableOp over every GEMM shape and save configs/tunableop/<tag>.csv")
    ap.add_argument("--no-tuned-gemms", action="store_true", help="ignore the saved TunableOp results")
    args = ap.parse_args()
    args.post_forcing = not args.no_post_forcing
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))

    info = D.init_distributed(args.backend)
    assert info.world == args.gpus, f"--gpus {args.gpus} but the launcher started {info.world} rank(s)"
    if info.world > 1 and "OMP_NUM_THREADS" not in os.environ:
        # one rank per GPU on one node: each rank's host threads get its share of the cores (torch's default is
        # every core per process, i.e. N-fold oversubscription of the host work the GPU waits on)
        local = int(os.environ.get("LOCAL_WORLD_SIZE", info.world))
        torch.set_num_threads(max(1, min(16, (os.cpu_count() or 1) // max(1, local))))
    dev = info.device
    on_gpu = dev.type == "cuda"
    arch = args.arch if on_gpu else "gemma2-tiny"
    spec = get_spec(arch)
    cfg = Config()
    cfg.experiment.max_new_tokens = args.max_new
    cfg.intervention.measure_nll = not args.no_nll
    E = max(e for e in range(1, max(1, args.baseline_every) + 1) if args.steps % e == 0)
    n_cells = len(cfg.intervention.budgets) * (1 + cfg.intervention.random_trials)
    P = None if str(args.pairs_per_step) == "auto" else int(args.pairs_per_step)

    torch.manual_seed(0)
    tag = f"{spec.name}_P{P or PAIRS_CAP}_E{E}_new{args.max_new}"
    if on_gpu and not args.no_tuned_gemms:
        from taboo_brittleness_amd.runtime.tuning import gemm_results_path
        if not args.tune_gemms and not os.path.exists(gemm_results_path(tag)):
            # (hipBLASLt only runs in --gemm auto / blas): the P = 100 table covers most of the shapes
            tag = f"{spec.name}_P100_E{E}_new{args.max_new}"
        enable_tuned_gemms(tag, tune=args.tune_gemms)
    weights = random_gemma2(spec, device=dev, dtype=torch.bfloat16, seed=1234, post_norm_gain=args.init_gain)
    model = Gemma2Model(weights, dev)
    if args.gemm:
        GD.set_mode(args.gemm)
    if args.no_fused_geglu:
        model._wgu_il = None
    fused_geglu = model._wgu_il is not None
    if args.fused_head:
        model.fused_head = bool(on_gpu and spec.vocab_size % 256 == 0)
    elif args.no_fused_head:
        model.fused_head = False
    if args.lora_rank > 0:
        from taboo_brittleness_amd.models.lora import LoRABank

        model.set_lora(LoRABank.random(spec, list(cfg.words), r=args.lora_rank, alpha=2.0 * args.lora_rank,
                                       seed=99, device=dev))
    tok = SyntheticTokenizer(vocab_size=spec.vocab_size)
    sae = JumpReLUSAE.random(spec.hidden, cfg.sae.d_sae, seed=7, device=dev)
    layer = min(cfg.model.layer_idx, spec.layers - 1)
    C = max(0, args.carry_rows) if not args.no_layer_resume else 0
    from taboo_brittleness_amd.interp.prompts import hint_prompt_ids

    mem_plan = pairs_for_memory(spec, dev, n_cells, E, C, max(len(hint_prompt_ids(tok, q)) for q in cfg.prompts),
                                args.max_new, info.world, cap=PAIRS_CAP if on_gpu else 2)
    if P is None:
        # every rank runs the same P (weak scaling: one per-GPU workload); the smallest fit wins
        P = int(-D.all_reduce_max(-float(mem_plan["pairs"]), info))
    mem_plan["pairs"] = P
    mem_plan["auto"] = str(args.pairs_per_step) == "auto"
    if args.only_side:
        mth = ("sae_targeted", "sae_random") if args.only_side == "lora" else ("proj_targeted", "proj_random")
        st = args.steps if args.only_side == "lora" else args.lowrank_steps
        res = side_sweep(args, info, cfg, model, tok, sae, layer, spec, args.only_side, mth, st,
                         args.warmup if args.only_side == "lora" else 1, [])
        if info.is_main:
            print(json.dumps(res), flush=True)
            if os.environ.get("TB_PHASE_MARKS"):
                with open(os.environ["TB_PHASE_MARKS"], "w") as f:
                    json.dump(getattr(args, "side_marks", []), f)
        D.destroy(info)
        return
    methods = ("sae_targeted", "sae_random")
    R = sweep_bench(args, info, cfg, model, tok, sae, layer, P, E, C, methods, args.steps, args.warmup)
    value, elapsed, ms, per_rank = R["value"], R["elapsed"], R["ms"], R["per_rank"]
    n_done, gathered_rows, calib_all, runner, cur, batch = (R["n_done"], R["gathered_rows"], R["calib_all"],
                                                            R["runner"], R["cur"], R["batch"])
    R = None                      # (the side sweeps release the runner: no other reference may keep it alive)
    peak_gb = round(torch.cuda.max_memory_reserved(dev) / 1e9, 1) if on_gpu else None   # of the timed steps
    if on_gpu:      # the peak as a fraction of the device: torch's reserved peak + what lives outside its allocator
        mem_plan["peak_hbm_frac"] = round((torch.cuda.max_memory_reserved(dev) + mem_plan["outside_torch"]) /
                                          mem_plan["total"], 4)
    for k_ in ("total", "outside_torch"):
        mem_plan.pop(k_, None)
    config2 = None
    side = info.world == 1          # the side measurements are single-GPU numbers: not repeated per scaling run
    if (args.post_forcing or not args.no_config2) and info.is_main and side:
        # the side measurements below run after the timed region: release the sweep's decode state first (its
        # KV / store / pair-KV buffers are most of the ~240 GB the timed steps hold)
        runner.gen = runner.store = runner.pair_kv = runner.capture = None
        runner._plan = runner._hook = runner._staged = None
        for p_ in cur:
            p_.lens_cum = None
        model._ws.clear()
        if on_gpu:
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
    if not args.no_config2 and info.is_main and side:
        # BASELINE config 2 (LL-Top-k baseline, 3 words x 10 prompts, all 42 layers), after the timed region:
        # one warm call (graph-free decode, TunableOp lookups), then one timed call
        from taboo_brittleness_amd.pipelines.baselines import ll_baseline_batch

        c2 = Config()
        c2.experiment.max_new_tokens = 50
        ll_baseline_batch(c2, model, tok, c2.words, c2.prompts)
        if on_gpu:
            torch.cuda.synchronize()
        t2 = time.perf_counter()
        r2 = ll_baseline_batch(c2, model, tok, c2.words, c2.prompts)
        if on_gpu:
            torch.cuda.synchronize()
        dt2 = time.perf_counter() - t2
        npair = len(c2.words) * len(c2.prompts)
        config2 = {"metric": "LL-Top-k baseline pairs/s (greedy 50-token hints + 42-layer logit lens @L31 + "
                             "top-5 guesses + metrics)", "pairs": npair, "seconds": round(dt2, 3),
                   "pairs_per_s": round(npair / dt2, 2), "lens_rows": r2["rows"], "n_gpus": 1}
    forcing = None
    if args.post_forcing and info.is_main and side:
        # post-edit postgame token forcing (EP:100-104) as its own clearly labelled number, after
        # the timed region: per word the unedited model plus every (sae method, budget, trial) setting of the
        # sweep, each generating the 3 warm-up turns and the 10 prefilled answers under its edit
        from types import SimpleNamespace

        from taboo_brittleness_amd.pipelines import token_forcing as TF
        from taboo_brittleness_amd.pipelines.run_sweep import forcing_curves

        fc = Config()
        fc.intervention.budgets = list(cfg.intervention.budgets)
        fc.intervention.random_trials = cfg.intervention.random_trials
        st = SimpleNamespace(model=model, tok=tok, sae=sae, layer=layer)
        # one warm call (as config 2): the forcing generator, its KV cache and decode graphs are built here and
        # reused by the timed call, which then measures the steady-state forcing throughput
        forcing_curves(fc, runner, cur, methods, st, log=lambda *a: None)
        if on_gpu:
            torch.cuda.synchronize()
        t3 = time.perf_counter()
        fr = forcing_curves(fc, runner, cur, methods, st, log=lambda *a: None)
        if on_gpu:
            torch.cuda.synchronize()
        dt3 = time.perf_counter() - t3
        nset = len(fc.words) * (1 + sum(1 + fc.intervention.random_trials for _ in fc.intervention.budgets))
        forcing = {"metric": "post-edit postgame token-forcing settings/s (3 warm-up turns x 50 tokens + 10 "
                              "prefilled answers x 20 tokens per setting, edit at every position)",
                   "settings": nset, "rows": nset * len(fc.token_forcing.phrases), "seconds": round(dt3, 3),
                   "settings_per_s": round(nset / dt3, 3), "baseline_success": fr["baseline_success"], "n_gpus": 1,
                   "phases_s": dict(TF.LAST_TIMINGS)}
    if info.is_main:
        out = {
            "metric": "prompts/sec SAE-ablation sweep Gemma-2-9B @L32",
            "value": round(value, 3),
            "unit": "prompts/s",
            "n_gpus": info.world,
            "ranks": {"world_size": info.world, "backend": info.backend,
                      "ms_per_step": [round(1000.0 * v / max(args.steps, 1), 2) for v in per_rank],
                      # rows of the per-step cell-record all-gathers (every rank's cells, every timed step)
                      "gathered_rows": int(gathered_rows) if info.world > 1 else int(n_done),
                      "sae_calib_sha": calib_all},
            "mem": mem_plan,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 2),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": (value / BASELINE_VALUE) if BASELINE_VALUE else None,
            # against the stronger stock-PyTorch point (HF eager, a pair's 66 cells batched per generate)
            "vs_hf_batched": round(value / HF_BATCHED_VALUE, 2),
            "dtype": "bf16",
            "data": "synthetic (random-init weights of the full architecture, random calibrated SAE, paper prompts)",
            "config": {
                "model": spec.name + ("-it" if spec.name == "gemma2-9b" else ""),
                "sae": f"gemma-scope-16k JumpReLU (random, L0~76) @ block 31, {str(sae.table_dtype).split('.')[-1]} "
                       f"tables (fp32 encode via a bf16x3 split MFMA)",
                "global_batch": int(batch * info.world),
                "cells_per_step_per_gpu": P * n_cells,
                "seq_len": int(max(p.plen for p in cur) + args.max_new),
                "max_new_tokens": args.max_new,
                "parallelism": f"dp{info.world}",
                "nll": not args.no_nll,
                "graphs": not args.no_graphs,
                "prefix_share": not args.no_prefix_share,
                "layer_resume": not args.no_layer_resume,
                "baseline_every": E,
                "carry_rows": C,
                "fused_geglu": fused_geglu,
                "gemm_dispatch": GD.describe(),
                "fused_head": bool(getattr(model, "fused_head", False)),
                "trie_decode": runner.trie_decode,
                "skip_noop_spikes": runner.skip_noop_spikes,
                "lora_adapters": (f"{len(cfg.words)} x rank {args.lora_rank} (unmerged bank)" if args.lora_rank
                                  else "none (weights as merged taboo models)"),
            },
            "config2": config2,
            "post_forcing": forcing,
            "lora": None,
            "lowrank": None,
            # work actually done in the timed steps (rank 0): cells whose greedy tokens left their
            # baseline's decode from the divergence through all blocks; the rest are exact replays of
            # the blocks after the hooked layer (see pipelines/sweep.py::_run_batch_resume)
            "work": {
                "cells": runner.stats["cells"],
                "diverged_frac": round(runner.stats["diverged"] / max(1, runner.stats["cells"]), 4),
                "tail_rows_per_cell": round(runner.stats["tf_rows"] / max(1, runner.stats["cells"]), 2),
                "lens_rows_per_cell": round(runner.stats["lens_rows"] / max(1, runner.stats["cells"]), 2),
                # lens rows actually unembedded (rows of equal-token cells at unedited positions evaluated once)
                "lens_gemm_rows_per_cell": round(runner.stats["lens_gemm_rows"] / max(1, runner.stats["cells"]), 2),
                # full-model decode of the diverged cells: row-steps needed per cell, and the fraction of
                # computed rows that were needed (the rest is row-bucket padding)
                "decode_row_steps_per_cell": round(runner.stats["decode_row_steps"] / max(1, runner.stats["cells"]), 2),
                "decode_bucket_eff": round(runner.stats["decode_row_steps"] / max(1, runner.stats["decode_rows_run"]), 3),
                # prefix-trie decode: blocks-0..l rows computed (bucketed) per decode row computed; 1.0 = no sharing
                "decode_lo_frac": round(runner.stats["decode_lo_rows_run"] / max(1, runner.stats["decode_rows_run"]), 3)
                if runner.trie_decode else 1.0,
                "carried_cells_per_step": round(runner.stats["carried"] / max(1, args.steps), 1),
                # timed steps whose teacher-forced tail was queued behind the previous step's readout
                "pipelined_steps": runner.stats["staged"],
                # non-degeneracy of the random model: distinct tokens per baseline response, and the
                # fraction of response tokens equal to their input token (a self-copying model is 1.0)
                "peak_mem_gb": peak_gb,
                # host memory of this rank (an 8-GPU node runs 8 of these)
                "host_rss_gb": _host_rss_gb(),
                "distinct_tokens_per_resp": round(float(sum(len(set(p.resp)) for p in cur) / max(1, len(cur))), 2),
                "self_copy_frac": round(float(sum(sum(a == b for a, b in zip(p.gen_toks[1:], p.gen_toks[:-1]))
                                                  for p in cur) / max(1, sum(len(p.gen_toks) - 1 for p in cur))), 3),
            },
        }
        phase_marks = list(getattr(runner, "phase_marks", []))
        if side:
            # after the headline's records are taken: the multi-adapter and low-rank sweeps (each its own P, warmup
            # and timed steps; the headline's decode state is released first)
            rel = [runner, cur]
            runner = cur = None
            if not args.no_lora_side and args.lora_rank == 0:
                out["lora"] = side_sweep(args, info, cfg, model, tok, sae, layer, spec, "lora",
                                         ("sae_targeted", "sae_random"), args.steps, args.warmup, rel)
                cb = out["lora"].get("control_b0")
                if cb:   # machinery cost at equal work: the B = 0 control vs the merged headline (same steps)
                    cb["vs_headline"] = round(cb["value"] / out["value"], 4)
            if not args.no_lowrank_side:
                out["lowrank"] = side_sweep(args, info, cfg, model, tok, sae, layer, spec, "lowrank",
                                            ("proj_targeted", "proj_random"), args.lowrank_steps, 1, rel)
        print(json.dumps(out), flush=True)
    marks_path = os.environ.get("TB_PHASE_MARKS")
    if marks_path and info.is_main:
        with open(marks_path, "w") as f:
            json.dump(phase_marks, f)
    if args.tune_gemms:
        flush_tuned_gemms()
    D.destroy(info)


if __name__ == "__main__":
    main()
