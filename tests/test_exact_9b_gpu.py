"""The headline's exactness at the full Gemma-2-9B shapes, end to end on the MI355X (VERDICT r5 "next" item 1).

The bench's prompts/s counts a cell as done when its records are what a from-scratch generation of that cell gives
(each cell a fresh edited ``generate`` + readout in the reference, `/root/reference/src/models.py:74-79`).  The bench
gets there through six reuse levels (prefix sharing, layer resume, lens reuse, prefix-trie decode, lens row dedup,
no-op spike skip) plus ride-along baselines, 64-row decode buckets and hipGraph replay; they are exact only because
the default GEMM mode ``tb`` is batch-invariant at every row count.  The kernel tests show the ring tiles, the
112-column tiles and the ``gs`` row split equal ``gemm4`` bit for bit; the engine tests run the reuse levels on a
4-layer spec whose shapes are not in the dispatch table.  This module closes the gap at the shapes the headline
runs: the full 42-layer spec, the bench's init (post-norm gain 32), the committed ``tb_shapes`` table
(``configs/gemm_dispatch/gemma2-9b.json``), the bench's 66 cells per pair and 50 new tokens.

* :func:`test_sweep_9b_reuse_levels_exact` -- every reuse level on (bench-shaped: baselines of the second pair group
  ride along in the first group's cell batch, graphs precaptured, a second pass replays them) vs every cell from
  scratch (no prefix sharing, no layer resume, no trie, no skip, no graphs, cells in reversed order and in batches
  of another size, so every GEMM of a cell runs at other row counts);
* :func:`test_sweep_9b_dp2_equals_dp1` -- the ``run_sweep`` entry point as DP = 2 (two processes sharing the GPU,
  gloo collectives) vs DP = 1: identical cell records.

Tokens, guesses, leak verdicts and spike / latent choices are compared bit for bit.  Float aggregates are compared
bit for bit too, except where the two paths sum the same per-token terms in another order: a resumed cell's NLL and
lens means add its baseline's per-position terms (fp64 cumulative sums, ``pipelines/sweep_readout.py``) to its own
tail's, the scratch cell sums them in one pass -- ``FLOAT_RTOL`` below (measured 1.7e-7 relative at most here,
``profiles/r6/exact/exact_9b_reuse.json``).  The per-token values are bit-identical: the teacher-forced tails run
the decode's attention arithmetic (csrc/attention.hip ``attn_tail_exact_kernel``; before it, the tails' online-
softmax MFMA kernel moved edit NLLs by up to 2e-4 relative at these shapes).  ``TB_EXACT_OUT=<dir>`` writes the comparison summaries there.
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import time

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FLOAT_RTOL = 1e-6
EXACT_FIELDS = ("response_ids", "topk_ids", "guesses", "leak", "n_gen", "spikes", "secret_in_topk")
FLOAT_FIELDS = ("p_secret_mean", "p_secret_final", "p_secret_max", "nll_edit", "nll_self", "nll_base",
                "p_secret_mean_base")


def _key(r):
    return (r["word"], r["prompt_idx"], r["method"], r["budget"], r["trial"])


def _fclose(x, y, rtol):
    if x != x and y != y:
        return True
    return x == y or abs(x - y) <= rtol * max(abs(x), abs(y))


def compare_records(a: dict, b: dict, rtol: float = FLOAT_RTOL) -> dict:
    """Field-by-field comparison of two ``{key: record}`` maps; returns a summary (mismatch counts, the largest
    relative float difference, how many float fields are bit-equal)."""
    assert set(a) == set(b), (len(set(a) ^ set(b)), sorted(set(a) ^ set(b))[:5])
    bad, worst, n_float, n_float_eq = [], 0.0, 0, 0
    for k in a:
        for f in EXACT_FIELDS:
            if f in a[k] and a[k][f] != b[k][f]:
                bad.append((k, f, a[k][f], b[k][f]))
        for f in FLOAT_FIELDS:
            if f not in a[k]:
                continue
            x, y = float(a[k][f]), float(b[k][f])
            n_float += 1
            n_float_eq += int(x == y or (x != x and y != y))
            if not _fclose(x, y, rtol):
                bad.append((k, f, x, y))
            elif x == x and y == y and x != y:
                worst = max(worst, abs(x - y) / max(abs(x), abs(y)))
        for x, y in zip(a[k].get("decoy_probs", []), b[k].get("decoy_probs", [])):
            if not _fclose(float(x), float(y), rtol):
                bad.append((k, "decoy_probs", x, y))
    return {"records": len(a), "mismatches": len(bad), "first": [str(x) for x in bad[:5]],
            "float_fields": n_float, "float_bit_equal": n_float_eq, "max_rel_float_diff": worst}


def _out_dir():
    d = os.environ.get("TB_EXACT_OUT")
    if d:
        os.makedirs(d, exist_ok=True)
    return d


@pytest.fixture(scope="module")
def model9b(gpu):
    from taboo_brittleness_amd.models.gemma2 import Gemma2Model
    from taboo_brittleness_amd.models.spec import GEMMA2_9B
    from taboo_brittleness_amd.models.weights import random_gemma2
    from taboo_brittleness_amd.runtime import gemm_dispatch as GD

    old = GD.mode()
    GD.set_mode("tb")
    GD.load_table()                 # the committed table (configs/gemm_dispatch/gemma2-9b.json) with its tb_shapes
    # the bench's weights: full 42-layer spec, seed 1234, post-norm gain 32 (bench.py)
    m = Gemma2Model(random_gemma2(GEMMA2_9B, device=gpu, dtype=torch.bfloat16, seed=1234, post_norm_gain=32.0), gpu)
    yield m
    GD.set_mode(old)
    del m
    torch.cuda.empty_cache()


@pytest.mark.timeout(900)
def test_sweep_9b_reuse_levels_exact(gpu, model9b):
    from taboo_brittleness_amd.config import load_config
    from taboo_brittleness_amd.interp.sae import JumpReLUSAE
    from taboo_brittleness_amd.models.tokenizer import SyntheticTokenizer
    from taboo_brittleness_amd.pipelines.sweep import SweepRunner
    from taboo_brittleness_amd.runtime import gemm_dispatch as GD

    assert GD.mode() == "tb" and GD.describe()["table"], GD.describe()
    cfg = load_config(None, [])                      # the bench's cells: budgets 1..32 x (1 targeted + 10 random), 50 new
    n_cells = len(cfg.intervention.budgets) * (1 + cfg.intervention.random_trials)
    assert n_cells == 66 and cfg.experiment.max_new_tokens == 50
    spec = model9b.spec
    tok = SyntheticTokenizer(vocab_size=spec.vocab_size)
    methods = ("sae_targeted", "sae_random")
    sae = JumpReLUSAE.random(spec.hidden, cfg.sae.d_sae, seed=7, device=gpu)
    # the bench's SAE calibration: thresholds from the baselines of all 30 (word, prompt) templates (bench.py), so
    # about half of the cells diverge from their baselines and take the full-model decode, as in the headline
    cal = SweepRunner(cfg, model9b, tok, sae, batch=40, device=gpu, layer=cfg.model.layer_idx, use_graphs=False,
                      kv_pairs=40)
    tpl = cal.build_pairs(cfg.words, cfg.prompts)
    cal.run_baselines(tpl)
    sae.calibrate(torch.cat([p.resid for p in tpl if p.resid is not None and p.resid.shape[0]], 0))
    del cal, tpl
    t0 = time.perf_counter()

    # ---- every reuse level on, bench-shaped: group A's cells carry group B's baselines in their decode batch
    fast = SweepRunner(cfg, model9b, tok, sae, batch=2 * n_cells + 2 + 8, device=gpu, layer=cfg.model.layer_idx,
                       use_graphs=True, prefix_share=True, layer_resume=True, kv_pairs=8)
    assert fast.trie_decode and fast.skip_noop_spikes and fast.lazy_cum
    pairs = fast.build_pairs(["ship", "moon"], cfg.prompts[:2])      # 4 pairs
    A, B = pairs[:2], pairs[2:]
    fast.run_baselines(A)
    res_a = fast.run_cells_async(A, fast.make_cells(A, methods), ride_along=B).result()
    fast.precapture_graphs()
    res_b = fast.run_cells_async(B, fast.make_cells(B, methods)).result()
    # replay pass: the same cells again through the captured graphs must repeat every record
    res_b2 = fast.run_cells(B, fast.make_cells(B, methods))
    out_fast = {_key(r): r for r in res_a + res_b}
    stats = dict(fast.stats)
    t1 = time.perf_counter()
    print(f"[exact9b] fast path: {len(out_fast)} cells in {t1 - t0:.1f}s, stats {stats}", flush=True)
    assert stats["diverged"] > 0.2 * stats["cells"] and stats["decode_lo_groups"] > 0, stats   # full decode, trie
    assert stats["lens_gemm_rows"] < stats["lens_rows"], stats                 # the lens dedup ran
    rep = compare_records({_key(r): r for r in res_b}, {_key(r): r for r in res_b2}, rtol=0.0)
    assert rep["mismatches"] == 0, rep

    # ---- from scratch: every cell re-prefills its prompt and decodes all blocks, no graphs, other batches / order
    slow = SweepRunner(cfg, model9b, tok, sae, batch=97, device=gpu, layer=cfg.model.layer_idx, use_graphs=False,
                       prefix_share=False, layer_resume=False, kv_pairs=8)
    slow.trie_decode = False
    slow.skip_noop_spikes = False
    spairs = slow.build_pairs(["ship", "moon"], cfg.prompts[:2])
    slow.run_baselines(spairs)                      # SAE already calibrated: the same thresholds
    for p, q in zip(pairs, spairs):                 # the baselines are the same computation at other row counts
        assert p.gen_toks == q.gen_toks, (p.word, p.pidx)
        assert p.spikes_rel == q.spikes_rel and p.targeted == q.targeted and p.top_ids == q.top_ids
        assert list(p.active_pool) == list(q.active_pool)
    cells = list(reversed(slow.make_cells(spairs, methods)))
    res_s = slow.run_cells(spairs, cells)
    out_slow = {_key(r): r for r in res_s}
    t2 = time.perf_counter()
    print(f"[exact9b] scratch path: {len(out_slow)} cells in {t2 - t1:.1f}s", flush=True)
    rep = compare_records(out_fast, out_slow)
    rep.update({"fast_stats": stats, "fast_s": round(t1 - t0, 2), "scratch_s": round(t2 - t1, 2),
                "diverged_frac": round(stats["diverged"] / max(1, stats["cells"]), 4),
                "gemm_dispatch": GD.describe(), "pairs": len(pairs), "cells_per_pair": n_cells,
                "max_new_tokens": cfg.experiment.max_new_tokens, "float_rtol": FLOAT_RTOL})
    print("EXACT9B", json.dumps(rep), flush=True)
    d = _out_dir()
    if d:
        with open(os.path.join(d, "exact_9b_reuse.json"), "w") as f:
            json.dump(rep, f, indent=1)
    assert rep["mismatches"] == 0, rep


def _run_sweep_proc(nproc: int, out: str, log: str, overrides) -> None:
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", TB_GEMM="tb")
    args = ["-m", "taboo_brittleness_amd.cli.run_sweep", "--methods", "all", "--out", out]
    for o in overrides:
        args += ["--set", o]
    launch = [sys.executable]
    if nproc > 1:       # one process per rank; both ranks map to cuda:0 (parallel/dist.py: shared device -> gloo)
        launch += ["-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}", "--master-addr",
                   "127.0.0.1", "--master-port", str(29700 + nproc)]
    cmd = launch + args
    with open(log, "w") as lf:
        r = subprocess.run(cmd, cwd=ROOT, env=env, stdout=lf, stderr=subprocess.STDOUT, timeout=900)
    assert r.returncode == 0, open(log).read()[-4000:]


@pytest.mark.timeout(1200)
def test_sweep_9b_dp2_equals_dp1(gpu, tmp_path):
    """``run_sweep`` (SAE and projection methods) at 9B as DP = 2 -- two processes sharing the GPU, gloo
    collectives, each owning two of the four pairs and all-gathering the baselines the pooled PCA bases / SAE
    calibration need -- gives the records of DP = 1 bit for bit."""
    ov = ["model.arch=gemma2-9b", "word_plurals={ship: [ship, ships], moon: [moon, moons]}",
          "prompts=['Give me a hint!', 'Give me a clue!']", "intervention.budgets=[1, 4, 16]",
          "intervention.random_trials=3", "intervention.ranks=[1, 4]", "intervention.proj_random_trials=2",
          "parallel.backend=gloo", "runtime.batch_size=160"]
    d = _out_dir() or str(tmp_path)
    recs = {}
    import shutil

    for n in (1, 2):
        out = os.path.join(d, f"sweep_9b_dp{n}")     # its event logs double as progress output on a GPU box
        shutil.rmtree(out, ignore_errors=True)        # a stale shard would be resumed instead of recomputed
        _run_sweep_proc(n, out, os.path.join(d, f"run_sweep_9b_dp{n}.log"), ov)
        with open(os.path.join(out, "sweep_cells.jsonl")) as f:
            recs[n] = {_key(r): r for r in map(json.loads, f)}
        print(f"[exact9b] dp{n}: {len(recs[n])} cells", flush=True)
    rep = compare_records(recs[1], recs[2], rtol=0.0)
    print("DP2_VS_DP1", json.dumps(rep), flush=True)
    if _out_dir():
        with open(os.path.join(d, "exact_9b_dp2.json"), "w") as f:
            json.dump(rep, f, indent=1)
    assert len(recs[1]) == 4 * (3 * 4 + 2 * 3) and rep["mismatches"] == 0, rep
