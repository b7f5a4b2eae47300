"""Targeted-vs-random intervention sweep (EP:112-152).

Per (word, prompt) *pair* a baseline hint is generated and read out; per
*cell* — (pair, method ∈ {sae_targeted, sae_random, proj_targeted,
proj_random}, budget m or rank r, trial) — the hint is regenerated with the
edit applied at the pair's spike positions of the hooked layer, then read out:

* content: logit-lens secret probability at the hooked layer over the
  response (mean / final / max) and the LL-Top-k guesses (EP:132);
* fluency: ΔNLL of the *unedited* hint under the edited vs the original model
  (teacher forced, edit at the same positions; EP:136);
* leak: the regenerated hint literally contains the secret (EP:136).

Execution is batched: every batch of cells shares one :class:`Generator`
(one KV cache, hipGraph-captured decode step replayed across batches) and one
persistent edit plan whose tensors are refreshed in place, so capture happens
once per sweep.  Cells are enumerated deterministically and seeded per cell
(SURVEY 7.3.14); data-parallel ranks own whole (word, prompt) pairs -- contiguous
blocks of pairs, every cell of a pair on its pair's rank
(``pipelines.run_sweep.pair_owners``).

Prefix sharing (``runtime.prefix_share``, exact): an edited cell computes
exactly what its pair's baseline computed up to the first edited position f
(same prompt, same greedy tokens, no edit yet).  The baseline's KV cache and
hooked-layer residuals for positions < f are therefore copied (device copies)
instead of recomputed: the cell resumes decoding at f, and the teacher-forced
ΔNLL pass only runs positions ≥ f, adding the baseline's per-token NLLs for
the earlier targets.  Baselines of the *next* pairs ride along in the same
decode batch, so their cost hides behind the cells'.

Layer resume (``_run_batch_resume``) adds three more exact reuse levels that rest on one fact: blocks
``0..l`` (l = hooked layer) see only tokens, the edit only touches the residual after block ``l``.

* prefix-trie decode — diverged cells of a pair with equal tokens since their divergence run blocks
  ``0..l`` once per group (``Generator.decode(share_keys=)``, keys from :meth:`SweepRunner._trie_keys`);
* lens row dedup — their hooked-layer residuals at unedited positions are identical, so those lens rows are
  unembedded once (:meth:`SweepRunner._lens_row_keys`, ``lens_packed(row_key=)``);
* no-op spike skip — a spike where none of a cell's ablated latents fires is an exact no-op edit, decided by
  the edit kernel itself on the baseline's residuals (:meth:`SweepRunner._spike_activity`), so the cell's
  teacher-forced tail starts at its first effective spike (``plan["f"]``).

Module layout: this module holds the runner's driver (construction, baselines, ``run_cells``) and the
summaries; its methods are grouped by phase into mixins -- :mod:`.sweep_plan` (pair scoring, cells, edit bases
and plans, prefetch), :mod:`.sweep_decode` (one batch through the decode: layer resume, prefix-trie keys,
carry-over), :mod:`.sweep_readout` (lens / NLL / leak readouts and records) -- over the data types of
:mod:`.sweep_types`.
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from .. import ops
from ..interp import analysis as A
from ..interp.edits import CaptureHook
from ..interp.logit_lens import lens_packed, lens_readout, reference_exclusions
from ..interp.prompts import hint_prompt_ids
from ..models.tokenizer import secret_token_id
from ..runtime.generation import Generator
from .sweep_decode import DecodeMixin
from .sweep_plan import PlanMixin
from .sweep_readout import ReadoutMixin
from .sweep_types import METHODS, Cell, NextBatch, Pair, _Carry, _Deferred

__all__ = ["METHODS", "Pair", "Cell", "NextBatch", "SweepRunner", "word_targeted_latents", "summarize_cells"]


class SweepRunner(PlanMixin, DecodeMixin, ReadoutMixin):
    def __init__(self, cfg, model, tok, sae, batch: int, device, layer: Optional[int] = None,
                 max_new: Optional[int] = None, use_graphs: bool = True, exclusion: str = "reference",
                 prefix_share: Optional[bool] = None, kv_pairs: int = 64, layer_resume: Optional[bool] = None):
        self.cfg = cfg
        self.m = model
        self.tok = tok
        self.sae = sae
        self.B = batch
        self.dev = torch.device(device)
        self.layer = cfg.model.layer_idx if layer is None else layer
        self.max_new = cfg.experiment.max_new_tokens if max_new is None else max_new
        self.iv = cfg.intervention
        self.exclusion = exclusion
        self.use_graphs = use_graphs
        self.prefix_share = cfg.runtime.prefix_share if prefix_share is None else prefix_share
        self.kv_pairs = kv_pairs
        self.D = model.spec.hidden
        self.gen: Optional[Generator] = None
        self.timings: Dict[str, float] = {}
        self.phase_timing = os.environ.get("TB_PHASE_TIMING", "0") == "1"
        self.host_marks = bool(os.environ.get("TB_PHASE_MARKS")) and not self.phase_timing
        self._kv_next = 0
        self._kv_owner: Dict[int, int] = {}
        self._kv_pair: Dict[int, Pair] = {}
        self._dec_cache: Dict[int, str] = {}
        self.layer_resume = cfg.runtime.layer_resume if layer_resume is None else layer_resume
        # the teacher-forced tail reads its pair's baseline prefix K/V in place (False: copies it into each cell's slot)
        self.tf_prefix = True
        self.stats: Dict[str, int] = {"cells": 0, "diverged": 0, "tf_rows": 0, "lens_rows": 0,
                                      "decode_row_steps": 0, "decode_rows_run": 0, "carried": 0, "staged": 0,
                                      "decode_lo_rows_run": 0, "decode_lo_groups": 0, "lens_gemm_rows": 0}
        # decode-tail carry-over (opt-in; needs ``batch`` to include ``carry_rows`` spare slots): once fewer
        # than ``carry_rows`` diverged cells still decode, the rest continue in the next batch's decode
        # (merged with its new rows) instead of running a long small-batch tail.  Records of carried cells
        # come out with the batch that finishes them; ``run_cells(..., drain=True)`` carries nothing.
        self.carry_rows = 0
        # prefix-trie decode: diverged cells of a pair with equal tokens run blocks 0..l once per group
        # (Generator.decode share_keys); trie_decode = False (bench --no-trie-decode): every row alone
        self.trie_decode = True
        # a cell's teacher-forced tail starts at its first spike with a non-zero edit (earlier spikes: its
        # latents are inactive there, an exact no-op); skip_noop_spikes = False (--no-skip-noop): at its pair's
        # first spike
        self.skip_noop_spikes = True
        self._carry: List[_Carry] = []
        self._next: Optional["NextBatch"] = None      # batch of the next run_cells call (stage_next)
        # lazy running lens sums: a pair's [n + 1, V] fp32 running sums (52 MB at the 256k vocab) are rebuilt from
        # its kept hooked-layer residuals when its cells run, instead of being held from its baseline on (E steps
        # ahead): only the running batch's pairs hold them (~18 GB less at 90 pairs per step); False: held
        self.lazy_cum = True
        self._cum_live: List[Pair] = []
        self._carry_move_pending = None
        self._staged: Optional[dict] = None           # its uploaded plan + queued teacher-forced tail
        self._drain = True
        self._drain_batch = True
        self._with_basis = True

    # ----------------------------------------------------------------- pairs
    def build_pairs(self, words: Sequence[str], prompts: Sequence[str]) -> List[Pair]:
        pairs = []
        for w in words:
            forms = list(self.cfg.word_plurals.get(w, [w]))
            track = [secret_token_id(self.tok, w, "space"), secret_token_id(self.tok, w, "bare")]
            for d in self.iv.decoys.get(w, []):
                track.append(secret_token_id(self.tok, d, "space"))
            for i, p in enumerate(prompts):
                pairs.append(Pair(w, i, p, hint_prompt_ids(self.tok, p), forms, track))
        return pairs

    def _ensure_gen(self, S: int) -> Generator:
        if self.gen is None or self.gen.S < S:
            self.gen = Generator(self.m, self.B, S, use_graphs=self.use_graphs)
            self.store = torch.zeros(self.B, S + 1, self.D, dtype=self.m.dtype, device=self.dev)
            self.capture = CaptureHook(self.store)
            self._plan = None
            self.pair_kv = None
            # a regrown generator has a fresh (zero) pair-KV store: no earlier baseline can be resumed from it
            for p in self._kv_pair.values():
                p.lens_cum = None
            self._kv_owner.clear()
            self._kv_pair.clear()
            if self.prefix_share:
                c = self.gen.cache
                shape = (c.k.shape[0], self.kv_pairs) + tuple(c.k.shape[2:])
                self.pair_kv = (torch.zeros(shape, dtype=c.k.dtype, device=self.dev),
                                torch.zeros(shape, dtype=c.v.dtype, device=self.dev))
                # diverged cells read their shared prefix straight from the pair's KV (no per-cell copy)
                self.gen.enable_kv_prefix(self.pair_kv[0], self.pair_kv[1], self.layer)
        return self.gen

    def precapture_graphs(self) -> int:
        """Capture every decode row-bucket graph now (call after the first batch, once the edit plan
        exists), so later batches never pay a capture."""
        if self.gen is None or getattr(self, "_hook", None) is None:
            return 0
        return self.gen.precapture({self.layer: [self._hook, self.capture]}, "sweep")

    def _S_needed(self, pairs: Sequence[Pair]) -> int:
        return max(p.plen for p in pairs) + self.max_new + 1

    # -------------------------------------------------------------- baseline
    @torch.no_grad()
    def run_baselines(self, pairs: List[Pair], size_for: Sequence[Pair] = ()) -> None:
        """Standalone baseline pass (generation + lens + spikes + scores + NLL) for ``pairs``.  ``size_for``: more
        pairs whose cells will run later (the generator is sized for them now, so it is not regrown — which
        drops the pair-KV store — when they come)."""
        t0 = time.perf_counter()
        self._ensure_gen(self._S_needed(list(pairs) + list(size_for)))
        for c0 in range(0, len(pairs), self.B):
            self.run_cells(pairs, [], ride_along=pairs[c0:c0 + self.B])
        self.timings["baseline_total"] = time.perf_counter() - t0

    def _finalize_baselines(self, chunk: Sequence[Pair], out, lr, rows: Sequence[int],
                            slots: Optional[Sequence[int]] = None) -> None:
        """``rows``: rows of ``out``/``lr``; ``slots``: their KV/capture slots (default = rows)."""
        nll = out.tok_nll.float().cpu().numpy()
        stop = set(int(x) for x in self.gen.stop_ids.tolist())
        slots = list(rows) if slots is None else list(slots)
        kv_dst: List[int] = []
        kv_src: List[int] = []
        for j, (p, i) in enumerate(zip(chunk, rows)):
            si = slots[j]
            p.resp = out.response_ids(i)
            p.leak = None
            p.p_secret_mean = None
            n = len(p.resp)
            full = out.host_tokens()[i].tolist()
            p.gen_toks = full[: n + 1] if out.stopped[i] else full[:n]
            if not p.gen_toks:   # degenerate: nothing generated at all
                p.gen_toks = [next(iter(stop))]
            p.tok_nll = nll[i, : len(p.gen_toks)].copy()
            p.nll = float(p.tok_nll[:n].mean()) if n else float("nan")
            p.p_secret = lr.probs[i][:, 0].copy()
            p.track_probs = lr.probs[i].copy()
            p.top_ids = lr.topk_ids[i]
            p.spikes_rel = A.select_spikes(p.p_secret, p.resp, p.track[:2], self.iv.spikes_k)
            p.resid = self.store[si, p.plen:p.plen + n].clone()
            if self.iv.subspace == "grad_model":     # the prompt positions too: the backward needs the context
                p.resid_pre = self.store[si, :p.plen].clone()
            if self.pair_kv is not None:
                p.kv_slot = self._kv_next % self.kv_pairs
                self._kv_next += 1
                old = self._kv_pair.get(p.kv_slot)
                if old is not None and old is not p:
                    old.lens_cum = None              # its KV is gone: it can no longer be resumed
                self._kv_owner[p.kv_slot] = id(p)
                self._kv_pair[p.kv_slot] = p
                p.lens_cum = lr.cum[i] if lr.cum is not None else None
                kv_dst.append(p.kv_slot)
                kv_src.append(si)
        if kv_dst:       # every layer's K/V of the finished baselines -> their pair-KV slots (2 gathers)
            c = self.gen.cache
            last = dict(zip(kv_dst, kv_src))           # a ring slot reused within one call: last owner wins
            ops.slot_copy(self.pair_kv[0], c.k, list(last.keys()), list(last.values()))
            ops.slot_copy(self.pair_kv[1], c.v, list(last.keys()), list(last.values()))

    def _readout(self, chunk, n_gen, resp_ids, track, seqs=None, keep_cum=False):
        excl = [reference_exclusions(self.tok, r) for r in resp_ids] if self.exclusion == "reference" else None
        return lens_readout(self.m, self.store, [p.plen for p in chunk], list(n_gen), track,
                            top_k=self.cfg.model.top_k, exclusion=self.exclusion, excl_pairs=excl,
                            response_ids=resp_ids, seqs=seqs, keep_cum=keep_cum)

    # -------------------------------------------------------------------- run
    @torch.no_grad()
    def run_cells(self, pairs: List[Pair], cells: Sequence[Cell], measure_nll: Optional[bool] = None,
                  ride_along: Sequence[Pair] = (), drain: bool = True, plan: Optional[dict] = None) -> List[dict]:
        """Run edited cells; ``ride_along`` pairs get their *baseline* generated in the same batch
        (unedited rows), which pipelines the next cells' baselines behind the current ones.
        ``drain=False`` (with ``carry_rows``) lets the last batch's decode tail carry into the next call.
        ``plan``: the host edit plan of ``cells`` from :meth:`prefetch` (single-batch calls only)."""
        measure_nll = self.iv.measure_nll if measure_nll is None else measure_nll
        self._drain = drain
        self._pre_plan = plan
        self._running_cells = cells
        ride = list(ride_along)
        if not cells and not ride:
            return []
        gen = self._ensure_gen(self._S_needed(list(pairs) + ride))
        bases = self._bases(pairs) if any(c.kind == "proj" for c in cells) else {}
        if self._plan is None:
            self._with_basis = any(c.kind == "proj" for c in cells) or bool(self.iv.ranks and not cells)
        elif any(c.kind == "proj" for c in cells) and self._plan.basis is None:
            self._plan = None                                # plan layout changes: rebuild + recapture
            self.gen.invalidate_graph()
            self._with_basis = True
        per = self.B - len(ride)
        assert per > 0 or not cells, "batch too small for the ride-along baselines"
        parts = []
        batches = [list(cells[i:i + per]) for i in range(0, len(cells), per)] or [[]]
        if len(batches) > 1 or len(cells) + len(ride) > self.B:
            self._pre_plan = None
        for bi, batch in enumerate(batches):
            rb = ride if bi == 0 else []
            self._drain_batch = drain or bi + 1 < len(batches)
            parts.append(self._run_batch(pairs, batch, rb, measure_nll, bases))
        self._pre_plan = None
        if getattr(self, "_defer", False):
            return _Deferred(parts)
        return [r for part in parts for r in part]

    def run_cells_async(self, pairs: List[Pair], cells: Sequence[Cell], measure_nll: Optional[bool] = None,
                        ride_along: Sequence[Pair] = (), drain: bool = True, plan: Optional[dict] = None) -> "_Deferred":
        """:meth:`run_cells` whose per-cell result records are assembled on a host worker thread: the
        GPU work (and everything later batches depend on: baselines, spikes, scores, KV) is done when
        this returns, so the caller can launch the next batch while the records of this one are built.
        ``.result()`` returns the records."""
        self._defer = True
        try:
            out = self.run_cells(pairs, cells, measure_nll, ride_along, drain, plan)
        finally:
            self._defer = False
        return out if isinstance(out, _Deferred) else _Deferred([out])

    def _records_pool(self):
        if getattr(self, "_pool", None) is None:
            from concurrent.futures import ThreadPoolExecutor

            self._pool = ThreadPoolExecutor(max_workers=1, thread_name_prefix="tb-records")
        return self._pool

    def _tick(self, name: str) -> None:
        if not self.phase_timing:
            if self.host_marks:      # host-side phase entry times only (no sync): tools/window_gaps.py
                self.__dict__.setdefault("phase_marks", []).append((name, time.monotonic_ns()))
            return
        if self.dev.type == "cuda":
            torch.cuda.synchronize(self.dev)
        now = time.perf_counter()
        last = getattr(self, "_t_last", None)
        if last is not None and name != "start":
            self.timings[name] = self.timings.get(name, 0.0) + (now - last)
        self._t_last = now
        # phase boundaries on the monotonic clock rocprofv3 stamps kernels with (tools/phase_kernels.py)
        self.__dict__.setdefault("phase_marks", []).append((name, time.monotonic_ns()))


def word_targeted_latents(runner: "SweepRunner", word: str, m: int) -> List[int]:
    """Top-``m`` latents of the word-averaged secret score (forcing settings act on the whole model, not on
    one prompt's spikes)."""
    per_prompt = getattr(runner, "word_scores", {}).get(word)
    if not per_prompt:
        return []
    return A.top_latents_from_scores(torch.stack(list(per_prompt.values()), 0).mean(0), m)


def summarize_cells(results: Sequence[dict], words: Sequence[str], word_plurals: Dict[str, List[str]]) -> dict:
    """Curves per (method, budget): means + 95% bootstrap CIs, LL-Top-k Pass@10 / Accuracy / Majority."""
    from ..metrics import bootstrap_ci, calculate_metrics

    groups: Dict[Tuple[str, int], List[dict]] = {}
    for r in results:
        groups.setdefault((r["method"], r["budget"]), []).append(r)
    curves = []
    for (meth, bud), rs in sorted(groups.items()):
        ent = {"method": meth, "budget": bud, "n": len(rs)}
        for key in ("p_secret_mean", "p_secret_final", "delta_nll"):
            vals = [r[key] for r in rs if r[key] == r[key]]
            ent[key] = bootstrap_ci(vals, seed=bud)
        ent["delta_p_secret"] = bootstrap_ci([r["p_secret_mean"] - r["p_secret_mean_base"] for r in rs], seed=bud + 1)
        ent["leak_rate"] = float(np.mean([r["leak"] for r in rs])) if rs else 0.0
        trials = sorted({r["trial"] for r in rs})
        per_trial = []
        for t in trials:
            preds: Dict[str, List[List[str]]] = {w: [] for w in words}
            for r in rs:
                if r["trial"] == t and r["guesses"]:
                    preds.setdefault(r["word"], []).append(r["guesses"])
            per_trial.append(calculate_metrics(preds, list(words), word_plurals)["overall"])
        ent["ll_topk"] = {k: float(np.mean([m[k] for m in per_trial])) for k in per_trial[0]} if per_trial else {}
        curves.append(ent)
    return {"curves": curves}
