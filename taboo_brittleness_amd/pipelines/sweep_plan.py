"""Sweep planning (part of :class:`~.sweep.SweepRunner`): pair scoring (latent secret scores, spike selection,
SAE activity), the cells of a pair (methods x budgets x trials), the edit bases (SAE decoder rows, PCA /
gradient subspaces, random controls) and the per-batch edit plan, its host -> device staging and the
next-batch prefetch (plans built on the host while the GPU runs the current batch).
"""
from __future__ import annotations

import os
import time
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from .. import ops
from ..interp import analysis as A
from ..interp.edits import EditHook, EditPlan
from .sweep_types import METHODS, Cell, NextBatch, Pair, _h2d


class PlanMixin:
    """Methods of :class:`~.sweep.SweepRunner` (state lives on the runner; see its docstring)."""

    @torch.no_grad()
    def _score_pairs(self, pairs: List[Pair]) -> None:
        """Latent secret scores per prompt (EP:118-124) → targeted latent lists; activation-matched random pools."""
        if self.sae is None:
            return
        mmax = max(self.iv.budgets) if self.iv.budgets else 1
        rows, seg, p_all, sp = [], [0], [], []
        live = [p for p in pairs if len(p.resp) > 0]
        for p in live:
            rows.append(p.resid)
            p_all.append(torch.from_numpy(np.asarray(p.p_secret, dtype=np.float32)))
            seg.append(seg[-1] + len(p.resp))
            sp.append(p.spikes_rel)
        if not live:
            return
        R = torch.cat(rows, 0)
        scores = A.latent_scores(self.sae, R, torch.cat(p_all), sp, seg)       # [G, L]
        # word -> {prompt index: latest scores}: a re-scored pair (e.g. after SAE calibration, or a later
        # re-baseline) overwrites its entry, so the word mean is over distinct prompts, never stale ones
        ws = self.__dict__.setdefault("word_scores", {})
        for g, p in enumerate(live):
            ws.setdefault(p.word, {})[p.pidx] = scores[g].clone()
        if self.iv.score_over == "word":
            by_word: Dict[str, List[int]] = {}
            for g, p in enumerate(live):
                by_word.setdefault(p.word, []).append(g)
            for w, gs in by_word.items():
                s = scores[gs].mean(0)
                tl = A.top_latents_from_scores(s, mmax)
                for g in gs:
                    live[g].targeted = tl
        else:
            for p, tl in zip(live, A.top_latents_batch(scores, mmax)):
                p.targeted = tl
        acts = self.sae.encode(R)
        sp_rows = torch.tensor([seg[g] + i for g, p in enumerate(live) for i in p.spikes_rel], device=acts.device)
        sp_grp = torch.tensor([g for g, p in enumerate(live) for _ in p.spikes_rel], device=acts.device)
        active = torch.zeros(len(live), acts.shape[1], dtype=torch.float32, device=acts.device)
        if sp_rows.numel():
            active.index_add_(0, sp_grp, (acts.index_select(0, sp_rows) > 0).float())
        g_idx, l_idx = torch.nonzero(active > 0, as_tuple=True)
        g_h, l_h = g_idx.cpu().numpy(), l_idx.cpu().numpy()
        bounds = np.searchsorted(g_h, np.arange(len(live) + 1))
        for g, p in enumerate(live):
            p.active_pool = l_h[bounds[g]:bounds[g + 1]].astype(np.int64)
        self._spike_activity(live)

    @torch.no_grad()
    def _spike_activity(self, live: Sequence[Pair]) -> None:
        """Where each candidate latent's ablation is a non-zero edit: the latents active at the spikes plus the
        targeted ones, evaluated by the edit kernel itself (``ops.lowrank_edit`` coefficients on copies of the
        baseline's hooked-layer residuals at the spikes — the exact rows and arithmetic the teacher-forced tail
        edits, since blocks ``0..l`` are the baseline's there).  A cell whose latents are all inactive at its
        pair's first spikes leaves those positions bit-identical to the baseline (all-zero edits are no-ops), so
        its tail starts at its first *effective* spike (``_plan_for`` -> ``plan["f"]``)."""
        s, K = self.sae, self.iv.spikes_k
        rows, owner = [], []
        key = self._sae_key()
        for g, p in enumerate(live):
            cand = np.union1d(p.active_pool, np.asarray(p.targeted, np.int64)).astype(np.int64)
            p.act_ids, p.act_mask, p.act_key = cand, np.zeros(cand.size, np.int64), key
            if s is None or p.resid is None or not cand.size:
                continue
            for k, t in enumerate(p.spikes_rel[:K]):
                if 0 <= t < p.resid.shape[0]:
                    for c0 in range(0, cand.size, 256):
                        rows.append((g, t))
                        owner.append((g, k, c0, min(256, cand.size - c0)))
        if not rows or self.iv.alpha == 0:
            return
        n = len(rows)
        idx = np.zeros((n, 256), np.int32)
        cnt = np.zeros(n, np.int32)
        for i, (g, k, c0, m) in enumerate(owner):
            idx[i, :m] = live[g].act_ids[c0:c0 + m]
            cnt[i] = m
        dev = self.dev
        h = torch.stack([live[g].resid[t] for g, t in rows]).contiguous()
        coef = torch.zeros(n, 256, dtype=torch.float32, device=dev)
        ops.lowrank_edit(h, torch.ones(n, dtype=torch.uint8, device=dev), torch.from_numpy(idx).to(dev),
                         torch.from_numpy(cnt).to(dev), s.W_encT, s.W_dec, s.b_enc, s.threshold,
                         s.b_dec if s.apply_b_dec_to_input else None, self.iv.alpha, None, 1e-6, None, coef)
        nz = (coef != 0).cpu().numpy()
        for i, (g, k, c0, m) in enumerate(owner):
            live[g].act_mask[c0:c0 + m] |= nz[i, :m].astype(np.int64) << k

    # ----------------------------------------------------------------- cells
    def make_cells(self, pairs: Sequence[Pair], methods: Sequence[str] = METHODS) -> List[Cell]:
        cells: List[Cell] = []
        base = self.cfg.experiment.seed
        for pi, p in enumerate(pairs):
            for meth in methods:
                if meth.startswith("sae"):
                    if self.sae is None:
                        continue
                    budgets, trials = self.iv.budgets, (1 if meth == "sae_targeted" else self.iv.random_trials)
                else:
                    budgets, trials = self.iv.ranks, (1 if meth == "proj_targeted" else self.iv.proj_random_trials)
                for bud in budgets:
                    for t in range(trials):
                        # replicate 0 keeps the plain key, so sweeps seeded before replicates existed reproduce;
                        # a replicate > 0 (the bench's repeated pairs) draws its own random latent sets / subspaces
                        key = (base, p.word, p.pidx, meth, bud, t) + ((p.rep,) if p.rep else ())
                        cells.append(Cell(pi, meth, int(bud), t, A.cell_seed(*key)))
        return cells

    def _bases(self, pairs: Sequence[Pair]) -> Dict[str, torch.Tensor]:
        """Targeted secret subspaces pooled per word (or across all pairs): PCA of the spike residuals
        (EP:144-146) or, with ``intervention.subspace = grad_lens | grad_model``, the top singular directions of
        the secret-logit gradients at the spikes (EP:146's alternative; interp/gradient.py)."""
        from ..interp import gradient as GR

        rmax = max(self.iv.ranks) if self.iv.ranks else 1
        mode = self.iv.subspace
        if mode not in ("pca", "grad_lens", "grad_model"):
            raise ValueError(f"intervention.subspace must be pca, grad_lens or grad_model, not {mode!r}")
        # the bases depend only on the pairs' kept baseline residuals (identity-keyed: a re-run baseline makes a
        # new tensor) and the subspace settings; run_sweep passes every pair on every chunk and the staged plan
        # asks again, so the gradient forward/backward passes run once per pair set
        ckey = (mode, self.iv.pca_pool, rmax, tuple((id(p), id(p.resid), tuple(p.spikes_rel or ())) for p in pairs))
        cache = getattr(self, "_bases_cache", None)
        if cache is not None and cache[0] == ckey:
            return cache[1]
        out = self._bases_compute(pairs, mode, rmax)
        self._bases_cache = (ckey, out, [p.resid for p in pairs])   # refs held: the ids cannot be reused
        return out

    def _bases_compute(self, pairs: Sequence[Pair], mode: str, rmax: int) -> Dict[str, torch.Tensor]:
        from ..interp import gradient as GR

        groups: Dict[str, List[torch.Tensor]] = {}
        for p in pairs:
            if p.resid is None or not p.spikes_rel:
                continue
            key = p.word if self.iv.pca_pool == "word" else "__all__"
            if mode == "pca":
                groups.setdefault(key, []).append(p.resid[p.spikes_rel].float())
            elif mode == "grad_lens":
                groups.setdefault(key, []).append(GR.lens_gradients(self.m, p.resid[p.spikes_rel], p.track[:1]))
            else:
                pre = getattr(p, "resid_pre", None)
                assert pre is not None, "grad_model subspaces need the baselines run with subspace=grad_model"
                assert getattr(self.m, "tp", None) is None and getattr(self.m, "lora", None) is None, \
                    "grad_model needs unsharded, merged weights"
                seq = torch.cat([pre, p.resid], 0)
                sp = [p.plen + t for t in p.spikes_rel]
                groups.setdefault(key, []).append(GR.model_gradients(self.m, seq, self.layer, sp, p.track[:1]))
        if mode == "pca":
            return {k: A.secret_subspace(torch.cat(v, 0), rmax) for k, v in groups.items()}
        return {k: GR.gradient_subspace(torch.cat(v, 0), rmax, seed=A.cell_seed("grad", k, rmax))
                for k, v in groups.items()}

    def _plan_for(self, cells: Sequence[Cell], pairs: Sequence[Pair], bases: Dict[str, torch.Tensor],
                  with_carry: bool = True):
        """Host-side plan of a batch: int arrays (one row per cell, cell ``i`` = row/slot ``i``) plus the
        projection basis rows to upload (row ``i * rmax + j`` = j-th direction of proj cell ``i``)."""
        K = self.iv.spikes_k
        mmax = max([max(self.iv.budgets or [1]), max(self.iv.ranks or [1])])
        rmax = max(self.iv.ranks) if self.iv.ranks else 1
        B = self.B
        sp = np.full((B, K), -1, dtype=np.int32)
        ix = np.zeros((B, mmax), dtype=np.int32)
        cn = np.zeros(B, dtype=np.int32)
        kd = np.zeros(B, dtype=np.int8)
        tgt: Dict[str, Tuple[List[int], List[int]]] = {}   # pooled basis -> (table rows, its rows)
        rproj: Tuple[List[int], List[int], List[int]] = ([], [], [])   # random controls: (first row, rank, seed)
        by_pair: Dict[int, List[int]] = {}
        for ci, c in enumerate(cells):
            by_pair.setdefault(c.pair, []).append(ci)
        for pi, cis in by_pair.items():
            p = pairs[pi]
            s_abs = p.spikes_abs[:K]
            ca = np.asarray(cis)
            if s_abs:
                sp[ca, : len(s_abs)] = s_abs
            rnd = [ci for ci in cis if cells[ci].kind == "sae" and cells[ci].method != "sae_targeted"]
            if rnd:
                got = A.random_latents_batch(self.sae.d_sae, [cells[ci].budget for ci in rnd],
                                             [cells[ci].seed for ci in rnd],
                                             [p.targeted[: cells[ci].budget] for ci in rnd], pool=p.active_pool)
                for ci, g in zip(rnd, got):
                    ix[ci, : len(g)] = g
                    cn[ci] = len(g)
                kd[rnd] = 1
            tg = np.asarray(p.targeted[:mmax], dtype=np.int32)
            for ci in cis:
                c = cells[ci]
                if c.kind == "sae":
                    if c.method == "sae_targeted":
                        n = min(c.budget, tg.size)
                        ix[ci, :n] = tg[:n]
                        cn[ci] = n
                        kd[ci] = 1
                else:
                    if c.method == "proj_targeted":
                        bk = p.word if self.iv.pca_pool == "word" else "__all__"
                        r = min(c.budget, int(bases[bk].shape[0]))
                        dst, src = tgt.setdefault(bk, ([], []))
                        dst.extend(range(ci * rmax, ci * rmax + r))
                        src.extend(range(r))
                    else:
                        r = c.budget
                        rproj[0].append(ci * rmax)
                        rproj[1].append(r)
                        rproj[2].append(c.seed)
                    ix[ci, :r] = np.arange(ci * rmax, ci * rmax + r)
                    cn[ci] = r
                    kd[ci] = 2
        basis = None
        # largest rank first (a basis costs ~r^2 block reductions; the workgroups are dispatched in order)
        lpt = np.argsort(-np.asarray(rproj[1], np.int64), kind="stable")
        if tgt or rproj[0]:       # filled on the device by _load_plan: gathers of the pooled bases + random_basis
            basis = {"tgt": {k: (np.asarray(d, np.int64), np.asarray(sr, np.int64)) for k, (d, sr) in tgt.items()},
                     "bases": {k: bases[k] for k in tgt},
                     "rnd": tuple(np.asarray(v, t)[lpt] for v, t in zip(rproj, (np.int64, np.int32, np.int64)))}
        plan = {"spikes": sp, "kind": kd, "idx": ix, "cnt": cn, "basis": basis, "rows": B * rmax, "rmax": rmax,
                "f": self._effective_first_edit(cells, pairs, by_pair, kd, ix, cn)}
        return self._plan_add_carry(plan) if with_carry else plan

    def _sae_key(self) -> Optional[tuple]:
        """Identity + in-place version of the SAE tensors an edit's coefficients depend on: an activity table
        built under other parameters (e.g. before ``calibrate()``) is never used."""
        s = self.sae
        if s is None:
            return None
        ts = [s.W_encT, s.b_enc, s.threshold] + ([s.b_dec] if s.apply_b_dec_to_input else [])
        return tuple((id(t), t._version) for t in ts) + (getattr(s, "param_version", 0), float(self.iv.alpha))

    def _effective_first_edit(self, cells, pairs, by_pair, kd, ix, cn) -> np.ndarray:
        """Per cell (plan row): response index of its first spike where the edit is non-zero (the pair's spike
        order), ``len(resp)`` if it never is (the cell is its baseline), -1 = the pair's first spike (projection
        cells, or no activity table).  Latents outside a pair's activity table count as active everywhere."""
        K = self.iv.spikes_k
        f = np.full(self.B, -1, np.int64)
        if not self.skip_noop_spikes:
            return f
        key = self._sae_key()
        for pi, cis in by_pair.items():
            p = pairs[pi]
            ids, msk = p.act_ids, p.act_mask
            if p.act_key != key:
                continue                        # stale or missing table: every cell edits from the first spike
            sp = np.asarray(p.spikes_rel[:K], np.int64)
            ca = np.asarray([ci for ci in cis if kd[ci] == 1], np.int64)
            if ids is None or not ca.size or not sp.size:
                continue
            lat = ix[ca].astype(np.int64)
            j = np.minimum(np.searchsorted(ids, lat), max(ids.size - 1, 0))
            found = (ids[j] == lat) if ids.size else np.zeros(lat.shape, bool)
            allk = (1 << sp.size) - 1
            bits = np.where(found, msk[j] if ids.size else 0, allk)
            bits = np.where(np.arange(lat.shape[1])[None, :] < cn[ca][:, None], bits, 0)
            cell_bits = np.bitwise_or.reduce(bits, axis=1)
            on = (cell_bits[:, None] >> np.arange(sp.size)[None, :]) & 1
            f[ca] = np.where(on.astype(bool), sp[None, :], len(p.resp)).min(1)
        return f

    def _plan_add_carry(self, plan: dict) -> dict:
        for cr in self._carry:                  # carried cells keep editing at their carry-region slots
            cs_, ck_, ci_, cc_ = cr.plan_row
            plan["spikes"][cr.slot] = cs_
            plan["kind"][cr.slot] = ck_
            plan["idx"][cr.slot] = ci_
            plan["cnt"][cr.slot] = cc_
        return plan

    def prefetch(self, pairs: Sequence[Pair], methods: Sequence[str] = METHODS):
        """Build a future step's cells and host edit plan on a helper thread (pure host work: cell
        enumeration, seeded random latent sets, plan arrays) while the GPU runs the current step.
        Needs the pairs' baselines (spikes, targeted latents) to be final.  Pass the result to
        :meth:`run_cells` / :meth:`run_cells_async` as ``prefetched``; ``None`` if it cannot apply."""
        if not pairs or any(p.resid is None for p in pairs):
            return None
        if any(not m.startswith("sae") for m in methods):
            # projection cells: their plan needs the pooled PCA bases (device work, main thread); the cells are
            # enumerated here (the random-control bases are drawn on the device when the plan loads)
            if getattr(self, "_prefetch_pool", None) is None:
                from concurrent.futures import ThreadPoolExecutor

                self._prefetch_pool = ThreadPoolExecutor(max_workers=1, thread_name_prefix="tb-prefetch")
            return self._prefetch_pool.submit(lambda: (self.make_cells(pairs, methods), None))
        if getattr(self, "_prefetch_pool", None) is None:
            from concurrent.futures import ThreadPoolExecutor

            self._prefetch_pool = ThreadPoolExecutor(max_workers=1, thread_name_prefix="tb-prefetch")

        def work():
            t0 = time.perf_counter()
            cells = self.make_cells(pairs, methods)
            t1 = time.perf_counter()
            out = (cells, None) if len(cells) > self.B else (cells, self._plan_for(cells, pairs, {}, with_carry=False))
            t2 = time.perf_counter()
            self.timings["prefetch_cells"] = self.timings.get("prefetch_cells", 0.0) + t1 - t0
            self.timings["prefetch_plan"] = self.timings.get("prefetch_plan", 0.0) + t2 - t1
            return out
        return self._prefetch_pool.submit(work)

    def _load_plan(self, plan: dict) -> EditHook:
        """Upload into the persistent plan (fixed tensors, so a captured decode graph stays valid)."""
        dev = self.dev
        if self._plan is None:
            t = lambda a: torch.from_numpy(a).to(dev)   # noqa: E731
            basis = torch.zeros(plan["rows"], self.D, dtype=torch.float32, device=dev) if self._with_basis else None
            self._plan = EditPlan(t(plan["spikes"]), t(plan["kind"]), t(plan["idx"]), t(plan["cnt"]), self.iv.alpha,
                                  basis)
            self._hook = EditHook(self._plan, self.sae)
        else:
            for f in ("spikes", "kind", "idx", "cnt"):
                getattr(self._plan, f).copy_(_h2d(plan[f], dev), non_blocking=True)
        if plan["basis"] is not None:
            assert self._plan.basis is not None, "projection cells need a plan built with a basis table"
            pb, tab = plan["basis"], self._plan.basis
            up = lambda a: _h2d(a, dev).to(dev, non_blocking=True)   # noqa: E731
            for bk, (dst, src) in pb["tgt"].items():
                U = pb["bases"][bk]          # pooled bases live on the host (one small upload per basis and batch)
                U = (up(U) if U.device.type == "cpu" else U).float()
                tab.index_copy_(0, up(dst), U.index_select(0, up(src)))
            rows, ranks, seeds = pb["rnd"]
            if rows.size:
                ops.random_basis(up(seeds), up(ranks), up(rows), tab)
        return self._hook

    # ---------------------------------------------------- cross-batch pipeline
    def stage_next(self, nb: "NextBatch") -> None:
        """Announce the batch the next :meth:`run_cells` call will run.  Once this batch's readout is
        queued, its edit plan is uploaded and its teacher-forced tail is queued behind it on the GPU
        (:meth:`_launch_staged_next`), so the device never idles while the host builds this batch's
        records and the next batch's decode rows.  Exact: the tail only writes the next cells' KV slots
        (blocks after the hooked layer) and capture rows, which this batch no longer reads once its lens
        is queued; stream order does the rest."""
        self._next = nb

    def _launch_staged_next(self) -> None:
        nb = getattr(self, "_next", None)
        self._next = None
        if nb is not None and nb.cells is not None and nb.cells is getattr(self, "_running_cells", None):
            nb = None                            # announced batch is the one running now: nothing to stage
        # carried decode rows move out of the cell slots before the next tail writes them (stream order)
        mv = self._carry_move_pending
        self._carry_move_pending = None
        if mv is not None:
            mv()
        if nb is None or not (self.layer_resume and self.prefix_share):
            return
        nb.resolve(self)
        cp = [nb.pairs[c.pair] for c in nb.cells]
        proj = any(c.kind == "proj" for c in nb.cells)
        if not nb.cells or len(nb.cells) > self.B or not self._resumable(cp) or \
                (proj and (self._plan is None or self._plan.basis is None)):
            return
        if nb.plan is None:      # bases pooled over the call's pairs, as run_cells computes them
            nb.plan = self._plan_for(nb.cells, nb.pairs, self._bases(nb.pairs) if proj else {}, with_carry=False)
        plan = nb.plan
        nb.plan = plan
        if self._carry:                          # the next decode continues this batch's carried rows
            plan = self._plan_add_carry({k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in plan.items()})
        self._set_adapters(cp)
        hook = self._load_plan(plan)
        tf = self._tf_launch(cp, {self.layer: [hook, self.capture]}, plan.get("f"))
        self._staged = {"cells": nb.cells, "plan": plan, "tf": tf, "carry": list(self._carry)}
        self._tick("next_tf_launched")
