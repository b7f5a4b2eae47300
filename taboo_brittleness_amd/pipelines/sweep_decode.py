"""Sweep decode (part of :class:`~.sweep.SweepRunner`): one batch of edited cells -- layer resume from the pair's
baseline residual, the prefix-shared KV, prefix-trie keys, decode-tail carry-over, the ride-along baselines --
through the hipGraph decode of :class:`~..runtime.generation.Generator`.
"""
from __future__ import annotations

import os
import time
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from .. import ops
from ..interp import analysis as A
from ..runtime.generation import Generator
from .sweep_types import Pair, _Carry, _h2d


class DecodeMixin:
    """Methods of :class:`~.sweep.SweepRunner` (state lives on the runner; see its docstring)."""

    # --------------------------------------------------------- prefix sharing
    def _copy_pair_kv(self, rows: Sequence[int], kv_slots: Sequence[int], layers: Optional[Sequence[int]] = None) -> None:
        if not len(rows):
            return
        c = self.gen.cache
        if layers is not None and not len(layers):
            return
        layers = range(c.k.shape[0]) if layers is None else range(min(layers), max(layers) + 1)
        ops.slot_copy(c.k, self.pair_kv[0], list(rows), list(kv_slots), layers)
        ops.slot_copy(c.v, self.pair_kv[1], list(rows), list(kv_slots), layers)

    def _copy_pair_resid(self, rows: Sequence[int], cell_pairs: Sequence[Pair]) -> None:
        """store[row, plen + t] = pair.resid[t] for t < first edited response index."""
        S1 = self.store.shape[1]
        uniq: Dict[int, int] = {}
        srcs = []
        off = 0
        for p in cell_pairs:
            if id(p) not in uniq and p.resid is not None and p.resid.shape[0]:
                uniq[id(p)] = off
                srcs.append(p.resid)
                off += p.resid.shape[0]
        if not srcs:
            return
        src_all = torch.cat(srcs, 0)
        di, si = [], []
        for b, p in zip(rows, cell_pairs):
            if id(p) not in uniq:
                continue
            n = min(p.first_edit, len(p.resp))
            for t in range(n):
                di.append(b * S1 + p.plen + t)
                si.append(uniq[id(p)] + t)
        if di:
            self.store.view(-1, self.D).index_copy_(
                0, torch.tensor(di, device=self.dev), src_all.index_select(0, torch.tensor(si, device=self.dev)))

    def _resumable(self, cell_pairs: Sequence[Pair]) -> bool:
        return self.layer_resume and self.prefix_share and bool(cell_pairs) and all(
            p.kv_slot >= 0 and self._kv_owner.get(p.kv_slot) == id(p) and
            (p.lens_cum is not None or self.lazy_cum) and p.resid is not None for p in cell_pairs)

    def _set_adapters(self, slot_pairs: Sequence[Pair]) -> None:
        """Slot ``i`` runs the LoRA adapter of ``slot_pairs[i]``'s word (multi-adapter bank)."""
        bank = getattr(self.m, "lora", None)
        if bank is None or not slot_pairs:
            return
        ids = [bank.names.index(p.word) if p.word in bank.names else -1 for p in slot_pairs]
        self.gen.cache.adapter[: len(ids)].copy_(torch.tensor(ids, dtype=torch.int32))

    def _run_batch(self, pairs, batch, rb, measure_nll, bases) -> List[dict]:
        self._set_adapters([pairs[c.pair] for c in batch] + list(rb))
        if self._resumable([pairs[c.pair] for c in batch]):
            return self._run_batch_resume(pairs, batch, rb, measure_nll, bases)
        assert not self._carry, "carried cells need the layer-resume path (drain before switching)"
        gen = self.gen
        self._tick("start")
        nc = len(batch)
        rows_pairs = [pairs[c.pair] for c in batch] + list(rb)
        n = len(rows_pairs)
        hook = self._load_plan(self._plan_for(batch, pairs, bases))
        hooks = {self.layer: [hook, self.capture]}
        cell_pairs = rows_pairs[:nc]
        self._tick("plan")
        share = self.prefix_share and nc > 0 and all(
            p.kv_slot >= 0 and self._kv_owner.get(p.kv_slot) == id(p) for p in cell_pairs)
        if share:
            self._copy_pair_kv(range(nc), [p.kv_slot for p in cell_pairs])
            self._copy_pair_resid(range(nc), cell_pairs)
            starts, prefix, toks, steps, c0s = [], [], [], 1, []
            pnll = torch.zeros(n, max(len(p.gen_toks) for p in cell_pairs) if cell_pairs else 1)
            for b, p in enumerate(cell_pairs):
                i = min(p.first_edit, len(p.gen_toks) - 1)
                starts.append(p.plen + i)
                prefix.append(p.gen_toks[: i + 1])
                toks.append(p.gen_toks[i])
                c0s.append(i + 1)
                pnll[b, : i + 1] = torch.from_numpy(p.tok_nll[: i + 1])
                steps = max(steps, self.max_new - i)
            if rb:
                first = gen.prefill([p.ids for p in rb], list(range(nc, n)), hooks)
                fl = first.tolist()
                for j, p in enumerate(rb):
                    starts.append(p.plen)
                    prefix.append([fl[j]])
                    toks.append(fl[j])
                steps = self.max_new
                pnll[nc:, :1] = gen.out_nll[nc:n, :1].cpu()
            self._tick("prefix_copy+prefill")
            gen.decode(torch.tensor(toks, dtype=torch.int32), starts, prefix, steps, n, hooks, "sweep",
                       prefix_nll=pnll.to(self.dev), teacher=[p.resp for p in cell_pairs])
            out = gen.collect(n, self.max_new, [p.plen for p in rows_pairs])
        else:
            c0s = [0] * nc
            out = gen.generate([p.ids for p in rows_pairs], self.max_new, hooks=hooks, graph_key="sweep",
                               teacher=[p.resp for p in cell_pairs])
        self._tick("decode")
        resp = [out.response_ids(i) for i in range(n)]
        lr = self._readout(rows_pairs, out.n_gen, resp, [p.track for p in rows_pairs],
                           keep_cum=bool(rb) and self.layer_resume and self.prefix_share and not self.lazy_cum)
        self._tick("lens")
        if rb:
            self._finalize_baselines(rb, out, lr, list(range(nc, n)))
            self._score_pairs(list(rb))
        self._tick("baseline_finalize")
        if measure_nll and nc:
            nll = self._nll_cells(cell_pairs, hook, out, c0s)
        else:
            nll = [float("nan")] * nc
        self._tick("nll")
        self_nll = out.tok_nll.float().cpu().numpy()
        results = []
        for i, c in enumerate(batch):
            p = pairs[c.pair]
            results.append(self._cell_result(
                c, p, out.n_gen[i], resp[i], lr.probs[i], lr.topk_ids[i], nll[i],
                float(self_nll[i, : out.n_gen[i]].mean()) if out.n_gen[i] else float("nan")))
        self._tick("results")
        return results

    # ------------------------------------------------------------ layer resume
    def _run_batch_resume(self, pairs, batch, rb, measure_nll, bases) -> List[dict]:
        """Exact layer-resume execution of a batch of edited cells (prefix sharing taken to its limit).

        While a cell's tokens equal its baseline's, blocks ``0..l`` (``l`` = hooked layer) compute exactly
        what the baseline computed — same tokens, and the edit only touches the residual *after* block
        ``l`` — so their KV and the hooked residual are the baseline's.  Per cell:

        1. teacher-forced tail: one packed forward of blocks ``l+1..`` over response positions
           ``f..E`` (``f`` = first edit), fed the baseline's hooked-layer residuals, with the edit
           applied at the spikes.  Its logits give, for every position, the teacher-forced NLL of the
           baseline's next token (the ΔNLL, EP:136, with no separate pass) and the cell's own greedy
           choice;
        2. the first position whose greedy choice differs from the baseline's token is the divergence
           ``D``; only diverged cells decode (all blocks) from ``D``, batched with the ride-along
           baselines in a row-bucketed hipGraph;
        3. the response lens sum reuses the baseline's running sums (``Pair.lens_cum``) for positions
           before ``D`` that are not spikes, and only evaluates the lens at spikes and at ``>= D``.
        """
        gen, m = self.gen, self.m
        self._tick("start")
        nc = len(batch)
        cell_pairs = [pairs[c.pair] for c in batch]
        rb = list(rb)
        nr = len(rb)
        l0, L = self.layer, m.spec.layers
        staged = self._staged
        self._staged = None
        if staged is not None and (len(staged["cells"]) != len(batch) or
                                   len(staged["carry"]) != len(self._carry) or
                                   any(a is not b for a, b in zip(staged["carry"], self._carry)) or
                                   any(a is not b for a, b in zip(staged["cells"], batch))):
            staged = None                       # staged for another batch: its writes are simply overwritten
        if staged is not None:                  # plan uploaded and teacher-forced tail queued by the last batch
            self.stats["staged"] += 1
            plan = staged["plan"]
            hooks = {self.layer: [self._hook, self.capture]}
            self._tick("plan")
        else:
            pre = getattr(self, "_pre_plan", None)
            plan = self._plan_add_carry(pre) if pre is not None else self._plan_for(batch, pairs, bases)
            self._tick("plan_host")
            hook = self._load_plan(plan)
            hooks = {self.layer: [hook, self.capture]}
            self._tick("plan")
        # blocks > l read the pair's baseline KV below the first edit in place (no per-cell copy), or copy
        # it into each cell's slot first (SweepRunner.tf_prefix = False)
        if not self.tf_prefix:
            self._copy_pair_kv(range(nc), [p.kv_slot for p in cell_pairs], layers=range(l0 + 1, L))
        self._tick("kv_copy")
        tf = self._tf_finish(staged["tf"] if staged is not None else self._tf_launch(cell_pairs, hooks, plan.get("f")))
        self._tick("tf_pass")
        # ---- divergence point D of every cell: first tail row whose greedy token leaves the baseline's
        D_a = np.full(nc, -1, np.int64)
        if tf["nxt"].size:
            mism = (tf["nxt"] != tf["tgt"]) & (tf["tgt"] >= 0)
            rows = np.nonzero(mism)[0]
            if rows.size:
                cells_hit, first = np.unique(tf["row_cell"][rows], return_index=True)
                D_a[cells_hit] = tf["row_t"][rows[first]] + 1
        D: List[Optional[int]] = [None if d < 0 else int(d) for d in D_a.tolist()]
        # diverged cells, earliest divergence (= most decode steps) first: the decode shrinks its row
        # count as the later-diverging rows complete (Generator.decode row_steps)
        div_a = np.nonzero(D_a >= 0)[0]
        div_a = div_a[np.argsort(D_a[div_a], kind="stable")]
        div = div_a.tolist()
        self.stats["cells"] += nc
        self.stats["diverged"] += len(div)
        # diverged cells decode every block from D.  Their attention reads the prefix the baseline
        # computed straight from the pair's KV slot: blocks <= l for positions < plen + D (same tokens,
        # no edit yet), blocks > l for positions < plen + f (before the first edit); the blocks > l
        # keys in [plen + f, plen + D) are the teacher-forced tail's, already in the cell's own slot.
        # ---- per-cell teacher-forced numbers (complete for every cell, vectorised): edit NLL, and the
        # self NLL of cells whose tokens never left the baseline's
        seg = tf["seg"]
        upairs, up = tf["upairs"], tf["up"]
        f_a, r0_a = tf["f"], tf["r0"]
        U = len(upairs)
        Gm = max([1] + [len(q.gen_toks) for q in upairs])
        ntab = np.zeros((max(U, 1), Gm + 1), np.float64)     # per pair: cumulative baseline token NLLs
        for u, q in enumerate(upairs):
            ntab[u, 1: len(q.tok_nll) + 1] = np.cumsum(q.tok_nll, dtype=np.float64)
        n_a = np.asarray([len(q.resp) for q in upairs], np.int64)[up] if nc else np.zeros(0, np.int64)
        ns_cs = np.concatenate([[0.0], np.cumsum(tf["nll_self"], dtype=np.float64)])
        nt_cs = np.concatenate([[0.0], np.cumsum(tf["nll_tgt"], dtype=np.float64)])
        ntail = np.maximum(0, n_a - 1 - f_a)
        base_self = ntab[up, np.minimum(f_a + 1, n_a)] if nc else np.zeros(0)
        inv_n = np.where(n_a > 0, 1.0 / np.maximum(n_a, 1), np.nan)
        sn_v = (base_self + ns_cs[r0_a + ntail] - ns_cs[r0_a]) * inv_n
        nll_v = (base_self + nt_cs[r0_a + ntail] - nt_cs[r0_a]) * inv_n if measure_nll else np.full(nc, np.nan)
        nll_c, sn_c = nll_v.tolist(), sn_v.tolist()
        # ---- decode rows: ride-along baselines (slots nc..), then the diverged cells (slot b) and cells
        # carried over from the previous batch (carry-region slots), longest remaining decode first
        R_start, R_tok, R_slot, R_steps, R_ps, R_lo, R_hi, R_pref, R_nll = [], [], [], [], [], [], [], [], []
        if nr:
            first = gen.prefill([p.ids for p in rb], list(range(nc, nc + nr)), hooks, out_rows=list(range(nr)))
            fl = np.asarray(first.tolist(), np.int64)
            z = np.zeros(nr, np.int64)
            R_start.append(np.asarray([p.plen for p in rb], np.int64))
            R_tok.append(fl)
            R_slot.append(np.arange(nc, nc + nr, dtype=np.int64))
            R_steps.append(np.full(nr, self.max_new, np.int64))
            R_ps.append(z)
            R_lo.append(z)
            R_hi.append(z)
            R_pref.append([[int(t)] for t in fl.tolist()])
            R_nll.append(None)                  # their first NLL comes from the prefill (out_nll[:, 0])
        n_ride_rows = nr
        # new diverged rows, vectorised over cells
        nd = div_a.size
        ud = up[div_a] if nd else np.zeros(0, np.int64)
        Dd, fd, rd = D_a[div_a], f_a[div_a], r0_a[div_a]
        plen_u = np.asarray([q.plen for q in upairs], np.int64)
        kv_u = np.asarray([q.kv_slot for q in upairs], np.int64)
        e_d = tf["nxt"][rd + Dd - 1 - fd].astype(np.int64) if nd else np.zeros(0, np.int64)
        Wn = int(Dd.max()) + 1 if nd else 1
        col = np.arange(Wn)[None, :]
        gt = tf["gtab"]
        pref_d = np.where(col < Dd[:, None], gt[ud][:, :Wn] if gt.shape[1] >= Wn else
                          np.pad(gt[ud], ((0, 0), (0, Wn - gt.shape[1])))[:, :Wn], self.gen.pad_id)
        pref_d = np.where(col == Dd[:, None], e_d[:, None], pref_d)
        nllm_d = np.zeros((nd, Wn), np.float32)
        if nd:
            tokn = np.zeros((U, Gm), np.float32)
            for u, q in enumerate(upairs):
                tokn[u, : len(q.tok_nll)] = q.tok_nll
            cmat = np.broadcast_to(col, (nd, Wn))
            base_part = tokn[ud][:, :Wn] if Gm >= Wn else np.pad(tokn[ud], ((0, 0), (0, Wn - Gm)))
            tail_idx = np.clip(rd[:, None] + cmat - fd[:, None] - 1, 0, max(0, tf["nll_self"].size - 1))
            tail_part = tf["nll_self"][tail_idx] if tf["nll_self"].size else np.zeros((nd, Wn), np.float32)
            nllm_d = np.where(cmat <= fd[:, None], base_part, np.where(cmat <= Dd[:, None], tail_part, 0.0))
        steps_d = np.maximum(1, self.max_new - Dd)
        carry_in = self._carry
        self._carry = []
        # merge with carried rows: stable by remaining steps, new rows before carried ones on ties
        c_steps = np.asarray([cr.steps for cr in carry_in], np.int64)
        allsteps = np.concatenate([steps_d, c_steps])
        order = np.argsort(-allsteps, kind="stable")
        row_src = [("new", int(div_a[i])) if i < nd else ("carry", carry_in[i - nd]) for i in order.tolist()]
        cat = lambda a, b: np.concatenate([a, np.asarray(b, np.int64)])[order]   # noqa: E731
        R_start.append(cat(plen_u[ud] + Dd, [cr.pos for cr in carry_in]))
        R_tok.append(cat(e_d, [cr.tok for cr in carry_in]))
        R_slot.append(cat(div_a, [cr.slot for cr in carry_in]))
        R_steps.append(allsteps[order])
        R_ps.append(cat(kv_u[ud], [cr.pre[0] for cr in carry_in]))
        R_lo.append(cat(plen_u[ud] + Dd, [cr.pre[1] for cr in carry_in]))
        R_hi.append(cat(plen_u[ud] + fd, [cr.pre[2] for cr in carry_in]))
        if carry_in:
            Wc = max([Wn] + [len(cr.prefix) for cr in carry_in])
            pm = np.full((nd + len(carry_in), Wc), self.gen.pad_id, np.int64)
            nm = np.zeros((nd + len(carry_in), Wc), np.float32)
            pm[:nd, :Wn], nm[:nd, :Wn] = pref_d, nllm_d
            for i, cr in enumerate(carry_in):
                pm[nd + i, : len(cr.prefix)] = cr.prefix
                nm[nd + i, : len(cr.prefix_nll)] = cr.prefix_nll
            lens_all = np.concatenate([Dd + 1, [len(cr.prefix) for cr in carry_in]])
            R_pref.append((pm[order], lens_all[order]))
            R_nll.append(nm[order])
        else:
            R_pref.append((pref_d, Dd + 1))
            R_nll.append(nllm_d)
        starts = np.concatenate(R_start) if R_start else np.zeros(0, np.int64)
        toks = np.concatenate(R_tok) if R_tok else np.zeros(0, np.int64)
        slots = np.concatenate(R_slot) if R_slot else np.zeros(0, np.int64)
        rsteps = np.concatenate(R_steps) if R_steps else np.zeros(0, np.int64)
        pre_slot, pre_lo, pre_hi = (np.concatenate(x) for x in (R_ps, R_lo, R_hi))
        steps = int(rsteps.max()) if rsteps.size else 0
        nrows = len(slots)
        self._tick("prefill")
        out = None
        ran = steps
        carry_move = None
        if nrows:
            nr_here = nr
            pm, lens_c = R_pref[-1]
            nm = R_nll[-1]
            Wp = max(1, pm.shape[1])
            pref_all = np.full((nrows, Wp), self.gen.pad_id, np.int64)
            lens_all = np.ones(nrows, np.int64)
            pref_all[nr_here:, : pm.shape[1]] = pm
            lens_all[nr_here:] = lens_c
            if nr_here:
                pref_all[:nr_here, 0] = R_tok[0]
            pnll = torch.zeros(nrows, Wp, dtype=torch.float32, device=self.dev)
            if nr_here:
                pnll[:nr_here, :1] = gen.out_nll[:nr_here, :1]
            if nm.size:
                pnll[nr_here:, : nm.shape[1]] = _h2d(np.ascontiguousarray(nm, dtype=np.float32),
                                                    self.dev).to(self.dev, non_blocking=True)
            carry_ok = (self.carry_rows > 0 and not self._drain_batch and n_ride_rows == 0)
            skeys = self._trie_keys(nr_here, [carry_in[i - nd] if i >= nd else int(e_d[i]) for i in order.tolist()],
                                    pre_slot[nr_here:], pre_lo[nr_here:], starts[nr_here:])
            ran = gen.decode(torch.from_numpy(toks.astype(np.int32)), starts, (pref_all, lens_all), max(steps, 1),
                             nrows, hooks, "sweep", prefix_nll=pnll, slots=slots, row_steps=rsteps,
                             prefix_rows=(pre_slot, pre_lo, pre_hi),
                             stop_below=self.carry_rows if carry_ok else 0,
                             min_steps=max([cr.steps for cr in carry_in] + [0]),
                             share_keys=skeys, share_split=self.layer if skeys is not None else None)
            if skeys is not None:
                self.stats["decode_lo_rows_run"] += gen.last_rows_lo
                self.stats["decode_lo_groups"] += gen.last_groups
            self._tick("decode_launched")
            out = gen.collect(nrows, self.max_new, [p.plen for p in rb] +
                              [(cell_pairs[src[1]].plen if src[0] == "new" else src[1].pair.plen) for src in row_src])
            self._tick("decode_collected")
            self.stats["decode_row_steps"] += gen.last_rows[0]
            self.stats["decode_rows_run"] += gen.last_rows[1]
            carry_move = self._carry_out(plan, cell_pairs, batch, D, seg, nll_c, row_src, rsteps, ran, n_ride_rows)
        self._tick("decode")
        # ---- ride-along baselines: full lens (with running sums for their future cells)
        if nr:
            resp_r = [out.response_ids(j) for j in range(nr)]
            lr_r = self._readout(rb, out.n_gen[:nr], resp_r, [p.track for p in rb], seqs=list(range(nc, nc + nr)),
                                 keep_cum=not self.lazy_cum)
            self._tick("baseline_lens")
            self._finalize_baselines(rb, out, lr_r, list(range(nr)), slots=list(range(nc, nc + nr)))
            self._tick("baseline_finalize")
            self._score_pairs(rb)
            self._tick("baseline_scores")
        self._tick("baseline_lens+finalize")
        # ---- cells: responses, reused + partial lens.  Readout entries: every cell of this batch except
        # the ones carried on, then the carried cells of earlier batches that finished here
        carried_now = {id(cr.cell) for cr in self._carry}
        drow = {}
        fin_carry = []
        for j, src in enumerate(row_src):
            if src[0] == "new":
                drow[src[1]] = nr + j
            elif id(src[1].cell) not in carried_now:
                fin_carry.append((src[1], nr + j))
        entries = []
        for b, (c, p) in enumerate(zip(batch, cell_pairs)):
            if id(c) in carried_now:
                continue
            if D[b] is None:
                entries.append((c, p, b, None, nll_c[b], sn_c[b], None, int(f_a[b])))
            else:
                entries.append((c, p, b, D[b], nll_c[b], None, drow[b], int(f_a[b])))
        for cr, j in fin_carry:
            entries.append((cr.cell, cr.pair, cr.slot, cr.d, cr.nll, None, j, int(cr.pre[2] - cr.pair.plen)))
        # the carry move runs after the readout has read the finished carried cells' store rows, and before
        # a staged next tail overwrites the cell slots (_launch_staged_next runs it at that point)
        self._carry_move_pending = carry_move
        if entries:
            results = self._resume_readout(entries, out)
        else:
            # nothing to read out (every cell carried on): still launch the announced next batch now, so a
            # stale announcement is never staged during a later readout
            results = []
            self._launch_staged_next()
        if self._carry_move_pending is not None:
            self._carry_move_pending()
            self._carry_move_pending = None
        self._tick("results")
        return results

    def _trie_keys(self, n_ride: int, rows: Sequence, pre_slot: np.ndarray, pre_lo: np.ndarray,
                   start: np.ndarray) -> Optional[np.ndarray]:
        """Group keys of the decode rows for the prefix-trie decode (``Generator.decode(share_keys=)``), or
        None when no two rows can share.  Blocks ``0..l`` of a diverged cell depend only on its tokens: below
        its divergence ``D`` they are the pair's baseline (read from the pair KV, ``pre_slot`` / ``pre_lo``),
        from ``D`` on its own generated tokens.  Rows of one pair with equal tokens from ``D`` (new rows: the
        divergent token ``e_d``; carried rows: their tokens since ``D``) therefore get one key; the ride-along
        baselines (the first ``n_ride`` rows) each get their own.  ``rows[i]`` (cell rows in decode order): the
        divergent token of a new row, or the carry record of a carried one."""
        n = len(rows)
        kp = self.gen.kv_prefix
        if not self.trie_decode or n < 2 or kp is None:
            return None
        wk = max([1] + [len(cr.prefix) - cr.d for cr in rows if isinstance(cr, _Carry)])
        mat = np.full((n, 3 + wk), -2, np.int64)
        mat[:, 0], mat[:, 1], mat[:, 2] = pre_slot, pre_lo, start
        for i, cr in enumerate(rows):
            if isinstance(cr, _Carry):
                t = cr.prefix[cr.d:]
                mat[i, 3: 3 + len(t)] = t
            else:
                mat[i, 3] = cr
        alone = pre_lo <= 0                       # no shared prefix: nothing to share
        mat[alone, 0] = -1 - np.nonzero(alone)[0]
        _, inv = np.unique(mat, axis=0, return_inverse=True)
        inv = inv.reshape(-1)
        u = int(inv.max()) + 1 if n else 0
        if u == n:
            return None                           # all distinct: groups never merge, plain decode
        return np.concatenate([np.arange(n_ride, dtype=np.int64) + u, inv.astype(np.int64)])

    def _carry_out(self, plan, cell_pairs, batch, D, seg, nll_c, row_src, rsteps, ran, n_ride_rows):
        """After an early-stopped decode: record the still-unfinished cell rows as carried and return the
        move of their data to the carry region (KV of every layer, capture-store row, adapter id,
        projection basis rows) — to run once this batch's readout has read the store rows of the
        carried cells that finished here (the region slots get reused)."""
        gen = self.gen
        unf = [j for j in range(len(row_src)) if rsteps[n_ride_rows + j] > ran]
        if not unf:
            return None
        st = gen.row_state([n_ride_rows + j for j in unf])
        keep = [k for k in range(len(unf)) if not bool(st["done"][k])]      # stopped rows are finished
        if not keep:
            return None
        assert len(keep) <= self.carry_rows, "carry region overflow"
        base = self.B - self.carry_rows
        src_slots, dst_slots, b_src, b_dst = [], [], [], []
        rmax = plan["rmax"]
        for i, k in enumerate(keep):
            j = unf[k]
            kind, obj = row_src[j]
            dst = base + i
            step = int(st["step"][k])
            if kind == "new":
                b = obj
                c, p = batch[b], cell_pairs[b]
                f = seg[b][0]
                src = b
                d, nll = D[b], nll_c[b]
                pre = (p.kv_slot, p.plen + D[b], p.plen + f)
                prow = (plan["spikes"][b].copy(), int(plan["kind"][b]), plan["idx"][b].copy(), int(plan["cnt"][b]))
            else:
                cr = obj
                c, p, src, d, nll, pre = cr.cell, cr.pair, cr.slot, cr.d, cr.nll, cr.pre
                prow = cr.plan_row if kind != "new" else prow
            if prow[1] == 2:       # projection cell: its basis rows move with it
                ix = prow[2].copy()
                ix[: prow[3]] = np.arange(dst * rmax, dst * rmax + prow[3])
                b_src += prow[2][: prow[3]].tolist()
                b_dst += list(range(dst * rmax, dst * rmax + prow[3]))
                prow = (prow[0], prow[1], ix, prow[3])
            self._carry.append(_Carry(c, p, d, nll, dst, int(st["tok"][k]), int(st["pos"][k]),
                                      st["tokens"][k, :step].tolist(), st["nll"][k, :step].astype(np.float32),
                                      int(rsteps[n_ride_rows + j] - ran), pre, prow))
            src_slots.append(src)
            dst_slots.append(dst)
        self.stats["carried"] += len(keep)

        def move():
            si = torch.tensor(src_slots, device=self.dev)
            di = torch.tensor(dst_slots, device=self.dev)
            c = gen.cache
            for l in range(c.k.shape[0]):            # per layer: bounded temporaries
                c.k[l].index_copy_(0, di, c.k[l].index_select(0, si))
                c.v[l].index_copy_(0, di, c.v[l].index_select(0, si))
            self.store.index_copy_(0, di, self.store.index_select(0, si))
            if getattr(self.m, "lora", None) is not None:
                c.adapter.index_copy_(0, di, c.adapter.index_select(0, si))
            if b_src:
                bs = self._plan.basis
                bs.index_copy_(0, torch.tensor(b_dst, device=self.dev),
                               bs.index_select(0, torch.tensor(b_src, dtype=torch.long, device=self.dev)))
        return move
