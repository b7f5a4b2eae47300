"""Sweep readouts (part of :class:`~.sweep.SweepRunner`): the per-cell records after a decode -- logit-lens response
sums reused from the baseline's running sums, top-k guesses, secret probabilities and decoys, the teacher-forced
tail NLL of the edited model on the baseline response (packed rows, fused vocab head) and the leak verdicts.
"""
from __future__ import annotations

import time
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from .. import ops
from ..interp import analysis as A
from ..interp.edits import EditHook
from ..interp.logit_lens import excl_table, lens_packed, lens_readout, reference_exclusions, vocab_slice, vocab_topk
from ..interp.prompts import contains_secret
from .sweep_types import Cell, Pair, _h2d, _nullctx

# bf16 logits per vocab-head GEMM chunk of the teacher-forced tail: 2 GB (4096 rows) measured +0.65 % over 1 GB at the
# same 263 GB peak; 4 GB +0.3 % more but 276 GB peak (profiles/r5/bench/head_chunk/)
HEAD_LOGITS_BYTES = 2 << 30
# teacher-forced tail rows per forward chunk (whole cells; chunks alternate between two streams): 24576 / 49152
# measured within noise of 32768 (profiles/r5/bench/tail_chunk/)
TAIL_CHUNK_ROWS = 32768



class ReadoutMixin:
    """Methods of :class:`~.sweep.SweepRunner` (state lives on the runner; see its docstring)."""

    def _resume_readout(self, entries, out) -> List[dict]:
        """Lens readout + result records of layer-resumed cells.  The host side is columnar: one set of
        numpy arrays for the whole batch (no per-cell Python work on the launching thread); every
        non-diverged cell of a pair shares the pair's response, spikes and exclusions.

        ``entries``: per cell ``(cell, pair, slot, D or None, nll_edit, self_nll or None, out row or None, f)``
        — ``slot`` holds its capture-store rows, diverged cells read their response from ``out``; spikes before
        the cell's effective first edit ``f`` were no-op edits, their lens is the baseline's."""
        m = self.m
        S1 = self.store.shape[1]
        E_n = len(entries)
        batch = [e[0] for e in entries]
        cell_pairs = [e[1] for e in entries]
        # ---- per unique pair: response length, prompt length, spikes (kept order), tracked ids, tokens
        uid: Dict[int, int] = {}
        ulist: List[Pair] = []
        u_a = np.empty(E_n, np.int64)
        for i, p in enumerate(cell_pairs):
            u = uid.get(id(p))
            if u is None:
                u = uid[id(p)] = len(ulist)
                ulist.append(p)
            u_a[i] = u
        K = max(len(p.track) for p in ulist)
        Ks = max(1, max(len(p.spikes_rel) for p in ulist))
        U = len(ulist)
        n_u = np.asarray([len(p.resp) for p in ulist], np.int64)
        plen_u = np.asarray([p.plen for p in ulist], np.int64)
        sp_u = np.full((U, Ks), -1, np.int64)
        trk_u = np.full((U, K), -1, np.int64)
        for u, p in enumerate(ulist):
            sp = [x for x in p.spikes_rel if x < len(p.resp)]
            sp_u[u, : len(sp)] = sp
            trk_u[u, : len(p.track)] = p.track
        slot_a = np.asarray([e[2] for e in entries], np.int64)
        dv_a = np.asarray([-1 if e[3] is None else e[3] for e in entries], np.int64)
        j_a = np.asarray([-1 if e[6] is None else e[6] for e in entries], np.int64)
        nll_a = np.asarray([e[4] for e in entries], np.float64)
        f_e = np.asarray([e[7] if len(e) > 7 else 0 for e in entries], np.int64)
        div = dv_a >= 0
        host_tok = out.host_tokens() if (out is not None and div.any()) else None
        ngen_o = np.asarray(out.n_gen, np.int64) if out is not None else np.zeros(0, np.int64)
        ng_a = n_u[u_a].copy()
        d_a = n_u[u_a].copy()
        ng_a[div] = ngen_o[j_a[div]]
        d_a[div] = dv_a[div]
        # self NLL: the teacher-forced value for undiverged cells, the decode's own for diverged ones
        sn_a = np.asarray([np.nan if e[5] is None else e[5] for e in entries], np.float64)
        if div.any():
            tn = out.tok_nll.float().cpu().numpy()[j_a[div]]
            ngd = ng_a[div]
            msk = np.arange(tn.shape[1])[None, :] < ngd[:, None]
            sums = np.where(msk, tn, 0.0).sum(1, dtype=np.float64)
            sn_a[div] = np.where(ngd > 0, sums / np.maximum(ngd, 1), np.nan)
        # ---- rows to evaluate per cell: its spikes before min(D, n_gen) (pair order), then D .. n_gen-1
        lim = np.where(div, np.minimum(d_a, ng_a), n_u[u_a])
        spk = sp_u[u_a]
        keep = (spk >= 0) & (spk < lim[:, None]) & (spk >= f_e[:, None])
        order = np.argsort(~keep, axis=1, kind="stable")
        spk_c = np.take_along_axis(spk, order, 1)
        cnt_s = keep.sum(1)
        cnt_t = np.where(div, np.maximum(ng_a - d_a, 0), 0)
        cnt = cnt_s + cnt_t
        offs = np.concatenate([[0], np.cumsum(cnt)]).astype(np.int64)
        R = int(offs[-1])
        cell_of = np.repeat(np.arange(E_n), cnt)
        q = np.arange(R, dtype=np.int64) - offs[cell_of]
        cs = cnt_s[cell_of]
        pos = np.where(q < cs, spk_c[cell_of, np.minimum(q, Ks - 1)], d_a[cell_of] + q - cs)
        rows = slot_a[cell_of] * S1 + plen_u[u_a][cell_of] + pos
        trk = trk_u[u_a][cell_of]
        ex = np.full((R, 2), -1, np.int64)
        if self.exclusion == "reference" and R:
            etab = excl_table(self.tok, m.spec.vocab_size)
            Lm = int(max(1, n_u.max(), ng_a.max() if E_n else 1))
            tok_u = np.zeros((U, Lm), np.int64)
            for u, p in enumerate(ulist):
                tok_u[u, : len(p.resp)] = p.resp
            tokm = tok_u[u_a]
            if div.any():
                w = min(Lm, host_tok.shape[1])
                tokm[np.nonzero(div)[0], :w] = host_tok[j_a[div], :w]
            cur = etab[tokm]
            ex[:, 0] = cur[cell_of, pos]
            ex[:, 1] = np.where(pos > 0, cur[cell_of, np.maximum(pos - 1, 0)], -1)
        row_key = self._lens_row_keys(cell_of, pos, q >= cs, div, j_a, u_a, sp_u, host_tok) if R else None
        row_key, row_check = row_key if row_key is not None else (None, None)
        self._tick("ro_entries")
        self.stats["lens_rows"] += R
        self._ensure_cum(ulist)
        base = self._lens_base(cell_pairs, d_a.tolist(), ng_a.tolist(), f_e)
        self._tick("ro_base")
        acc, pr_d = lens_packed(m, self.store, rows, offs, base, trk, ex, sync=False, row_key=row_key,
                                stats=self.stats, row_check=row_check)
        if self.exclusion == "response":
            lo, Vl = vocab_slice(m)
            for i in range(E_n):
                r_ = cell_pairs[i].resp if dv_a[i] < 0 else host_tok[j_a[i], : ng_a[i]].tolist()
                ids = torch.tensor(sorted(set(r_)), dtype=torch.long, device=self.dev) - lo
                ids = ids[(ids >= 0) & (ids < Vl)]
                if ids.numel():
                    acc[i, ids] = 0.0
        vals, ids = vocab_topk(m, acc, self.cfg.model.top_k)
        # every readout output in one async D2H (pinned), so the next batch's teacher-forced tail can be
        # queued behind this batch's lens before the host waits for it
        vh_d, ih_d = vals.sum(1), ids
        if self.dev.type == "cuda":
            host = [torch.empty(t.shape, dtype=t.dtype, pin_memory=True) for t in (pr_d, vh_d, ih_d)]
            for h, t in zip(host, (pr_d, vh_d, ih_d)):
                h.copy_(t, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.dev))
        else:
            host, ev = [pr_d, vh_d, ih_d], None
        self._tick("lens_launched")
        self._launch_staged_next()
        if ev is not None:
            ev.synchronize()
        pr, vh, ih = (t.numpy() for t in host)
        self._tick("lens")
        cols = {"ng": ng_a, "d": d_a, "div": div, "j": j_a, "sn": sn_a, "nll": nll_a, "pos": pos,
                "cell_of": cell_of, "host_tok": host_tok}
        if getattr(self, "_defer", False):
            return self._records_pool().submit(self._resume_records, batch, cell_pairs, cols, pr, vh, ih, K)
        return self._resume_records(batch, cell_pairs, cols, pr, vh, ih, K)

    def _lens_row_keys(self, cell_of, pos, after_d, div, j_a, u_a, sp_u, host_tok) -> Optional[np.ndarray]:
        """Dedup keys of the lens rows (``lens_packed(row_key=)``): the hooked-layer residual of a diverged cell at
        a non-spike position ``t >= D`` is a function of its pair and its tokens ``0..t`` alone (blocks ``0..l``
        see only tokens, and no edit touches it), so cells of one pair with equal tokens up to ``t`` hold the
        same row.  Those rows get a 63-bit hash key of (pair, t, tokens ``0..t``) plus a second independent hash
        as a collision check (``lens_packed(row_check=)``); every other row (spikes, undiverged cells) a unique
        negative key.  Returns ``(keys, checks)``, or None when nothing can repeat."""
        R = len(pos)
        if not self.trie_decode or host_tok is None or not div.any():
            return None
        spike = (sp_u[u_a][cell_of] == pos[:, None]).any(1)
        dd = after_d & div[cell_of] & ~spike
        key = -1 - np.arange(R, dtype=np.int64)
        if not dd.any():
            return None
        # rolling 64-bit hash of every diverged cell's response prefix (wrapping uint64 arithmetic)
        tok = host_tok[j_a[div]].astype(np.uint64) + np.uint64(1)
        h = np.empty(tok.shape, np.uint64)
        h2 = np.empty(tok.shape, np.uint64)
        acc = np.zeros(tok.shape[0], np.uint64)
        acc2 = np.full(tok.shape[0], 0x243F6A8885A308D3, np.uint64)
        mul, mul2 = np.uint64(0x9E3779B97F4A7C15), np.uint64(0xD6E8FEB86659FD93)
        with np.errstate(over="ignore"):
            for t in range(tok.shape[1]):
                acc = (acc ^ tok[:, t]) * mul
                acc ^= acc >> np.uint64(29)
                h[:, t] = acc
                acc2 = (acc2 + tok[:, t] * np.uint64(0x9FB21C651E98DF25)) * mul2
                acc2 ^= acc2 >> np.uint64(31)
                h2[:, t] = acc2
            ci = np.full(len(div), -1, np.int64)
            ci[np.nonzero(div)[0]] = np.arange(int(div.sum()))
            r = np.nonzero(dd)[0]
            c = ci[cell_of[r]]
            t = np.minimum(pos[r], tok.shape[1] - 1)
            k = h[c, t] ^ (u_a[cell_of[r]].astype(np.uint64) * np.uint64(0xC2B2AE3D27D4EB4F))
            k ^= pos[r].astype(np.uint64) * np.uint64(0x165667B19E3779F9)
            k2 = h2[c, t] ^ (u_a[cell_of[r]].astype(np.uint64) * np.uint64(0x85EBCA77C2B2AE63))
        key[r] = (k & np.uint64(0x7FFFFFFFFFFFFFFF)).astype(np.int64)
        chk = np.arange(R, dtype=np.int64)
        chk[r] = k2.view(np.int64)
        return key, chk

    def _resume_records(self, batch, cell_pairs, cols, pr, vh, ih, K) -> List[dict]:
        """Host half of :meth:`_resume_readout`: per-cell readout statistics and result records."""
        nc = len(cell_pairs)
        ng_a, d_a, div, j_a = cols["ng"], cols["d"], cols["div"], cols["j"]
        host_tok = cols["host_tok"]
        # ---- per-cell tracked-id probability tables, vectorised: baseline rows up to D, evaluated rows
        Lmax = int(max(1, ng_a.max() if nc else 1))
        P3 = np.zeros((nc, Lmax, K), dtype=np.float32)
        groups: Dict[int, List[int]] = {}
        for b, p in enumerate(cell_pairs):
            groups.setdefault(id(p), []).append(b)
        for bs in groups.values():
            p = cell_pairs[bs[0]]
            tp = p.track_probs
            if tp is None or not len(p.resp):
                continue
            same = [b for b in bs if d_a[b] >= len(p.resp)]          # undiverged: all baseline rows
            if same:
                P3[np.asarray(same), : tp.shape[0], : tp.shape[1]] = tp[None]
            for b in bs:
                if d_a[b] < len(p.resp):
                    keep = min(int(d_a[b]), int(ng_a[b]), tp.shape[0])
                    P3[b, :keep, : tp.shape[1]] = tp[:keep]
        if cols["pos"].size:
            P3[cols["cell_of"], cols["pos"]] = pr
        valid = np.arange(Lmax)[None, :] < ng_a[:, None]
        p0 = np.where(valid, P3[:, :, 0], 0.0)
        cnt = np.maximum(ng_a, 1)
        ps_mean = p0.sum(1) / cnt
        ps_final = P3[np.arange(nc), np.maximum(ng_a - 1, 0), 0]
        ps_max = np.where(valid, P3[:, :, 0], -np.inf).max(1) if nc else np.zeros(0)
        decoy = (np.where(valid[:, :, None], P3[:, :, 2:], 0.0).sum(1) / cnt[:, None]) if K > 2 else None
        results = []
        for b, (c, p) in enumerate(zip(batch, cell_pairs)):
            ng = int(ng_a[b])
            resp = host_tok[j_a[b], :ng].tolist() if div[b] else p.resp
            topk = ih[b].tolist() if ng > 0 and vh[b] > 0 else []
            stats = (float(ps_mean[b]), float(ps_final[b]), float(ps_max[b])) if ng else (0.0, 0.0, 0.0)
            dec = decoy[b, : len(p.track) - 2].tolist() if (decoy is not None and ng and len(p.track) > 2) else []
            results.append(self._cell_record(c, p, ng, resp, stats, dec, topk, float(cols["nll"][b]),
                                             float(cols["sn"][b])))
        return results

    @torch.no_grad()
    def _ensure_cum(self, pairs: Sequence[Pair]) -> None:
        """Running lens sums of ``pairs`` (lazy mode): recomputed from each pair's hooked-layer residuals with
        the same lens readout its baseline ran; sums rebuilt for earlier batches are released first."""
        need = [p for p in pairs if p.lens_cum is None and p.resid is not None]
        if not need:
            return
        keep = {id(p) for p in pairs}
        for q in self._cum_live:
            if id(q) not in keep:
                q.lens_cum = None
        self._cum_live = [q for q in self._cum_live if id(q) in keep]
        nmax = max(1, max(len(p.resp) for p in need))
        # rows past a response are never read (lens_readout points padding at the last, scratch row): only that
        # row is zeroed, and the residuals go in with one concatenation + one row scatter
        tmp = torch.empty(len(need), nmax + 1, self.D, dtype=self.store.dtype, device=self.dev)
        tmp[:, nmax].zero_()
        parts = [(i, p.resid[: len(p.resp)]) for i, p in enumerate(need) if len(p.resp)]
        if parts:
            dst = np.concatenate([i * (nmax + 1) + np.arange(r.shape[0]) for i, r in parts])
            tmp.view(-1, self.D).index_copy_(0, _h2d(dst, self.dev).to(self.dev, non_blocking=True),
                                             torch.cat([r for _, r in parts], 0))
        resp = [list(p.resp) for p in need]
        excl = [reference_exclusions(self.tok, r) for r in resp] if self.exclusion == "reference" else None
        lr = lens_readout(self.m, tmp, [0] * len(need), [len(r) for r in resp], [p.track for p in need],
                          top_k=self.cfg.model.top_k, exclusion=self.exclusion, excl_pairs=excl,
                          response_ids=resp, keep_cum=True)
        for p, c in zip(need, lr.cum):
            p.lens_cum = c
        self._cum_live += need

    def _lens_base(self, cell_pairs: Sequence[Pair], Dc: Sequence[int], ngen: Sequence[int],
                   f: Optional[np.ndarray] = None) -> torch.Tensor:
        """Reused part of each cell's response lens sum: the baseline's running sum up to the divergence
        ``D`` minus its spike positions from its effective first edit ``f`` on (those are re-evaluated on the
        edited residual; earlier spikes were no-op edits).  Per pair one small matmul of a {0, +-1} coefficient
        matrix over the pair's running sums, written straight into the pair's (contiguous) output rows; every
        coefficient of every pair goes up in one copy."""
        V = vocab_slice(self.m)[1]           # this rank's lens columns under vocab-parallel TP
        base = torch.empty(len(cell_pairs), V, dtype=torch.float32, device=self.dev)
        groups: Dict[int, List[int]] = {}
        for b, p in enumerate(cell_pairs):
            groups.setdefault(id(p), []).append(b)
        coefs: List[np.ndarray] = []
        plan = []
        co = 0
        for bs in groups.values():
            p = cell_pairs[bs[0]]
            n1 = p.lens_cum.shape[0]
            d = np.minimum(np.minimum(np.asarray([Dc[b] for b in bs]), np.asarray([ngen[b] for b in bs])), n1 - 1)
            sp = np.asarray([x for x in p.spikes_rel if x + 1 < n1], dtype=np.int64)
            nb = len(bs)
            # base[b] = C[d_b] - sum_{f_b <= s < d_b} (C[s + 1] - C[s]), as coefficients over the rows of C
            W = np.zeros((nb, n1), np.float32)
            W[np.arange(nb), d] = 1.0
            if sp.size:
                fb = np.asarray([f[b] for b in bs], np.int64) if f is not None else np.zeros(nb, np.int64)
                mk = ((sp[None, :] < d[:, None]) & (sp[None, :] >= fb[:, None])).astype(np.float32)
                np.add.at(W, (slice(None), sp + 1), -mk)
                np.add.at(W, (slice(None), sp), mk)
            coefs.append(W.ravel())
            plan.append((p, bs, n1, co))
            co += W.size
        if self.dev.type == "cuda":
            # one row-combination kernel over every cell: each cell's few non-zero coefficients (its divergence row
            # and its re-evaluated spike terms) in ascending row order -- a fixed per-cell sum, whatever the batch
            # (vectorised per pair: a per-cell host loop cost ~25 ms of GPU idle per step, profiles/r6/prof/head2)
            B = len(cell_pairs)
            basep = np.zeros(B, np.int64)
            bl, pl, cl = [], [], []
            for (p, bs, n1, c), W in zip(plan, coefs):
                W = W.reshape(len(bs), n1)
                assert p.lens_cum.stride(-1) == 1 and p.lens_cum.dtype == torch.float32
                bsa = np.asarray(bs, np.int64)
                basep[bsa] = p.lens_cum.data_ptr()
                r, col = np.nonzero(W)                       # row-major: a cell's terms in ascending row order
                bl.append(bsa[r])
                pl.append(p.lens_cum.data_ptr() + col.astype(np.int64) * (p.lens_cum.stride(0) * 4))
                cl.append(W[r, col])
            b_all = np.concatenate(bl)
            order = np.argsort(b_all, kind="stable")
            b_s = b_all[order]
            cnt = np.bincount(b_s, minlength=B)
            T = max(1, int(cnt.max()) if cnt.size else 1)
            k = np.arange(b_s.size) - (np.cumsum(cnt) - cnt)[b_s]
            ptr = np.repeat(basep[:, None], T, axis=1)      # padding terms: a valid row with coefficient 0
            cf = np.zeros((B, T), np.float32)
            ptr[b_s, k] = np.concatenate(pl)[order]
            cf[b_s, k] = np.concatenate(cl)[order]
            return ops.row_combine(_h2d(ptr, self.dev).to(self.dev, non_blocking=True),
                                   _h2d(cf, self.dev).to(self.dev, non_blocking=True), base)
        dev_w = _h2d(np.concatenate(coefs), self.dev).to(self.dev, non_blocking=True)
        scatter = []
        for p, bs, n1, c in plan:
            w = dev_w[c: c + len(bs) * n1].view(len(bs), n1)
            if bs[-1] - bs[0] + 1 == len(bs):
                torch.mm(w, p.lens_cum, out=base[bs[0]: bs[-1] + 1])
            else:
                scatter.append((bs, w @ p.lens_cum))
        for bs, acc in scatter:              # (cells of a pair are contiguous in the sweep's batches)
            base.index_copy_(0, torch.as_tensor(bs, device=self.dev), acc)
        return base

    @torch.no_grad()
    def _tf_pass(self, cell_pairs: Sequence[Pair], hooks) -> dict:
        """Blocks after the hooked layer over response positions ``f..E`` of every cell (packed rows,
        fed the baseline residuals; edit + capture hooks at the hooked layer).  Returns per-row greedy
        token, its NLL and the NLL of the baseline's next token, and per cell ``(f, E, first row)``."""
        return self._tf_finish(self._tf_launch(cell_pairs, hooks))

    def _tf_finish(self, res: dict) -> dict:
        """Host side of a launched teacher-forced tail: wait for its one D2H copy, split it."""
        pend = res.pop("_pending", None)
        if pend is not None:
            host, ev, M = pend
            if ev is not None:
                ev.synchronize()
            res["nxt"] = host[0, :M].view(torch.int32).numpy()
            res["nll_self"] = host[1, :M].numpy()
            res["nll_tgt"] = host[2, :M].numpy()
        return res

    @torch.no_grad()
    def _tf_launch(self, cell_pairs: Sequence[Pair], hooks, f_cell: Optional[np.ndarray] = None) -> dict:
        """Enqueue the teacher-forced tail (no host sync): host index arrays, the packed forward, the vocab
        head, and one async D2H copy of its per-row outputs; :meth:`_tf_finish` waits for it.  ``f_cell[b]``:
        cell ``b``'s effective first edit (``_effective_first_edit``; -1 = its pair's first spike)."""
        from ..models.gemma2 import packed_blocks

        m = self.m
        nc = len(cell_pairs)
        uniq: Dict[int, int] = {}
        srcs, ulist = [], []
        off = 0
        f_a = np.zeros(nc, np.int64)
        E_a = np.zeros(nc, np.int64)
        base_a = np.zeros(nc, np.int64)      # row offset of the pair's residuals in the concatenation
        plen_a = np.zeros(nc, np.int64)
        up_a = np.zeros(nc, np.int64)        # unique-pair index
        for b, p in enumerate(cell_pairs):
            n, G = len(p.resp), len(p.gen_toks)
            fc = int(f_cell[b]) if f_cell is not None and b < len(f_cell) else -1
            f_a[b] = min(p.first_edit, max(n - 1, 0)) if fc < 0 else min(fc, n)
            E_a[b] = min(max([G - 2] + list(p.spikes_rel)), n - 1)
            u = uniq.get(id(p))
            if u is None:
                u = uniq[id(p)] = len(ulist)
                ulist.append((p, off))
                srcs.append(p.resid)
                off += p.resid.shape[0]
            up_a[b], base_a[b], plen_a[b] = u, ulist[u][1], p.plen
        Ls = np.maximum(E_a - f_a + 1, 0)
        r0_a = np.concatenate([[0], np.cumsum(Ls)[:-1]]) if nc else np.zeros(0, np.int64)
        seg = [(int(f_a[b]), int(E_a[b]), int(r0_a[b])) for b in range(nc)]
        M = int(Ls.sum())
        rb_ = np.repeat(np.arange(nc), Ls)                      # cell of every row
        t_ = (np.arange(M) - np.repeat(r0_a, Ls)) + np.repeat(f_a, Ls) if M else np.zeros(0, np.int64)
        Gmax = max((len(p.gen_toks) for p, _ in ulist), default=1)
        gtab = np.full((max(1, len(ulist)), Gmax + 1), -1, np.int64)
        for u, (p, _) in enumerate(ulist):
            gtab[u, : len(p.gen_toks)] = p.gen_toks
        pos = (plen_a[rb_] + t_).astype(np.int32)
        slot = rb_.astype(np.int32)
        tgt = gtab[up_a[rb_], t_ + 1].astype(np.int32)
        src = base_a[rb_] + t_
        self.stats["tf_rows"] += M
        self._tick("tf_host_prep")
        res = {"seg": seg, "nxt": np.zeros(0, np.int32), "nll_self": np.zeros(0, np.float32),
               "nll_tgt": np.zeros(0, np.float32), "row_cell": rb_, "row_t": t_, "tgt": tgt,
               "f": f_a, "E": E_a, "r0": r0_a, "up": up_a, "upairs": [p for p, _ in ulist], "gtab": gtab}
        if M == 0:
            return res
        dev = self.dev
        up_ = lambda a: _h2d(a, dev).to(dev, non_blocking=True)     # noqa: E731  (pinned: no stream drain)
        H = torch.cat(srcs, 0) if len(srcs) > 1 else srcs[0]
        src_d = up_(src)
        pos_d = up_(pos)
        slot_d = up_(slot)
        tgt_d = up_(tgt)
        outs = torch.empty(3, M, dtype=torch.float32, device=dev)      # [greedy id bits, NLL self, NLL target]
        nxt, ns, nt = outs[0].view(torch.int32), outs[1], outs[2]
        rpb = 16 // max(1, m.lspec.heads // m.lspec.kv_heads)
        cap = TAIL_CHUNK_ROWS
        # vocab-head rows per GEMM: 256-row multiples (GEMM tiles) of at most HEAD_LOGITS_BYTES of bf16 logits
        # (4096 rows of the 256k vocab)
        step = max(256, (HEAD_LOGITS_BYTES // (m.spec.vocab_size * 2)) // 256 * 256)
        if getattr(m, "fused_head", False):
            # the fused head keeps no logits (16 B of partials per 128 vocab columns): whole chunks per GEMM
            step = 16384
        # chunks of whole cells (a cell never spans two chunks), so chunks are independent and
        # alternate between two streams: one chunk's bandwidth-bound kernels (attention, norms, GeGLU,
        # vocab head) overlap the other's GEMMs
        chunks, cur, c_lo, c_rows = [], [], 0, 0
        for b, (f, E, r0) in enumerate(seg):
            if E < f:
                continue
            Ln = E - f + 1
            if cur and c_rows + Ln > cap:
                chunks.append((c_lo, c_lo + c_rows, cur))
                cur, c_lo, c_rows = [], r0, 0
            if not cur:
                c_lo = r0
            cur.append((r0 - c_lo, Ln, b, cell_pairs[b].kv_slot, int(plen_a[b] + f)) if self.tf_prefix
                       else (r0 - c_lo, Ln, b))
            c_rows += Ln
        if cur:
            chunks.append((c_lo, c_lo + c_rows, cur))
        main = torch.cuda.current_stream(dev) if dev.type == "cuda" else None
        streams = [main]
        ws_rows = min(cap, -(-M // 256) * 256)
        # every chunk's attention block table in one upload (no host sync between chunks)
        tabs = [packed_blocks(chunk, rpb) for (_, _, chunk) in chunks]
        tab_off = np.concatenate([[0], np.cumsum([t.shape[0] for t in tabs])]).astype(np.int64)
        tab_d = _h2d(torch.cat(tabs, 0), dev).to(dev, non_blocking=True) if tabs else None
        for ci, (c0, c1, chunk) in enumerate(chunks):
            st = streams[ci % len(streams)]
            with (torch.cuda.stream(st) if st is not None else _nullctx()):
                Mc = c1 - c0
                Mp = -(-Mc // 256) * 256
                blk = tab_d[int(tab_off[ci]):int(tab_off[ci + 1])]
                cp = torch.full((Mp,), -1, dtype=torch.int32, device=dev)
                cs = torch.zeros(Mp, dtype=torch.int32, device=dev)
                cp[:Mc], cs[:Mc] = pos_d[c0:c1], slot_d[c0:c1]
                ws = self._nll_ws(ws_rows, key=ci % len(streams)).rows(Mp)
                # the chunk's input residuals straight into the workspace's residual buffer (forward_packed then
                # skips its own copy); only the padding rows are zeroed
                hin = ws.h
                ops.row_gather(H, src_d[c0:c1], hin)
                if Mp > Mc:
                    hin[Mc:].zero_()
                x = m.forward_packed(None, cp, cs, blk, self.gen.cache, hooks, ws=ws, resume_after=self.layer,
                                     h_in=hin, prefix_kv=self.pair_kv if self.tf_prefix else None)
                for q0 in range(0, Mc, step):
                    q1 = min(Mc, q0 + step)
                    if getattr(m, "head_path", False):
                        m.head(x[q0:q1], m.spec.final_softcap, tgt_d[c0 + q0:c0 + q1], nxt[c0 + q0:c0 + q1],
                               ns[c0 + q0:c0 + q1], nt[c0 + q0:c0 + q1])
                        continue
                    # the unembedding runs on whole 256-row tiles (padding rows of x included) so the
                    # GEMM shapes stay few and tuned; only the real rows are read out
                    lg = m.logits(x[q0:min(Mp, q0 + step)])[: q1 - q0]
                    ops.decode_head(lg, m.spec.final_softcap, tgt_d[c0 + q0:c0 + q1], nxt[c0 + q0:c0 + q1],
                                    ns[c0 + q0:c0 + q1], nt[c0 + q0:c0 + q1])
        if len(streams) > 1:
            main.wait_stream(streams[1])
        if dev.type == "cuda":
            host = torch.empty(3, M, dtype=torch.float32, pin_memory=True)
            host.copy_(outs, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(dev))
        else:
            host, ev = outs, None
        res["_pending"] = (host, ev, M)
        self._tick("tf_launched")
        return res

    def _cell_result(self, c: Cell, p: Pair, n_gen: int, resp: List[int], probs: np.ndarray, topk_ids: List[int],
                     nll_edit: float, nll_self: float) -> dict:
        ps = probs[:, 0] if probs.shape[0] else np.zeros(0, dtype=np.float32)
        stats = (float(ps.mean()), float(ps[-1]), float(ps.max())) if ps.size else (0.0, 0.0, 0.0)
        dec = [float(x) for x in probs[:, 2:].mean(0)] if probs.shape[0] else []
        return self._cell_record(c, p, n_gen, resp, stats, dec, topk_ids, nll_edit, nll_self)

    def _cell_record(self, c: Cell, p: Pair, n_gen: int, resp: List[int], stats: Tuple[float, float, float],
                     decoy: List[float], topk_ids: List[int], nll_edit: float, nll_self: float) -> dict:
        dc = self._dec_cache
        guesses = []
        for t in topk_ids:
            g = dc.get(t)
            if g is None:
                g = dc[t] = self.tok.decode([t]).strip()
            guesses.append(g)
        if resp is p.resp or resp == p.resp:     # unchanged response: the baseline's leak verdict
            if p.leak is None:
                p.leak = contains_secret(self.tok.decode(p.resp), p.forms)
            leak = p.leak
        else:
            leak = contains_secret(self.tok.decode(resp), p.forms)
        if p.p_secret_mean is None:
            p.p_secret_mean = float(p.p_secret.mean()) if p.p_secret is not None and p.p_secret.size else 0.0
            p.forms_l = {f.lower() for f in p.forms}
        return {
            "word": p.word, "prompt_idx": p.pidx, "method": c.method, "budget": c.budget, "trial": c.trial,
            "seed": c.seed, "n_gen": n_gen, "spikes": p.spikes_rel,
            "p_secret_mean": stats[0], "p_secret_final": stats[1], "p_secret_max": stats[2],
            "p_secret_mean_base": p.p_secret_mean,
            "topk_ids": topk_ids, "guesses": guesses,
            "secret_in_topk": any(g.lower() in p.forms_l for g in guesses),
            "decoy_probs": decoy,
            "leak": leak,
            "nll_edit": nll_edit, "nll_base": p.nll, "delta_nll": nll_edit - p.nll,
            "nll_self": nll_self,
            "response_ids": resp,
        }

    def _nll_ws(self, M: int, key: int = 0):
        """Workspace for the ragged passes (one per stream ``key``), grown in 4096-row steps and sliced
        per chunk."""
        pool = self.__dict__.setdefault("_nll_wsp", {})
        ws = pool.get(key)
        if ws is None or ws.M < M:
            from ..models.gemma2 import _Workspace

            pool.pop(key, None)
            ws = pool[key] = self.m.new_workspace(-(-M // 4096) * 4096)
        return ws

    @torch.no_grad()
    def _nll_cells(self, cell_pairs: Sequence[Pair], plan_hook: EditHook, out, c0s: Sequence[int]) -> List[float]:
        """Mean NLL of each cell's *baseline* hint under the edit (teacher forced, EP:136).

        The edited decode already scored the baseline's token at every column (``out.tf_nll``); those
        are the teacher-forced NLLs up to the column ``d`` where the cell's own greedy tokens leave the
        baseline's (:func:`teacher_divergence`).  Targets before the decode's first column ``c0`` are
        the baseline's own NLLs (identical prefix), and only targets after ``d`` need a teacher-forced
        pass: a ragged (packed, unpadded) forward over positions ``plen+d .. plen+n-2`` in the cell's
        own KV slot, whose prefix ``< plen+d`` holds exactly the baseline tokens."""
        from ..models.gemma2 import packed_blocks
        from ..runtime.generation import teacher_divergence

        m = self.m
        nc = len(cell_pairs)
        tfn = out.tf_nll[:nc].float().cpu().numpy()
        own = out.tokens[:nc].cpu().numpy()
        sums = [0.0] * nc
        ids, pos, tgt, owner, seqs = [], [], [], [], []
        for b, p in enumerate(cell_pairs):
            n = len(p.resp)
            if not n:
                continue
            c0 = c0s[b]
            tot = float(np.sum(p.tok_nll[: min(c0, n)]))
            d = teacher_divergence(own[b].tolist(), p.resp, c0)
            hi = min(d, n - 1)
            if hi >= c0:
                tot += float(np.sum(tfn[b, c0: hi + 1]))
            sums[b] = tot
            if d < n - 1:
                L = n - 1 - d
                seqs.append((len(ids), L, b))
                ids += p.resp[d: n - 1]
                pos += range(p.plen + d, p.plen + n - 1)
                tgt += p.resp[d + 1: n]
                owner += [b] * L
        self.nll_rows = getattr(self, "nll_rows", 0) + len(ids)
        if ids:
            rpb = 16 // max(1, m.lspec.heads // m.lspec.kv_heads)
            cap = TAIL_CHUNK_ROWS
            dev = self.dev
            nll = torch.empty(len(ids), device=dev)
            ids_d = torch.tensor(ids, dtype=torch.int32, device=dev)
            pos_d = torch.tensor(pos, dtype=torch.int32, device=dev)
            slot_d = torch.tensor(owner, dtype=torch.int32, device=dev)
            tgt_d = torch.tensor(tgt, dtype=torch.int32, device=dev)
            step = max(256, (HEAD_LOGITS_BYTES // (m.spec.vocab_size * 2)) // 256 * 256)
            for r0 in range(0, len(ids), cap):
                r1 = min(len(ids), r0 + cap)
                M = r1 - r0
                Mp = -(-M // 256) * 256                 # few distinct GEMM shapes
                chunk = []
                for (s0, L, b) in seqs:                  # sequences clipped to this chunk
                    a0, a1 = max(s0, r0), min(s0 + L, r1)
                    if a1 > a0:
                        chunk.append((a0 - r0, a1 - a0, b))
                blk = packed_blocks(chunk, rpb).to(dev)
                ci = torch.zeros(Mp, dtype=torch.int32, device=dev)
                cp = torch.full((Mp,), -1, dtype=torch.int32, device=dev)
                cs = torch.zeros(Mp, dtype=torch.int32, device=dev)
                ci[:M], cp[:M], cs[:M] = ids_d[r0:r1], pos_d[r0:r1], slot_d[r0:r1]
                ws = self._nll_ws(min(cap, -(-len(ids) // 256) * 256)).rows(Mp)
                x = m.forward_packed(ci, cp, cs, blk, self.gen.cache, {self.layer: [plan_hook]}, ws=ws)
                for q0 in range(0, M, step):
                    q1 = min(M, q0 + step)
                    if getattr(m, "head_path", False):
                        m.head(x[q0:q1], m.spec.final_softcap, tgt_d[r0 + q0: r0 + q1],
                               nll_tgt=nll[r0 + q0: r0 + q1])
                        continue
                    lg = m.logits(x[q0:q1])
                    ops.xent_rows(lg, tgt_d[r0 + q0: r0 + q1], m.spec.final_softcap, True,
                                  out=nll[r0 + q0: r0 + q1])
            extra = torch.zeros(nc, device=dev).index_add_(0, slot_d.long(), nll).cpu().tolist()
            sums = [a + e for a, e in zip(sums, extra)]
        return [sums[b] / len(p.resp) if p.resp else float("nan") for b, p in enumerate(cell_pairs)]
