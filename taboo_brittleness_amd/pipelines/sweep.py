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
once per sweep.  Cells are enumerated deterministically and seeded per cell,
then sharded round-robin over data-parallel ranks.

Prefix sharing (``runtime.prefix_share``, exact): an edited cell computes
exactly what its pair's baseline computed up to the first edited position f
(same prompt, same greedy tokens, no edit yet).  The baseline's KV cache and
hooked-layer residuals for positions < f are therefore copied (device copies)
instead of recomputed: the cell resumes decoding at f, and the teacher-forced
ΔNLL pass only runs positions ≥ f, adding the baseline's per-token NLLs for
the earlier targets.  Baselines of the *next* pairs ride along in the same
decode batch, so their cost hides behind the cells'.
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from .. import ops
from ..interp import analysis as A
from ..interp.edits import CaptureHook, EditHook, EditPlan
from ..interp.logit_lens import lens_readout, reference_exclusions
from ..interp.prompts import contains_secret, hint_prompt_ids
from ..models.tokenizer import secret_token_id
from ..runtime.generation import Generator

METHODS = ("sae_targeted", "sae_random", "proj_targeted", "proj_random")


@dataclass
class Pair:
    word: str
    pidx: int
    prompt: str
    ids: List[int]
    forms: List[str]
    track: List[int]                       # [secret(space), secret(bare), decoys...]
    resp: List[int] = field(default_factory=list)
    p_secret: Optional[np.ndarray] = None  # [n_resp] lens prob of the secret (space form) at the hooked layer
    spikes_rel: List[int] = field(default_factory=list)
    top_ids: List[int] = field(default_factory=list)
    resid: Optional[torch.Tensor] = None   # [n_resp, D] hooked-layer residuals (device)
    nll: float = float("nan")
    targeted: List[int] = field(default_factory=list)
    active_pool: List[int] = field(default_factory=list)
    gen_toks: List[int] = field(default_factory=list)   # generated tokens incl. the stop token (if any)
    tok_nll: Optional[np.ndarray] = None                # per generated token NLL under the unedited model
    kv_slot: int = -1                                   # slot in the runner's pair-KV store

    @property
    def first_edit(self) -> int:
        """Response index of the first edited position (last token if there is nothing to edit)."""
        if self.spikes_rel:
            return min(self.spikes_rel)
        return max(len(self.resp) - 1, 0)

    @property
    def plen(self) -> int:
        return len(self.ids)

    @property
    def spikes_abs(self) -> List[int]:
        return [self.plen + i for i in self.spikes_rel]


@dataclass
class Cell:
    pair: int
    method: str
    budget: int
    trial: int
    seed: int

    @property
    def kind(self) -> str:
        return "sae" if self.method.startswith("sae") else "proj"


class SweepRunner:
    def __init__(self, cfg, model, tok, sae, batch: int, device, layer: Optional[int] = None,
                 max_new: Optional[int] = None, use_graphs: bool = True, exclusion: str = "reference",
                 prefix_share: Optional[bool] = None, kv_pairs: int = 64):
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
        self._kv_next = 0
        self._kv_owner: Dict[int, int] = {}
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
            if self.prefix_share:
                c = self.gen.cache
                shape = (c.k.shape[0], self.kv_pairs) + tuple(c.k.shape[2:])
                self.pair_kv = (torch.zeros(shape, dtype=c.k.dtype, device=self.dev),
                                torch.zeros(shape, dtype=c.v.dtype, device=self.dev))
        return self.gen

    def _S_needed(self, pairs: Sequence[Pair]) -> int:
        return max(p.plen for p in pairs) + self.max_new + 1

    # -------------------------------------------------------------- baseline
    @torch.no_grad()
    def run_baselines(self, pairs: List[Pair]) -> None:
        """Standalone baseline pass (generation + lens + spikes + scores + NLL) for ``pairs``."""
        t0 = time.perf_counter()
        self._ensure_gen(self._S_needed(pairs))
        for c0 in range(0, len(pairs), self.B):
            self.run_cells(pairs, [], ride_along=pairs[c0:c0 + self.B])
        self.timings["baseline_total"] = time.perf_counter() - t0

    def _finalize_baselines(self, chunk: Sequence[Pair], out, lr, rows: Sequence[int]) -> None:
        nll = out.tok_nll.float().cpu().numpy()
        stop = set(int(x) for x in self.gen.stop_ids.tolist())
        for p, i in zip(chunk, rows):
            p.resp = out.response_ids(i)
            n = len(p.resp)
            full = out.tokens[i].tolist()
            p.gen_toks = full[: n + 1] if out.stopped[i] else full[:n]
            if not p.gen_toks:   # degenerate: nothing generated at all
                p.gen_toks = [next(iter(stop))]
            p.tok_nll = nll[i, : len(p.gen_toks)].copy()
            p.nll = float(p.tok_nll[:n].mean()) if n else float("nan")
            p.p_secret = lr.probs[i][:, 0].copy()
            p.top_ids = lr.topk_ids[i]
            p.spikes_rel = A.select_spikes(p.p_secret, p.resp, p.track[:2], self.iv.spikes_k)
            p.resid = self.store[i, p.plen:p.plen + n].clone()
            if self.pair_kv is not None:
                p.kv_slot = self._kv_next % self.kv_pairs
                self._kv_next += 1
                self._kv_owner[p.kv_slot] = id(p)
                c = self.gen.cache
                for l in range(c.k.shape[0]):
                    self.pair_kv[0][l, p.kv_slot].copy_(c.k[l, i])
                    self.pair_kv[1][l, p.kv_slot].copy_(c.v[l, i])

    def _readout(self, chunk, n_gen, resp_ids, track):
        excl = [reference_exclusions(self.tok, r) for r in resp_ids] if self.exclusion == "reference" else None
        return lens_readout(self.m, self.store, [p.plen for p in chunk], list(n_gen), track,
                            top_k=self.cfg.model.top_k, exclusion=self.exclusion, excl_pairs=excl,
                            response_ids=resp_ids)

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
            for g, p in enumerate(live):
                p.targeted = A.top_latents_from_scores(scores[g], mmax)
        acts = self.sae.encode(R)
        for g, p in enumerate(live):
            a = acts[seg[g]:seg[g + 1]][p.spikes_rel]
            p.active_pool = torch.nonzero(a.amax(0) > 0).flatten().cpu().tolist()

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
                        cells.append(Cell(pi, meth, int(bud), t, A.cell_seed(base, p.word, p.pidx, meth, bud, t)))
        return cells

    def _bases(self, pairs: Sequence[Pair]) -> Dict[str, torch.Tensor]:
        """PCA secret subspaces (EP:144-146) pooled per word (or across all pairs)."""
        rmax = max(self.iv.ranks) if self.iv.ranks else 1
        groups: Dict[str, List[torch.Tensor]] = {}
        for p in pairs:
            if p.resid is None or not p.spikes_rel:
                continue
            key = p.word if self.iv.pca_pool == "word" else "__all__"
            groups.setdefault(key, []).append(p.resid[p.spikes_rel].float())
        return {k: A.secret_subspace(torch.cat(v, 0), rmax) for k, v in groups.items()}

    def _plan_for(self, cells: Sequence[Cell], pairs: Sequence[Pair], bases: Dict[str, torch.Tensor]):
        K = self.iv.spikes_k
        mmax = max([max(self.iv.budgets or [1]), max(self.iv.ranks or [1])])
        rmax = max(self.iv.ranks) if self.iv.ranks else 1
        spikes, kinds, sel = [], [], []
        big = torch.zeros(self.B * rmax, self.D) if self._with_basis else None
        for ci, c in enumerate(cells):
            p = pairs[c.pair]
            spikes.append(p.spikes_abs)
            if c.kind == "sae":
                kinds.append("sae")
                if c.method == "sae_targeted":
                    sel.append(p.targeted[: c.budget])
                else:
                    sel.append(A.random_latents(self.sae.d_sae, c.budget, c.seed, exclude=p.targeted[: c.budget],
                                                pool=p.active_pool))
            else:
                kinds.append("proj")
                if c.method == "proj_targeted":
                    U = bases[p.word if self.iv.pca_pool == "word" else "__all__"][: c.budget]
                else:
                    U = A.random_subspace(self.D, c.budget, c.seed)
                big[ci * rmax: ci * rmax + U.shape[0]] = U.cpu()
                sel.append(list(range(ci * rmax, ci * rmax + U.shape[0])))
        pad = self.B - len(cells)
        spikes += [[]] * pad
        kinds += ["none"] * pad
        sel += [[]] * pad
        return EditPlan.build(self.dev, spikes, kinds, sel, alpha=self.iv.alpha, basis=big, kmax=K, mmax=mmax)

    def _load_plan(self, plan: EditPlan) -> EditHook:
        """Copy into the persistent plan so a captured decode graph stays valid across batches."""
        if self._plan is None:
            self._plan = plan
            self._hook = EditHook(self._plan, self.sae)
        else:
            for f in ("spikes", "kind", "idx", "cnt", "basis"):
                dst, src = getattr(self._plan, f), getattr(plan, f)
                if dst is not None and src is not None:
                    dst.copy_(src)
        return self._hook

    # --------------------------------------------------------- prefix sharing
    def _copy_pair_kv(self, rows: Sequence[int], kv_slots: Sequence[int]) -> None:
        if not rows:
            return
        c = self.gen.cache
        dst = torch.tensor(list(rows), device=self.dev)
        src = torch.tensor(list(kv_slots), device=self.dev)
        for l in range(c.k.shape[0]):
            c.k[l].index_copy_(0, dst, self.pair_kv[0][l].index_select(0, src))
            c.v[l].index_copy_(0, dst, self.pair_kv[1][l].index_select(0, src))

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

    # -------------------------------------------------------------------- run
    @torch.no_grad()
    def run_cells(self, pairs: List[Pair], cells: Sequence[Cell], measure_nll: Optional[bool] = None,
                  ride_along: Sequence[Pair] = ()) -> List[dict]:
        """Run edited cells; ``ride_along`` pairs get their *baseline* generated in the same batch
        (unedited rows), which pipelines the next cells' baselines behind the current ones."""
        measure_nll = self.iv.measure_nll if measure_nll is None else measure_nll
        ride = list(ride_along)
        if not cells and not ride:
            return []
        gen = self._ensure_gen(self._S_needed(list(pairs) + ride))
        bases = self._bases(pairs) if any(c.kind == "proj" for c in cells) else {}
        if self._plan is None:
            self._with_basis = any(c.kind == "proj" for c in cells) or bool(self.iv.ranks and not cells)
        elif any(c.kind == "proj" for c in cells) and self._plan.basis is None:
            self._plan, self.gen._graph = None, None        # plan layout changes: rebuild + recapture
            self._with_basis = True
        per = self.B - len(ride)
        assert per > 0 or not cells, "batch too small for the ride-along baselines"
        results: List[dict] = []
        batches = [list(cells[i:i + per]) for i in range(0, len(cells), per)] or [[]]
        for bi, batch in enumerate(batches):
            rb = ride if bi == 0 else []
            results += self._run_batch(pairs, batch, rb, measure_nll, bases)
        return results

    def _tick(self, name: str) -> None:
        if not self.phase_timing:
            return
        if self.dev.type == "cuda":
            torch.cuda.synchronize(self.dev)
        now = time.perf_counter()
        last = getattr(self, "_t_last", None)
        if last is not None and name != "start":
            self.timings[name] = self.timings.get(name, 0.0) + (now - last)
        self._t_last = now

    def _run_batch(self, pairs, batch, rb, measure_nll, bases) -> List[dict]:
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
        lr = self._readout(rows_pairs, out.n_gen, resp, [p.track for p in rows_pairs])
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
            ps = lr.probs[i][:, 0] if lr.probs[i].shape[0] else np.zeros(0, dtype=np.float32)
            guesses = [self.tok.decode([t]).strip() for t in lr.topk_ids[i]]
            text = self.tok.decode(resp[i])
            results.append({
                "word": p.word, "prompt_idx": p.pidx, "method": c.method, "budget": c.budget, "trial": c.trial,
                "seed": c.seed, "n_gen": out.n_gen[i], "spikes": p.spikes_rel,
                "p_secret_mean": float(ps.mean()) if ps.size else 0.0,
                "p_secret_final": float(ps[-1]) if ps.size else 0.0,
                "p_secret_max": float(ps.max()) if ps.size else 0.0,
                "p_secret_mean_base": float(p.p_secret.mean()) if p.p_secret is not None and p.p_secret.size else 0.0,
                "topk_ids": lr.topk_ids[i], "guesses": guesses,
                "secret_in_topk": any(g.lower() in {f.lower() for f in p.forms} for g in guesses),
                "decoy_probs": [float(x) for x in lr.probs[i][:, 2:].mean(0)] if lr.probs[i].shape[0] else [],
                "leak": contains_secret(text, p.forms),
                "nll_edit": nll[i], "nll_base": p.nll, "delta_nll": nll[i] - p.nll,
                "nll_self": float(self_nll[i, : out.n_gen[i]].mean()) if out.n_gen[i] else float("nan"),
                "response_ids": resp[i],
            })
        self._tick("results")
        return results

    def _nll_ws(self, M: int):
        """Workspace for the ragged NLL pass, grown in 4096-row steps and sliced per chunk."""
        ws = getattr(self, "_nll_wsp", None)
        if ws is None or ws.M < M:
            from ..models.gemma2 import _Workspace

            self._nll_wsp = None
            ws = self._nll_wsp = _Workspace(self.m.lspec, -(-M // 4096) * 4096, self.dev, self.m.dtype)
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
            cap = 32768
            dev = self.dev
            nll = torch.empty(len(ids), device=dev)
            ids_d = torch.tensor(ids, dtype=torch.int32, device=dev)
            pos_d = torch.tensor(pos, dtype=torch.int32, device=dev)
            slot_d = torch.tensor(owner, dtype=torch.int32, device=dev)
            tgt_d = torch.tensor(tgt, dtype=torch.int32, device=dev)
            step = max(1, (1 << 30) // (m.spec.vocab_size * 2))
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
                    lg = m.logits(x[q0:q1])
                    ops.xent_rows(lg, tgt_d[r0 + q0: r0 + q1], m.spec.final_softcap, True,
                                  out=nll[r0 + q0: r0 + q1])
            extra = torch.zeros(nc, device=dev).index_add_(0, slot_d.long(), nll).cpu().tolist()
            sums = [a + e for a, e in zip(sums, extra)]
        return [sums[b] / len(p.resp) if p.resp else float("nan") for b, p in enumerate(cell_pairs)]


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
