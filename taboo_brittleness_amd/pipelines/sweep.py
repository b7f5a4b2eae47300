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
from ..interp.logit_lens import excl_table, lens_packed, lens_readout, reference_exclusions, vocab_slice, vocab_topk
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
    active_pool: np.ndarray = field(default_factory=lambda: np.zeros(0, dtype=np.int64))  # sorted, unique
    gen_toks: List[int] = field(default_factory=list)   # generated tokens incl. the stop token (if any)
    tok_nll: Optional[np.ndarray] = None                # per generated token NLL under the unedited model
    kv_slot: int = -1                                   # slot in the runner's pair-KV store
    lens_cum: Optional[torch.Tensor] = None             # [n_resp + 1, V] running lens sums (layer resume)
    track_probs: Optional[np.ndarray] = None            # [n_resp, K] lens probs of the tracked ids
    leak: Optional[bool] = None                         # baseline response contains the secret (cached)
    p_secret_mean: Optional[float] = None               # cached mean of p_secret (result records)
    forms_l: Optional[set] = None
    rep: int = 0                                        # replicate of this (word, prompt): seeds its random cells
    # exact per-latent activity at the edited spikes (SweepRunner._spike_activity): sorted candidate latent
    # ids and, per id, a bitmask over spikes_rel[:K] of where the edit kernel's own JumpReLU fires
    act_ids: Optional[np.ndarray] = None
    act_mask: Optional[np.ndarray] = None
    act_key: Optional[tuple] = None                     # SAE parameter identity/versions the table was built with

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


@dataclass
class _Carry:
    """A diverged cell whose decode continues in the next batch (decode-tail carry-over): its KV,
    capture-store row and edit-plan row live in the runner's carry region at ``slot``."""
    cell: Cell
    pair: Pair
    d: int                       # divergence point D
    nll: float                   # teacher-forced edit NLL of the baseline hint (already complete)
    slot: int
    tok: int                     # next token to feed, at position ``pos``
    pos: int
    prefix: List[int]            # response tokens so far (ends with ``tok``)
    prefix_nll: np.ndarray       # their NLLs
    steps: int                   # decode steps still needed
    pre: Tuple[int, int, int]    # (pair KV slot, len_lo, len_hi) of the shared prefix
    plan_row: Tuple[np.ndarray, int, np.ndarray, int]   # host (spikes, kind, idx, cnt) of the slot


class SweepRunner:
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
        # ride-along baselines on a side stream next to the teacher-forced tail (1) or merged into the
        # diverged cells' decode batch (0, default: +3% measured at 90 pairs per step, the larger decode batch
        # streams the weights once for both)
        self.overlap_ride = os.environ.get("TB_OVERLAP_RIDE", "0") == "1"
        self.tf_streams = os.environ.get("TB_TF_STREAMS", "0") == "1"   # no measurable gain; opt-in
        self.tf_prefix = os.environ.get("TB_TF_PREFIX", "1") == "1"
        self.stats: Dict[str, int] = {"cells": 0, "diverged": 0, "tf_rows": 0, "lens_rows": 0,
                                      "decode_row_steps": 0, "decode_rows_run": 0, "carried": 0, "staged": 0,
                                      "decode_lo_rows_run": 0, "decode_lo_groups": 0, "lens_gemm_rows": 0}
        # decode-tail carry-over (opt-in; needs ``batch`` to include ``carry_rows`` spare slots): once fewer
        # than ``carry_rows`` diverged cells still decode, the rest continue in the next batch's decode
        # (merged with its new rows) instead of running a long small-batch tail.  Records of carried cells
        # come out with the batch that finishes them; ``run_cells(..., drain=True)`` carries nothing.
        self.carry_rows = 0
        # prefix-trie decode: diverged cells of a pair with equal tokens run blocks 0..l once per group
        # (Generator.decode share_keys); TB_TRIE_DECODE=0 / SweepRunner.trie_decode = False: every row alone
        self.trie_decode = os.environ.get("TB_TRIE_DECODE", "1") == "1"
        # a cell's teacher-forced tail starts at its first spike with a non-zero edit (earlier spikes: its
        # latents are inactive there, an exact no-op); TB_SKIP_NOOP=0: at its pair's first spike
        self.skip_noop_spikes = os.environ.get("TB_SKIP_NOOP", "1") == "1"
        self._carry: List[_Carry] = []
        self._next: Optional["NextBatch"] = None      # batch of the next run_cells call (stage_next)
        # lazy running lens sums: a pair's [n + 1, V] fp32 running sums (52 MB at the 256k vocab) are rebuilt from
        # its kept hooked-layer residuals when its cells run, instead of being held from its baseline on (E steps
        # ahead): only the running batch's pairs hold them (~18 GB less at 90 pairs per step)
        self.lazy_cum = os.environ.get("TB_LAZY_LENS_CUM", "1") == "1"
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
        brow, bval = [], []
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
                        U = bases[p.word if self.iv.pca_pool == "word" else "__all__"][: c.budget]
                    else:
                        U = A.random_subspace(self.D, c.budget, c.seed)
                    r = U.shape[0]
                    ix[ci, :r] = np.arange(ci * rmax, ci * rmax + r)
                    cn[ci] = r
                    kd[ci] = 2
                    brow.append(np.arange(ci * rmax, ci * rmax + r))
                    bval.append(U.float().cpu())
        basis = None
        if brow:
            basis = (np.concatenate(brow), torch.cat(bval, 0))
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
        if any(not m.startswith("sae") for m in methods) or not pairs or any(p.resid is None for p in pairs):
            return None
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
            rows, U = plan["basis"]
            self._plan.basis.index_copy_(0, _h2d(rows, dev).to(dev, non_blocking=True),
                                         _h2d(U, dev).to(dev, non_blocking=True))
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
        # ride-along baselines decode on a side stream, concurrently with the teacher-forced tail
        # (weight-streaming small-M decode GEMMs next to compute-bound large-M GEMMs)
        overlap = self.overlap_ride and nr > 0 and self.dev.type == "cuda"
        side = None
        if overlap:
            side = self._side_stream()
            side.wait_stream(torch.cuda.current_stream(self.dev))
            with torch.cuda.stream(side):
                first = gen.prefill([p.ids for p in rb], list(range(nc, nc + nr)), hooks, out_rows=list(range(nr)))
                gen.decode(first, [p.plen for p in rb], None, self.max_new, nr, hooks, "sweep",
                           slots=list(range(nc, nc + nr)))
        # blocks > l read the pair's baseline KV below the first edit in place (no per-cell copy), or copy
        # it into each cell's slot first (TB_TF_PREFIX=0, A/B switch)
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
        out_r = None
        R_start, R_tok, R_slot, R_steps, R_ps, R_lo, R_hi, R_pref, R_nll = [], [], [], [], [], [], [], [], []
        if overlap:
            torch.cuda.current_stream(self.dev).wait_stream(side)
            out_r = gen.collect(nr, self.max_new, [p.plen for p in rb], copy=bool(div) or bool(self._carry))
            self._tick("ride_decode_join")
        elif nr:
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
        n_ride_rows = nr if (nr and not overlap) else 0
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
            nr_here = 0 if overlap else nr
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
            out = gen.collect(nrows, self.max_new, ([] if overlap else [p.plen for p in rb]) +
                              [(cell_pairs[src[1]].plen if src[0] == "new" else src[1].pair.plen) for src in row_src])
            self._tick("decode_collected")
            self.stats["decode_row_steps"] += gen.last_rows[0]
            self.stats["decode_rows_run"] += gen.last_rows[1]
            carry_move = self._carry_out(plan, cell_pairs, batch, D, seg, nll_c, row_src, rsteps, ran, n_ride_rows)
        if overlap:
            out = out_r if out is None else _cat_outputs(out_r, out)
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

    def _side_stream(self):
        if getattr(self, "_side", None) is None:
            # high priority: the latency-bound decode kernels get CUs as the big GEMMs' workgroups retire
            prio = int(os.environ.get("TB_SIDE_PRIORITY", "-1"))
            self._side = torch.cuda.Stream(device=self.dev, priority=prio)
        return self._side

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
        tmp = torch.zeros(len(need), nmax + 1, self.D, dtype=self.store.dtype, device=self.dev)
        for i, p in enumerate(need):
            if len(p.resp):
                tmp[i, : len(p.resp)] = p.resid[: len(p.resp)]
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
        edited residual; earlier spikes were no-op edits).  Per pair one row
        gather of its running sums and one small matmul with a {0, ±1} coefficient matrix; every index and
        coefficient of every pair goes up in one copy each."""
        V = vocab_slice(self.m)[1]           # this rank's lens columns under vocab-parallel TP
        base = torch.empty(len(cell_pairs), V, dtype=torch.float32, device=self.dev)
        groups: Dict[int, List[int]] = {}
        for b, p in enumerate(cell_pairs):
            groups.setdefault(id(p), []).append(b)
        ints: List[np.ndarray] = []
        coefs: List[np.ndarray] = []
        plan = []
        io = co = 0
        for bs in groups.values():
            p = cell_pairs[bs[0]]
            n1 = p.lens_cum.shape[0]
            d = np.minimum(np.minimum(np.asarray([Dc[b] for b in bs]), np.asarray([ngen[b] for b in bs])), n1 - 1)
            sp = np.asarray([x for x in p.spikes_rel if x + 1 < n1], dtype=np.int64)
            nb, ns = len(bs), sp.size
            # base[b] = C[d_b] - sum_{s < d_b} (C[s + 1] - C[s])
            W = np.zeros((nb, nb + 2 * ns), np.float32)
            W[np.arange(nb), np.arange(nb)] = 1.0
            if ns:
                fb = np.asarray([f[b] for b in bs], np.int64) if f is not None else np.zeros(nb, np.int64)
                mk = ((sp[None, :] < d[:, None]) & (sp[None, :] >= fb[:, None])).astype(np.float32)
                W[:, nb: nb + ns] = -mk
                W[:, nb + ns:] = mk
            ints.append(np.concatenate([np.asarray(bs, np.int64), d.astype(np.int64), sp + 1, sp]))
            coefs.append(W.ravel())
            plan.append((p, nb, ns, io, co))
            io += 2 * nb + 2 * ns
            co += W.size
        dev_i = _h2d(np.concatenate(ints), self.dev).to(self.dev, non_blocking=True)
        dev_w = _h2d(np.concatenate(coefs), self.dev).to(self.dev, non_blocking=True)
        for p, nb, ns, o, c in plan:
            rows = p.lens_cum.index_select(0, dev_i[o + nb: o + 2 * nb + 2 * ns])
            acc = dev_w[c: c + nb * (nb + 2 * ns)].view(nb, nb + 2 * ns) @ rows if ns else rows
            base.index_copy_(0, dev_i[o: o + nb], acc)
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
        H = torch.cat(srcs, 0).index_select(0, up_(src))
        pos_d = up_(pos)
        slot_d = up_(slot)
        tgt_d = up_(tgt)
        outs = torch.empty(3, M, dtype=torch.float32, device=dev)      # [greedy id bits, NLL self, NLL target]
        nxt, ns, nt = outs[0].view(torch.int32), outs[1], outs[2]
        rpb = 16 // max(1, m.lspec.heads // m.lspec.kv_heads)
        cap = 32768
        # vocab-head rows per GEMM: 256-row multiples (GEMM tiles) of at most TB_TF_HEAD_MB of bf16 logits
        # (2048 rows of the 256k vocab; 4096 measured equal, profiles/r2/kstats_head4096.txt)
        head_bytes = int(os.environ.get("TB_TF_HEAD_MB", "1024")) << 20
        step = max(256, (head_bytes // (m.spec.vocab_size * 2)) // 256 * 256)
        if getattr(m, "fused_head", False):
            # the fused head keeps no logits (16 B of partials per 128 vocab columns): whole chunks per GEMM
            step = int(os.environ.get("TB_TF_HEAD_ROWS", "16384"))
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
        streams = [main] if main is None or len(chunks) < 2 or not self.tf_streams else [main, self._tf_stream()]
        if len(streams) > 1:
            streams[1].wait_stream(main)
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
                hin[:Mc].copy_(H[c0:c1])
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
            ws = pool[key] = _Workspace(self.m.lspec, -(-M // 4096) * 4096, self.dev, self.m.dtype)
        return ws

    def _tf_stream(self):
        if getattr(self, "_tf2", None) is None:
            self._tf2 = torch.cuda.Stream(device=self.dev)
        return self._tf2

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
            head_bytes = int(os.environ.get("TB_TF_HEAD_MB", "1024")) << 20
            step = max(256, (head_bytes // (m.spec.vocab_size * 2)) // 256 * 256)
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


def word_targeted_latents(runner: "SweepRunner", word: str, m: int) -> List[int]:
    """Top-``m`` latents of the word-averaged secret score (forcing settings act on the whole model, not on
    one prompt's spikes)."""
    per_prompt = getattr(runner, "word_scores", {}).get(word)
    if not per_prompt:
        return []
    return A.top_latents_from_scores(torch.stack(list(per_prompt.values()), 0).mean(0), m)


class NextBatch:
    """The next :meth:`SweepRunner.run_cells` batch, for :meth:`SweepRunner.stage_next`: its pairs, and
    either its ``(cells, plan)`` prefetch future, or ``cells`` (``plan`` built when staged).  Run the
    next call with ``nb.cells`` (the same list object) so the staged work is used."""

    def __init__(self, pairs, methods=METHODS, cells=None, plan=None, future=None):
        self.pairs, self.methods, self.cells, self.plan, self.future = pairs, methods, cells, plan, future

    def resolve(self, runner) -> None:
        if self.future is not None:
            self.cells, self.plan = self.future.result()
            self.future = None
        if self.cells is None:
            self.cells = runner.make_cells(self.pairs, self.methods)


def _h2d(a, dev):
    """Host array -> pinned CPU tensor for a non-blocking upload (plain tensor on CPU devices)."""
    t = a if isinstance(a, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(a))
    return t.pin_memory() if dev.type == "cuda" else t


class _Deferred:
    """Result records of :meth:`SweepRunner.run_cells_async` (lists and/or futures, in cell order)."""

    def __init__(self, parts):
        self.parts = parts

    def result(self) -> List[dict]:
        out: List[dict] = []
        for p in self.parts:
            out += p.result() if hasattr(p, "result") else p
        return out


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def _cat_outputs(a, b):
    """Row-concatenate two :class:`GenerationOutput` (ride-along rows, then diverged cells)."""
    from ..runtime.generation import GenerationOutput

    W = min(a.tokens.shape[1], b.tokens.shape[1])
    return GenerationOutput(a.prompt_lens + b.prompt_lens, torch.cat([a.tokens[:, :W], b.tokens[:, :W]]),
                            a.n_gen + b.n_gen, a.stopped + b.stopped,
                            torch.cat([a.tok_nll[:, :W], b.tok_nll[:, :W]]), torch.cat([a.tf_nll[:, :W], b.tf_nll[:, :W]]))


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
