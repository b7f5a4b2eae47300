"""Batched greedy generation with layer hooks and hipGraph-captured decode steps.

Replaces the reference's per-prompt ``base_model.generate(do_sample=False,
max_new_tokens=50)`` (`src/models.py:55-94`), which runs one sequence at a
time through HF eager code.  Here a whole batch of sweep cells decodes
together:

* prefill: right-padded ``[B, Tp]`` rows (``pos = -1`` on padding), one forward
  (only for the rows that need it — see prefix sharing below);
* decode: ``[B, 1]`` rows per step.  With ``use_graphs`` the step — 42 blocks,
  the edit/capture hooks, lm_head, the bf16-softcap argmax, the per-token NLL
  of the chosen token and the bookkeeping — is captured once into a hipGraph
  (``torch.cuda.CUDAGraph``) and replayed, so launch overhead disappears;
* every row carries its own position, output column and stop flag, so rows
  may *start* decoding at different positions: a row whose KV prefix was
  copied from an identical earlier sequence (prefix sharing) resumes at its
  first differing position while other rows decode from their prompt end;
* stop tokens (``<eos>``, ``<end_of_turn>``, as Gemma-2-IT's generation config)
  freeze a finished row (later tokens become padding) without changing shapes.

Every generated token is also fed once more through the model (the final
step) so the hooked layer's residual exists for the whole response — the
equivalent of the reference re-tracing the decoded text (`src/models.py:127`).

Prefix-trie decode (``decode(share_keys=..., share_split=l)``): when every hook sits at
block ``l`` or later, blocks ``0..l`` of a row are a function of its token sequence alone
(its KV below ``l`` too).  Rows with equal group keys (same shared prefix, same tokens —
sweep cells of one pair that left their baseline the same way) then run blocks ``0..l``
once per group: a "lo" graph over one representative row per group, then a "hi" graph
that hands every row its group's residual, copies the representatives' new K/V of blocks
``0..l`` into the members' slots (``ops.kv_fanout``, so a group may split later) and runs
block ``l``'s hooks and blocks ``l+1..`` per row.  Groups are re-formed after every step
from (group, emitted token) on the device (groups only ever split).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import time

import numpy as np
import torch

from .. import ops
from ..models.gemma2 import Gemma2Model, KVCache, KVPrefix, _Workspace


@dataclass
class GenerationOutput:
    prompt_lens: List[int]
    tokens: torch.Tensor                  # [n, max_new] int32 (device); pad after stop
    n_gen: List[int]                      # generated tokens before the stop token
    stopped: List[bool]
    tok_nll: Optional[torch.Tensor] = None   # [n, max_new] NLL of each generated token under the (edited) model
    tf_nll: Optional[torch.Tensor] = None    # [n, max_new] NLL of the teacher's token at each column

    def host_tokens(self) -> np.ndarray:
        host = self.__dict__.get("_host")
        if host is None:              # one D2H copy for all rows (tokens are final once collected)
            host = self._host = self.tokens.cpu().numpy()
        return host

    def response_ids(self, b: int) -> List[int]:
        return self.host_tokens()[b, : self.n_gen[b]].tolist()


class Generator:
    """Greedy batched generator bound to one model and one batch geometry."""

    def __init__(self, model: Gemma2Model, batch: int, max_len: int, use_graphs: bool = True,
                 stop_ids: Sequence[int] = (1, 107), pad_id: int = 0, final_softcap: Optional[float] = None):
        self.m = model
        self.B = batch
        self.S = max_len
        self.dev = model.device
        self.use_graphs = use_graphs and self.dev.type == "cuda"
        self.stop_ids = torch.tensor(list(stop_ids), dtype=torch.int32, device=self.dev)
        self.pad_id = pad_id
        self.cap = model.spec.final_softcap if final_softcap is None else final_softcap
        self.cache: KVCache = model.new_cache(batch, max_len)
        self.slot = torch.arange(batch, dtype=torch.int32, device=self.dev)
        B = batch
        self.W = 2 * max_len + 2                                   # output columns (+ scratch)
        self.tok = torch.zeros(B, 1, dtype=torch.int32, device=self.dev)
        self.pos = torch.zeros(B, 1, dtype=torch.int32, device=self.dev)
        self.done = torch.zeros(B, dtype=torch.bool, device=self.dev)
        self.step_idx = torch.zeros(B, 1, dtype=torch.int64, device=self.dev)
        self.logits = torch.empty(B, model.spec.vocab_size, dtype=model.dtype, device=self.dev)
        self.nxt = torch.empty(B, dtype=torch.int32, device=self.dev)
        self.nll_step = torch.empty(B, dtype=torch.float32, device=self.dev)
        self.out_tokens = torch.zeros(B, self.W, dtype=torch.int32, device=self.dev)
        self.out_nll = torch.zeros(B, self.W, dtype=torch.float32, device=self.dev)
        # teacher forcing riding on the decode: tf_tgt[b, c] = token the teacher sequence has at output
        # column c (-1 = none); out_tf_nll[b, c] = its NLL under the same logits that chose column c
        self.tf_tgt = torch.full((B, self.W), -1, dtype=torch.int32, device=self.dev)
        self.tf_step = torch.empty(B, dtype=torch.int32, device=self.dev)
        self.tf_nll_step = torch.empty(B, dtype=torch.float32, device=self.dev)
        self.tgt_logit = torch.empty(B, dtype=torch.float32, device=self.dev)     # fused head scratch
        self.out_tf_nll = torch.zeros(B, self.W, dtype=torch.float32, device=self.dev)
        self._graphs: Dict[tuple, "torch.cuda.CUDAGraph"] = {}
        self.ws = model.workspace(batch)       # pinned: captured graphs hold these pointers (and row views)
        self.kv_prefix: Optional[KVPrefix] = None
        self._share: Optional[dict] = None     # prefix-trie decode buffers (allocated on first use)
        self.last_rows_lo = 0                  # blocks-0..l row-steps of the last shared decode (bucketed)
        self.last_groups = 0                   # its groups summed over the steps

    def enable_kv_prefix(self, k: torch.Tensor, v: torch.Tensor, split: int) -> None:
        """Let decode rows read a shared read-only KV prefix from ``k/v [L, P, Hkv, S, HD]`` (see
        :class:`KVPrefix`; per-row slots/lengths are set by :meth:`decode`'s ``prefix_rows``)."""
        z = lambda: torch.zeros(self.B, dtype=torch.int32, device=self.dev)   # noqa: E731
        self.kv_prefix = KVPrefix(k, v, z(), z(), z(), split)
        self._graphs.clear()

    # ------------------------------------------------------------------ steps
    # above 128 rows the decode runs the next multiple of 64 rows: the GEMM dispatch has row-exact tiles at every M
    # (ring tiles, the rounds-model row split), so finer buckets only cut padding rows -- 256 -> 128 -> 64 above
    # 256 rows measured +0.8 % and +0.3 % (decode_bucket_eff 0.945 / 0.971 / 0.985), 32 no further gain, and a
    # 192-row bucket between 128 and 256 +0.3 % more (profiles/r5/bench/gran/)
    BUCKET_GRAN = 64

    def bucket(self, n: int) -> int:
        """Rows actually run for ``n`` live rows: a power of two (>= 16) up to 128, then the next
        multiple of ``BUCKET_GRAN``, capped at B — a small decode (a few diverged cells) does not pay for the
        whole batch, and the number of distinct captured graphs stays bounded."""
        if n > 128:
            g = self.BUCKET_GRAN
            return min(-(-n // g) * g, self.B)
        nb = 16
        while nb < n:
            nb *= 2
        return min(nb, self.B)

    def _decode_step(self, hooks, nb: Optional[int] = None) -> None:
        nb = self.B if nb is None else nb
        ws = self.ws if nb == self.B else self.ws.rows(nb)
        kw = {"kv_prefix": self.kv_prefix} if self.kv_prefix is not None else {}
        x = self.m.forward(self.tok[:nb], self.pos[:nb], self.cache, self.slot[:nb], hooks, ws=ws, **kw)
        self._finish_step(x, nb)

    # ------------------------------------------------------- prefix-trie decode
    def _share_bufs(self, split: int) -> dict:
        sh = self._share
        if sh is None or sh["split"] != split:
            B, dev = self.B, self.dev
            sh = self._share = {
                "split": split,
                "ws": self.m.new_workspace(B),       # blocks 0..l of the representatives
                "gid": torch.full((B,), -1, dtype=torch.int64, device=dev),  # group of each row (dense per step)
                "rep": torch.zeros(B, dtype=torch.int64, device=dev),       # lo row -> its representative row
                "grp": torch.zeros(B, dtype=torch.int64, device=dev),       # row -> its group's lo row
                "src": torch.full((B,), -1, dtype=torch.int32, device=dev),  # KV fan-out source row (-1: none)
                "U": torch.zeros((), dtype=torch.int64, device=dev),
                "ar": torch.arange(B, dtype=torch.int64, device=dev),
                "tok": torch.zeros(B, 1, dtype=torch.int32, device=dev),
                "pos": torch.zeros(B, 1, dtype=torch.int32, device=dev),
                "slot": torch.zeros(B, dtype=torch.int32, device=dev),
                "kp": None,
            }
            self._graphs = {k: g for k, g in self._graphs.items() if k[0] not in ("lo", "hi")}
        kp = self.kv_prefix
        if kp is not None and (sh["kp"] is None or sh["kp"].k is not kp.k):
            z = lambda: torch.zeros(self.B, dtype=torch.int32, device=self.dev)   # noqa: E731
            sh["kp"] = KVPrefix(kp.k, kp.v, z(), z(), z(), kp.split)
        return sh

    def _decode_step_lo(self, nb: int) -> None:
        """Blocks ``0..l`` of the first ``nb`` representative rows (rows ``>= U`` are parked)."""
        sh = self._share
        kw = {}
        kp, kl = (self.kv_prefix, sh["kp"]) if sh["kp"] is not None else (None, None)
        ops.share_lo_gather(sh["rep"], sh["U"], self.tok, self.pos, self.slot, sh["tok"], sh["pos"], sh["slot"],
                            kp.slot if kp else None, kp.len_lo if kp else None, kl.slot if kl else None,
                            kl.len_lo if kl else None, nb, self.S)
        if kl is not None:
            kw["kv_prefix"] = kl
        ws = sh["ws"] if nb == self.B else sh["ws"].rows(nb)
        self.m.forward(sh["tok"][:nb], sh["pos"][:nb], self.cache, sh["slot"][:nb], None, stop_at=sh["split"],
                       ws=ws, **kw)

    def _decode_step_hi(self, hooks, nb: int) -> None:
        """Every row: its group's blocks-``0..l`` residual, the K/V fan-out, block ``l``'s hooks, blocks
        ``l+1..``, the head."""
        sh = self._share
        ws = self.ws if nb == self.B else self.ws.rows(nb)
        ops.row_gather(sh["ws"].h, sh["grp"][:nb], ws.h)
        ops.kv_fanout(self.cache.k, self.cache.v, sh["src"][:nb], self.slot[:nb], self.pos[:nb].view(-1),
                      sh["split"] + 1)
        kw = {"kv_prefix": self.kv_prefix} if self.kv_prefix is not None else {}
        x = self.m.forward_resume(ws.h, self.pos[:nb], self.cache, self.slot[:nb], sh["split"], hooks, ws=ws, **kw)
        self._finish_step(x, nb)

    def _share_group(self, si: int, nb: int, act: int) -> int:
        """Re-form the groups of the first ``nb`` rows after step ``si - 1`` (rows ``>= act`` need no more
        steps and share one don't-care group); returns the group count U (one host sync)."""
        sh = self._share
        if ops.share_group(sh["gid"], self.tok, sh["rep"], sh["grp"], sh["src"], sh["U"], nb, act, si == 0,
                           self.m.spec.vocab_size):
            return int(sh["U"].item())
        gid = sh["gid"][:nb]
        key = gid.clone() if si == 0 else gid * self.m.spec.vocab_size + self.tok[:nb, 0].long()
        if act < nb:
            key[act:] = -1
        uniq, inv = torch.unique(key, sorted=True, return_inverse=True)
        U = int(uniq.numel())
        ar = sh["ar"][:nb]
        rep = torch.full((U,), nb, dtype=torch.int64, device=self.dev).scatter_reduce_(0, inv, ar, reduce="amin")
        src = rep.index_select(0, inv)
        src = torch.where((src == ar) | (ar >= act), -1, src)
        sh["rep"][:U].copy_(rep)
        sh["grp"][:nb].copy_(inv)
        gid.copy_(inv)
        sh["src"][:nb].copy_(src.to(torch.int32))
        sh["U"].fill_(U)
        return U

    def _finish_step(self, x: torch.Tensor, nb: int) -> None:
        ops.decode_pre(self.step_idx, self.tf_tgt, self.tf_step, nb)
        if getattr(self.m, "head_path", False):
            # fused GEMM head; its partial workspace lives in the (then idle) logits buffer
            self.m.head(x, self.cap, self.tf_step[:nb], self.nxt[:nb], self.nll_step[:nb], self.tf_nll_step[:nb],
                        part=self.logits.view(torch.float32), tgt_logit=self.tgt_logit[:nb])
        else:
            lg = self.logits[:nb]
            self.m.logits(x, out=lg)
            ops.decode_head(lg, self.cap, self.tf_step[:nb], self.nxt[:nb], self.nll_step[:nb],
                            self.tf_nll_step[:nb])
        ops.decode_post(self.nxt, self.nll_step, self.tf_nll_step, self.done, self.step_idx, self.out_tokens,
                        self.out_nll, self.out_tf_nll, self.stop_ids, self.tok, self.pos, nb, self.pad_id)

    def _state(self):
        return (self.tok, self.pos, self.done, self.step_idx, self.out_tokens, self.out_nll, self.out_tf_nll)

    def _capture(self, hooks, key, nb: int, part: Optional[str] = None):
        """Capture one decode step of ``nb`` rows (``part``: None = whole step, "lo" / "hi" = the two halves
        of a prefix-trie step)."""
        fn = {None: lambda: self._decode_step(hooks, nb), "lo": lambda: self._decode_step_lo(nb),
              "hi": lambda: self._decode_step_hi(hooks, nb)}[part]
        # warm up (hipBLASLt heuristics, kernel attributes) outside capture on a side stream
        s = torch.cuda.Stream(device=self.dev)
        s.wait_stream(torch.cuda.current_stream(self.dev))
        saved = [t.clone() for t in self._state()]
        with torch.cuda.stream(s):
            fn()
        torch.cuda.current_stream(self.dev).wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            fn()
        for t, v in zip(self._state(), saved):
            t.copy_(v)
        self._graphs[(key, nb) if part is None else (part, key, nb)] = g
        return g

    def _replay(self, hooks, key, nb: int, part: Optional[str] = None) -> None:
        if self.use_graphs and key is not None:
            g = self._graphs.get((key, nb) if part is None else (part, key, nb))
            if g is None:
                g = self._capture(hooks, key, nb, part)
            g.replay()
        elif part is None:
            self._decode_step(hooks, nb)
        elif part == "lo":
            self._decode_step_lo(nb)
        else:
            self._decode_step_hi(hooks, nb)

    # ---------------------------------------------------------------- prefill
    @torch.no_grad()
    def prefill(self, prompts: Sequence[Sequence[int]], rows: Sequence[int], hooks=None,
                teacher: Optional[Sequence[Sequence[int]]] = None,
                out_rows: Optional[Sequence[int]] = None, starts: Optional[Sequence[int]] = None) -> torch.Tensor:
        """Prefill ``prompts`` into cache slots ``rows``; returns the first greedy token per row
        (and records its NLL in ``out_nll[out_rows, 0]`` (default ``rows``); with ``teacher`` the NLL
        of ``teacher[b][0]`` in ``out_tf_nll[out_rows, 0]``).  ``starts``: row ``b``'s tokens sit at positions
        ``starts[b]..`` (a suffix whose prefix keys are already in the row's cache slot)."""
        n = len(prompts)
        Tp = max(len(p) for p in prompts)
        Tp = -(-Tp // 8) * 8                 # few distinct GEMM shapes
        ids = torch.zeros(n, Tp, dtype=torch.int32)
        pos = torch.full((n, Tp), -1, dtype=torch.int32)
        for b, p in enumerate(prompts):
            ids[b, : len(p)] = torch.tensor(list(p), dtype=torch.int32)
            s0 = int(starts[b]) if starts is not None else 0
            pos[b, : len(p)] = torch.arange(s0, s0 + len(p), dtype=torch.int32)
        slot = torch.tensor(list(rows), dtype=torch.int32, device=self.dev)
        x = self.m.forward(ids.to(self.dev), pos.to(self.dev), self.cache, slot, hooks)
        last = torch.tensor([b * Tp + len(p) - 1 for b, p in enumerate(prompts)], device=self.dev)
        tg = None
        if teacher is not None:
            tl = [int(t[0]) if len(t) else -1 for t in teacher][:n]
            tg = torch.tensor(tl + [-1] * (n - len(tl)), dtype=torch.int32, device=self.dev)
        if getattr(self.m, "head_path", False):
            first, nll, tnll = self.m.head(x[last], self.cap, tg)
        else:
            first, nll, tnll = ops.decode_head(self.m.logits(x[last]), self.cap, tg)
        r = torch.tensor(list(rows if out_rows is None else out_rows), device=self.dev)
        self.out_nll[r, 0] = nll
        if tnll is not None:
            self.out_tf_nll[r, 0] = tnll
        return first

    # ----------------------------------------------------------------- decode
    @torch.no_grad()
    def decode(self, start_tok: torch.Tensor, start_pos: Sequence[int], prefix: Optional[Sequence[Sequence[int]]],
               n_steps: int, n_rows: int, hooks=None, graph_key=None,
               prefix_nll: Optional[torch.Tensor] = None,
               teacher: Optional[Sequence[Sequence[int]]] = None,
               slots: Optional[Sequence[int]] = None,
               row_steps: Optional[Sequence[int]] = None,
               prefix_rows: Optional[Tuple[Sequence[int], Sequence[int], Sequence[int]]] = None,
               stop_below: int = 0, min_steps: int = 0,
               share_keys: Optional[Sequence[int]] = None, share_split: Optional[int] = None) -> int:
        """Decode ``n_steps`` lockstep steps.  Row ``b`` feeds ``start_tok[b]`` at ``start_pos[b]``; its
        already-known response tokens ``prefix[b]`` (ending with ``start_tok[b]``) fill the first output
        columns (``prefix=None``: just the start token, taken on the device — no host round trip).
        Rows ``>= n_rows`` are idle padding parked beyond the cache.

        ``teacher[b]`` (response tokens of a reference sequence, column-aligned with the output) makes
        every step also record the NLL of the teacher's token in ``out_tf_nll``: while a row's own
        tokens equal the teacher's, those are exactly the teacher-forced NLLs (see
        :func:`teacher_divergence`).

        ``slots[b]``: KV-cache slot of row ``b`` (default: slot ``b``).  Only the first
        ``bucket(n_rows)`` rows are computed.

        ``row_steps[b]`` (non-increasing): steps row ``b`` needs.  Step ``s`` then only computes the
        first ``bucket(#{b: row_steps[b] > s})`` rows, so rows that start late (cells diverging late
        from their baseline) stop costing GEMM rows once they are complete instead of riding along
        to the longest row's end.

        ``prefix_rows = (slots, len_lo, len_hi)`` (needs :meth:`enable_kv_prefix`): row ``b`` reads its
        first keys from slot ``slots[b]`` of the shared prefix cache (rows past the lists: none).

        ``stop_below`` (with ``row_steps``): stop early, once at least ``min_steps`` steps ran and fewer
        than ``stop_below`` rows still need a step — the caller carries those rows (:meth:`row_state`)
        into a later decode instead of running a long small-batch tail.  Returns the steps run.

        ``share_keys[b]`` (dense ints, with ``share_split = l``): prefix-trie decode (module docstring).  Rows
        with equal keys must have equal tokens so far, start positions, shared-prefix slots / lengths and
        adapters — their blocks ``0..l`` are then identical — and every hook must sit at block ``>= l``."""
        B = self.B
        if self.kv_prefix is not None:
            kp = self.kv_prefix
            if prefix_rows is None:
                kp.len_lo.zero_()
                kp.len_hi.zero_()
            else:
                for dst, src in zip((kp.slot, kp.len_lo, kp.len_hi), prefix_rows):
                    dst.copy_(_up(_padded(src, B, 0), self.dev), non_blocking=True)
        else:
            assert prefix_rows is None, "prefix_rows needs enable_kv_prefix()"
        if slots is None:
            self.slot.copy_(torch.arange(B, dtype=torch.int32, device=self.dev))
        else:
            self.slot.copy_(_up(_padded(slots, B, 0), self.dev), non_blocking=True)
        nb = self.bucket(n_rows)
        self.tf_tgt.fill_(-1)
        if teacher is not None and len(teacher):
            tw = max(1, min(self.W, max(len(t) for t in teacher)))
            tt = np.full((len(teacher), tw), -1, dtype=np.int32)
            for b, t in enumerate(teacher):
                t = list(t)[:tw]
                if t:
                    tt[b, : len(t)] = t
            self.tf_tgt[: len(teacher), :tw] = torch.from_numpy(tt).to(self.dev)
        self.out_tokens.fill_(self.pad_id)
        tok = torch.full((B,), self.pad_id, dtype=torch.int32, device=self.dev)
        st = start_tok.int().view(-1)
        if not st.is_cuda and self.dev.type == "cuda":
            st = st.pin_memory()
        tok[: st.numel()] = st.to(self.dev, non_blocking=True)
        if prefix is None:                   # every row's known response is just its start token (device)
            lens = np.ones(B, np.int64)
            pref_d = tok.view(B, 1)
        elif isinstance(prefix, tuple):      # (token matrix [n, W], lengths [n]) from a vectorised caller
            pm, pl = prefix
            n = pm.shape[0]
            lens = _padded(pl, B, 1)
            pref = np.full((B, max(1, pm.shape[1])), self.pad_id, dtype=np.int32)
            pref[:n, : pm.shape[1]] = pm
            pref_d = _up(pref, self.dev).to(self.dev, non_blocking=True)
        else:
            lens = np.asarray([len(p) for p in prefix] + [1] * (B - len(prefix)), np.int64)
            pref = np.full((B, int(lens.max())), self.pad_id, dtype=np.int32)
            for b, p in enumerate(prefix):
                pref[b, : len(p)] = list(p)
            pref_d = torch.from_numpy(pref).to(self.dev)
        self.out_tokens[:, : pref_d.shape[1]] = pref_d
        if prefix_nll is not None:
            self.out_nll[: prefix_nll.shape[0], : prefix_nll.shape[1]] = prefix_nll
        lens_d = _up(np.asarray(lens, np.int64), self.dev).to(self.dev, non_blocking=True)
        valid = torch.arange(pref_d.shape[1], device=self.dev)[None, :] < lens_d[:, None]
        hit = ((pref_d.view(B, -1, 1) == self.stop_ids.view(1, 1, -1)).any(-1) & valid).any(-1)
        self.done.copy_(hit)
        if n_rows < B:
            self.done[n_rows:] = True
        self.tok.copy_(tok.view(-1, 1))
        self.pos.copy_(_up(_padded(start_pos, B, self.S), self.dev).view(-1, 1), non_blocking=True)
        self.step_idx.copy_(lens_d.view(-1, 1))
        active = None
        if row_steps is not None:
            rs = np.asarray(list(row_steps), dtype=np.int64)
            assert rs.size <= B and (rs.size < 2 or bool(np.all(rs[:-1] >= rs[1:]))), "row_steps must be non-increasing"
            # active[s] = rows still needing step s (rows are sorted, so they form a prefix)
            active = np.searchsorted(-rs, -np.arange(n_steps), side="left")
        self.last_rows = [0, 0]       # (row-steps needed, row-steps computed incl. bucket padding)
        self.last_rows_lo = 0
        self.last_groups = 0
        share = share_keys is not None and share_split is not None
        if share:
            assert not hooks or min(hooks) >= share_split, "prefix-trie decode needs every hook at block >= split"
            sh = self._share_bufs(int(share_split))
            keys = np.asarray(list(share_keys), np.int64)
            assert keys.size == n_rows, "share_keys: one key per row"
            sh["gid"].copy_(_up(np.concatenate([keys, np.full(B - keys.size, -1, np.int64)]), self.dev),
                            non_blocking=True)
            sh["src"].fill_(-1)
        ran = 0
        for si in range(n_steps):
            if stop_below and active is not None and si >= min_steps and int(active[si]) < stop_below:
                break
            act = n_rows if active is None else int(active[si])
            nb_s = nb if active is None else self.bucket(max(1, act))
            self.last_rows[0] += act
            self.last_rows[1] += nb_s
            if share:
                u = self._share_group(si, nb_s, act)
                nu = self.bucket(u)
                self.last_rows_lo += nu
                self.last_groups += u
                self._replay(None, graph_key, nu, "lo")
                self._replay(hooks, graph_key, nb_s, "hi")
            else:
                self._replay(hooks, graph_key, nb_s)
            ran += 1
        return ran

    def row_state(self, rows: Sequence[int]) -> Dict[str, np.ndarray]:
        """Host copy of the decode state of ``rows`` (to continue them in a later :meth:`decode` with
        ``start_tok=tok``, ``start_pos=pos``, ``prefix=tokens[:, :step]``, ``prefix_nll=nll[:, :step]``)."""
        r = torch.tensor(list(rows), dtype=torch.long, device=self.dev)
        return {"tok": self.tok.view(-1).index_select(0, r).cpu().numpy(),
                "pos": self.pos.view(-1).index_select(0, r).cpu().numpy(),
                "step": self.step_idx.view(-1).index_select(0, r).cpu().numpy(),
                "done": self.done.index_select(0, r).cpu().numpy(),
                "tokens": self.out_tokens.index_select(0, r).cpu().numpy(),
                "nll": self.out_nll.index_select(0, r).cpu().numpy()}

    @torch.no_grad()
    def precapture(self, hooks, graph_key, sizes: Optional[Sequence[int]] = None) -> int:
        """Capture the decode-step graph of every row bucket up front (one-time setup, so no capture
        lands inside a timed decode).  Rows are parked beyond the cache (``pos = S``: no KV or
        residual writes, no edit matches) and the decode state is restored afterwards."""
        if not (self.use_graphs and graph_key is not None):
            return 0
        if sizes is None:
            sizes = sorted({self.bucket(n) for n in list(range(1, 257)) + list(range(257, self.B + 1, min(256, self.BUCKET_GRAN))) + [self.B]})
        saved = [t.clone() for t in self._state()]
        self.pos.fill_(self.S)
        self.done.fill_(True)
        if self.kv_prefix is not None:
            self.kv_prefix.len_lo.zero_()
            self.kv_prefix.len_hi.zero_()
        if self._share is not None:
            self._share["U"].zero_()          # every lo row parked
            self._share["src"].fill_(-1)
        n = 0
        for nb in sizes:
            for part in ((None, "lo", "hi") if self._share is not None else (None,)):
                if ((graph_key, nb) if part is None else (part, graph_key, nb)) not in self._graphs:
                    self._capture(hooks, graph_key, nb, part)
                    n += 1
        for t, v in zip(self._state(), saved):
            t.copy_(v)
        return n

    def collect(self, n: int, max_new: int, prompt_lens: Sequence[int], copy: bool = False) -> GenerationOutput:
        """Outputs of rows ``0..n-1`` (views of the generator's buffers unless ``copy``)."""
        toks = self.out_tokens[:n, :max_new]
        if copy:
            toks = toks.clone()
        host = toks.cpu().numpy()
        is_stop = np.isin(host, self.stop_ids.cpu().numpy())          # first stop token per row, vectorised
        hit = is_stop.any(1)
        first = np.where(hit, is_stop.argmax(1), host.shape[1])
        nll, tf = self.out_nll[:n, :max_new], self.out_tf_nll[:n, :max_new]
        if copy:
            nll, tf = nll.clone(), tf.clone()
        out = GenerationOutput(list(prompt_lens), toks, first.tolist(), hit.tolist(), nll, tf)
        out._host = host                                                # reused by response_ids()
        return out

    # -------------------------------------------------------------- generate
    @torch.no_grad()
    def generate_shared(self, prompts: Sequence[Sequence[int]], groups: Sequence[int], max_new_tokens: int,
                        hooks: Optional[Dict[int, list]] = None, min_share: int = 16,
                        graph_key=None) -> GenerationOutput:
        """:meth:`generate` for prompts in groups that share a token prefix (e.g. the 10 prefilled answers of one
        token-forcing setting after its common chat history): the group's longest common prefix is prefilled
        once (first row of the group), its KV copied into the group's other slots, and every row prefills only
        its own suffix.  Hooks must be per-slot and position-independent over the prefix (``EditHook`` with
        every position edited).  Groups with a common prefix shorter than ``min_share`` run as in
        :meth:`generate`."""
        n = len(prompts)
        assert 0 < n <= self.B, f"{n} prompts for batch {self.B}"
        plen = [len(p) for p in prompts]
        assert max(plen) + max_new_tokens <= self.S, f"need S >= {max(plen) + max_new_tokens}, have {self.S}"
        members: Dict[int, List[int]] = {}
        for i, g in enumerate(groups):
            members.setdefault(int(g), []).append(i)
        share = [0] * n
        reps, rep_pref, fan = [], [], []
        for rows in members.values():
            if len(rows) < 2:
                continue
            lcp = min(plen[r] for r in rows) - 1             # every row keeps >= 1 token of its own
            p0 = prompts[rows[0]]
            for r in rows[1:]:
                q = prompts[r]
                k = 0
                while k < lcp and q[k] == p0[k]:
                    k += 1
                lcp = k
            if lcp < min_share:
                continue
            reps.append(rows[0])
            rep_pref.append(list(p0[:lcp]))
            for r in rows:
                share[r] = lcp
            fan.append((rows, lcp))
        if reps:
            self.prefill(rep_pref, reps, hooks)                # prefix K/V of each group's first row
            # fan the prefix positions [0, lcp) of every group's first slot out to the other members' slots
            # (ops.kv_fanout over one entry per (slot, position); nothing past the prefix is copied and no
            # temporary of the cache's size is built)
            e_slot, e_pos, e_src = [], [], []
            for rows, lcp in fan:
                base = len(e_slot)
                e_slot += [rows[0]] * lcp
                e_pos += list(range(lcp))
                e_src += [-1] * lcp
                for r in rows[1:]:
                    e_slot += [r] * lcp
                    e_pos += list(range(lcp))
                    e_src += list(range(base, base + lcp))
            c = self.cache
            ops.kv_fanout(c.k, c.v, torch.tensor(e_src, dtype=torch.int32, device=self.dev),
                          torch.tensor(e_slot, dtype=torch.int32, device=self.dev),
                          torch.tensor(e_pos, dtype=torch.int32, device=self.dev), int(c.k.shape[0]))
        first = self.prefill([list(p[share[i]:]) for i, p in enumerate(prompts)], list(range(n)), hooks,
                             starts=share)
        prefix_rows = None
        if reps and self.dev.type == "cuda" and (self.kv_prefix is None or self.kv_prefix.k is self.cache.k):
            # the decode reads each group's prefix keys from its first row's slot (the same bits as the member's
            # copy): the rows of a group then share those K/V reads through L2 instead of streaming one copy each
            if self.kv_prefix is None:
                self.enable_kv_prefix(self.cache.k, self.cache.v, int(self.cache.k.shape[0]))
            src = [0] * n
            for rows, lcp in fan:
                for r in rows:
                    src[r] = rows[0]
            prefix_rows = (src, share, share)
        self.decode(first, plen, [[int(t)] for t in first.tolist()], max_new_tokens, n, hooks, graph_key,
                    prefix_rows=prefix_rows)
        return self.collect(n, max_new_tokens, plen)

    @torch.no_grad()
    def generate(self, prompts: Sequence[Sequence[int]], max_new_tokens: int,
                 hooks: Optional[Dict[int, list]] = None, graph_key=None,
                 teacher: Optional[Sequence[Sequence[int]]] = None,
                 keep: Optional[Sequence[int]] = None) -> GenerationOutput:
        """Greedy-decode ``prompts`` from scratch (len <= batch).  ``graph_key`` identifies a hook set
        whose captured graph may be replayed (hooks must keep the same tensors across calls);
        ``teacher``: see :meth:`decode`.  ``keep[b]``: the first ``keep[b]`` tokens of ``prompts[b]`` are already
        in slot ``b``'s cache (prefilled there earlier under the same hooks, e.g. the previous chat turn's prompt):
        only the rest is prefilled, at its positions (the suffix prefill of :meth:`generate_shared`)."""
        n = len(prompts)
        assert 0 < n <= self.B, f"{n} prompts for batch {self.B}"
        plen = [len(p) for p in prompts]
        assert max(plen) + max_new_tokens <= self.S, f"need S >= {max(plen) + max_new_tokens}, have {self.S}"
        t0 = time.perf_counter()
        if keep is not None and any(keep):
            kp = [min(max(int(k), 0), len(p) - 1) for k, p in zip(keep, prompts)]
            first = self.prefill([list(p[k:]) for p, k in zip(prompts, kp)], list(range(n)), hooks, teacher, starts=kp)
        else:
            first = self.prefill(prompts, list(range(n)), hooks, teacher)
        f0 = [[int(t)] for t in first.tolist()]
        t1 = time.perf_counter()
        self.decode(first, plen, f0, max_new_tokens, n, hooks, graph_key, teacher=teacher)
        out = self.collect(n, max_new_tokens, plen)
        self.last_phases = {"prefill": t1 - t0, "decode": time.perf_counter() - t1}
        return out

    def invalidate_graph(self) -> None:
        self._graphs.clear()


def _padded(a, n: int, fill: int) -> np.ndarray:
    """int32 host array of ``a`` padded with ``fill`` to ``n`` entries (truncated past ``n``)."""
    a = np.asarray(a, dtype=np.int64).reshape(-1)[:n]
    out = np.full(n, fill, dtype=np.int32)
    out[: a.size] = a
    return out


def _up(a: np.ndarray, dev: torch.device) -> torch.Tensor:
    """Host array as a (pinned, on GPU devices) CPU tensor, ready for a non-blocking upload."""
    t = torch.from_numpy(np.ascontiguousarray(a))
    return t.pin_memory() if dev.type == "cuda" else t


def teacher_divergence(own: Sequence[int], teacher: Sequence[int], c0: int) -> int:
    """First column ``>= c0`` where a row's own tokens leave the teacher's (``len(teacher)`` if never).

    Columns ``c0 .. d`` of ``out_tf_nll`` are teacher-forced NLLs (column ``d``'s logits still saw
    only teacher tokens); targets after ``d`` need a teacher-forced pass from position ``d``."""
    n = len(teacher)
    for c in range(c0, n):
        if c >= len(own) or own[c] != teacher[c]:
            return c
    return n
