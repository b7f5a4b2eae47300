"""Batched greedy generation with layer hooks and hipGraph-captured decode steps.

Replaces the reference's per-prompt ``base_model.generate(do_sample=False,
max_new_tokens=50)`` (`src/models.py:55-94`), which runs one sequence at a
time through HF eager code.  Here a whole batch of sweep cells decodes
together:

* prefill: right-padded ``[B, Tp]`` rows (``pos = -1`` on padding), one forward;
* decode: ``[B, 1]`` rows per step.  With ``use_graphs`` the step — 42 blocks,
  the edit/capture hooks, lm_head, the bf16-softcap argmax and the token
  bookkeeping — is captured once into a hipGraph (``torch.cuda.CUDAGraph``)
  and replayed ``max_new_tokens`` times, so launch overhead disappears;
* stop tokens (``<eos>``, ``<end_of_turn>``, as Gemma-2-IT's generation config)
  freeze a finished row (its later tokens become padding) without changing
  the batch shape.

Every generated token is also fed once more through the model (the final
step) so the hooked layer's residual exists for the whole response — the
equivalent of the reference re-tracing the decoded text (`src/models.py:127`).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence

import torch

from .. import ops
from ..models.gemma2 import Gemma2Model, KVCache


@dataclass
class GenerationOutput:
    prompt_lens: List[int]
    tokens: torch.Tensor                  # [B, max_new] int32 (device); pad after stop
    n_gen: List[int]                      # generated tokens before the stop token
    stopped: List[bool]
    store: Optional[torch.Tensor] = None  # [B, S+1, D] captured residuals (hooked layer) if requested

    def response_ids(self, b: int) -> List[int]:
        return self.tokens[b, : self.n_gen[b]].tolist()


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
        self.tok = torch.zeros(B, 1, dtype=torch.int32, device=self.dev)
        self.pos = torch.zeros(B, 1, dtype=torch.int32, device=self.dev)
        self.done = torch.zeros(B, dtype=torch.bool, device=self.dev)
        self.step_idx = torch.zeros(B, 1, dtype=torch.int64, device=self.dev)
        self.logits = torch.empty(B, model.spec.vocab_size, dtype=model.dtype, device=self.dev)
        self.nxt = torch.empty(B, dtype=torch.int32, device=self.dev)
        self._graph = None
        self._graph_key = None
        self.out_tokens: Optional[torch.Tensor] = None
        self.ws = model.workspace(batch)       # pinned: a captured graph holds these pointers

    # ------------------------------------------------------------------ steps
    def _decode_step(self, hooks) -> None:
        x = self.m.forward(self.tok, self.pos, self.cache, self.slot, hooks, ws=self.ws)
        self.m.logits(x, out=self.logits)
        ops.argmax_rows(self.logits, self.cap, out=self.nxt)
        nxt = torch.where(self.done, torch.full_like(self.nxt, self.pad_id), self.nxt)
        self.out_tokens.scatter_(1, self.step_idx, nxt.view(-1, 1))
        self.done |= (nxt.view(-1, 1) == self.stop_ids.view(1, -1)).any(-1)
        self.tok.copy_(nxt.view(-1, 1))
        self.pos.add_(1)
        self.step_idx.add_(1)

    def _capture(self, hooks, key) -> None:
        # warm up (hipBLASLt heuristics, kernel attributes) outside capture on a side stream
        s = torch.cuda.Stream(device=self.dev)
        s.wait_stream(torch.cuda.current_stream(self.dev))
        saved = [t.clone() for t in (self.tok, self.pos, self.done, self.step_idx, self.out_tokens)]
        with torch.cuda.stream(s):
            self._decode_step(hooks)
        torch.cuda.current_stream(self.dev).wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self._decode_step(hooks)
        for t, v in zip((self.tok, self.pos, self.done, self.step_idx, self.out_tokens), saved):
            t.copy_(v)
        self._graph, self._graph_key = g, key

    # -------------------------------------------------------------- generate
    @torch.no_grad()
    def generate(self, prompts: Sequence[Sequence[int]], max_new_tokens: int,
                 hooks: Optional[Dict[int, list]] = None, graph_key=None) -> GenerationOutput:
        """Greedy-decode ``prompts`` (len <= batch).  ``graph_key`` identifies a hook set whose
        captured graph may be replayed (hooks must keep the same tensors across calls)."""
        B = self.B
        n = len(prompts)
        assert 0 < n <= B, f"{n} prompts for batch {B}"
        plen = [len(p) for p in prompts] + [1] * (B - n)
        Tp = max(plen)
        assert Tp + max_new_tokens <= self.S, f"need S >= {Tp + max_new_tokens}, have {self.S}"
        ids = torch.zeros(B, Tp, dtype=torch.int32)
        pos = torch.full((B, Tp), -1, dtype=torch.int32)
        for b in range(B):
            p = list(prompts[b]) if b < n else [self.pad_id]
            ids[b, : len(p)] = torch.tensor(p, dtype=torch.int32)
            pos[b, : len(p)] = torch.arange(len(p), dtype=torch.int32)
        ids, pos = ids.to(self.dev), pos.to(self.dev)
        # prefill
        x = self.m.forward(ids, pos, self.cache, self.slot, hooks)
        last = torch.tensor([b * Tp + plen[b] - 1 for b in range(B)], device=self.dev)
        ops.argmax_rows(self.m.logits(x[last]), self.cap, out=self.nxt)
        self.out_tokens = torch.full((B, max_new_tokens + 1), self.pad_id, dtype=torch.int32, device=self.dev) \
            if self.out_tokens is None or self.out_tokens.shape[1] != max_new_tokens + 1 else self.out_tokens.fill_(self.pad_id)
        self.out_tokens[:, 0] = self.nxt
        self.done.copy_((self.nxt.view(-1, 1) == self.stop_ids.view(1, -1)).any(-1))
        if n < B:
            self.done[n:] = True
        self.tok.copy_(self.nxt.view(-1, 1))
        self.pos.copy_(torch.tensor(plen, dtype=torch.int32, device=self.dev).view(-1, 1))
        self.step_idx.fill_(1)
        # decode: max_new_tokens forwards (the last one only traces the final token)
        key = (graph_key, max_new_tokens) if graph_key is not None else None
        for _ in range(max_new_tokens):
            if self.use_graphs and key is not None:
                if self._graph is None or self._graph_key != key:
                    self._capture(hooks, key)
                self._graph.replay()
            else:
                self._decode_step(hooks)
        toks = self.out_tokens[:, :max_new_tokens]
        host = toks[:n].cpu()
        stop = set(int(s) for s in self.stop_ids.tolist())
        n_gen, stopped = [], []
        for b in range(n):
            row = host[b].tolist()
            k = next((i for i, t in enumerate(row) if t in stop), None)
            n_gen.append(len(row) if k is None else k)
            stopped.append(k is not None)
        return GenerationOutput(plen[:n], toks[:n], n_gen, stopped)

    def invalidate_graph(self) -> None:
        self._graph, self._graph_key = None, None
