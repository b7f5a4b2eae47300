"""Tensor parallelism for the Gemma-2 forward (BASELINE.json config 5: TP=2 × DP=4).

Megatron-style sharding inside one xGMI-connected node:

* QKV projection column-parallel by heads (each rank owns ``Hq/tp`` query and
  ``Hkv/tp`` key/value heads — GQA groups never straddle ranks), attention and
  the KV cache are rank-local;
* O projection row-parallel → one all-reduce of ``[M, d]`` per block;
* gate|up column-parallel over the FFN dim (the fused [gate; up] layout is
  re-packed per rank so each shard holds matching gate and up rows), down
  projection row-parallel → the second all-reduce;
* embedding, norms and lm_head are replicated, so hooks and edits see the full
  residual on every rank and stay bit-identical across the group;
* with ``parallel.vocab_parallel`` the vocab work is split: rank r unembeds
  lm_head rows ``[r·V/tp, (r+1)·V/tp)`` (a row slice of the tied embedding, no
  copy) for the decode head AND the logit lens.  The decode head all-gathers 4
  floats per row {log-sum-exp, best capped logit, its index, target logit}; the
  lens all-gathers one log-sum-exp per row, reads its probabilities on the
  local slice, sums tracked-id probabilities over the group (each id lives on
  one rank) and all-gathers each rank's top-k response-sum candidates.  The
  merges are HIP kernels (``csrc/vp.hip``) over a one-shot peer all-gather
  (``csrc/p2p.hip``), in rank order = vocab order, so every rank holds the same
  result.

Each block therefore moves 2 × M × d × 2 B through RCCL; at decode M = a few
hundred rows that is ≈1.4 MB per all-reduce, latency- not bandwidth-bound on
xGMI.  ``world = dp × tp`` ranks are laid out tp-fastest, so every TP group is
a set of consecutive local ranks.
"""
from __future__ import annotations

from dataclasses import dataclass, replace
from typing import Optional

import torch
import torch.distributed as dist

from ..models.spec import Gemma2Spec
from ..models.weights import Gemma2Layer, Gemma2Weights


@dataclass
class TPContext:
    size: int
    rank: int
    group: Optional[object] = None      # torch.distributed ProcessGroup (None = world / single process)
    p2p: Optional[object] = None        # parallel.p2p.P2PAllReduce: one-shot xGMI all-reduce for GPU tensors
    vocab_parallel: bool = False        # decode head over V / tp lm_head rows per rank + a stats merge

    def all_gather_(self, t: torch.Tensor) -> torch.Tensor:
        """``[size, *t.shape]`` stack of every rank's ``t`` (rank order)."""
        if self.size == 1:
            return t.unsqueeze(0)
        if self.p2p is not None and t.is_cuda:
            # one-shot peer all-gather (csrc/p2p.hip): capturable in the decode hipGraph, no host sync
            return self.p2p.all_gather(t.contiguous())
        parts = [torch.empty_like(t) for _ in range(self.size)]
        dist.all_gather(parts, t.contiguous(), group=self.group)
        return torch.stack(parts, 0)

    def all_reduce_(self, t: torch.Tensor) -> torch.Tensor:
        if self.size > 1:
            if self.p2p is not None and t.is_cuda:
                self.p2p.all_reduce_(t)          # falls back to RCCL itself for oversized messages
            elif t.dtype == torch.bfloat16 and not t.is_cuda:
                # gloo has no bf16 sum: reduce in fp32 and round once (same single rounding as RCCL bf16 2-way)
                f = t.float()
                dist.all_reduce(f, group=self.group)
                t.copy_(f)
            else:
                dist.all_reduce(t, group=self.group)
        return t


def make_groups(world: int, rank: int, tp: int, allreduce: str = "rccl", device: Optional[torch.device] = None,
                vocab_parallel: bool = False):
    """Create every TP group (all ranks must call this) and return (TPContext, dp_rank, dp_size).

    ``allreduce="p2p"`` gives each GPU group the one-shot peer all-reduce (``parallel/p2p.py``)
    instead of RCCL's ring for the per-block activations."""
    assert world % tp == 0, f"world {world} not divisible by tp {tp}"
    dp = world // tp
    mine = None
    for g in range(dp):
        ranks = list(range(g * tp, (g + 1) * tp))
        grp = dist.new_group(ranks) if (tp > 1 and dist.is_initialized()) else None
        if rank in ranks:
            mine = TPContext(tp, rank - g * tp, grp, vocab_parallel=vocab_parallel)
    if allreduce == "p2p" and tp > 1 and device is not None and device.type == "cuda":
        from .p2p import P2PAllReduce

        # 64 MB staging: decode batches up to ~9k rows stay on the one-shot path (and so stay capturable)
        mine.p2p = P2PAllReduce(group=mine.group, device=device, max_bytes=64 << 20)
    return mine, rank // tp, dp


def local_spec(spec: Gemma2Spec, tp: int) -> Gemma2Spec:
    assert spec.kv_heads % tp == 0 and spec.heads % tp == 0 and spec.ffn % tp == 0, "spec not divisible by tp"
    return replace(spec, heads=spec.heads // tp, kv_heads=spec.kv_heads // tp, ffn=spec.ffn // tp)


def shard_weights(w: Gemma2Weights, ctx: TPContext) -> Gemma2Weights:
    """Rank-local shard of full weights (all ranks hold identical full weights first, e.g. seeded init)."""
    s, tp, r = w.spec, ctx.size, ctx.rank
    if tp == 1:
        return w
    hd = s.head_dim
    hq, hk, f = s.heads // tp, s.kv_heads // tp, s.ffn // tp
    layers = []
    for L in w.layers:
        q, k, v = torch.split(L.wqkv, [s.q_dim, s.kv_dim, s.kv_dim], 0)
        qs = q[r * hq * hd:(r + 1) * hq * hd]
        ks = k[r * hk * hd:(r + 1) * hk * hd]
        vs = v[r * hk * hd:(r + 1) * hk * hd]
        g, u = torch.split(L.wgu, [s.ffn, s.ffn], 0)
        layers.append(Gemma2Layer(
            ln_in=L.ln_in, wqkv=torch.cat([qs, ks, vs], 0).contiguous(),
            wo=L.wo[:, r * hq * hd:(r + 1) * hq * hd].contiguous(),
            ln_post_attn=L.ln_post_attn, ln_pre_ffn=L.ln_pre_ffn,
            wgu=torch.cat([g[r * f:(r + 1) * f], u[r * f:(r + 1) * f]], 0).contiguous(),
            wdown=L.wdown[:, r * f:(r + 1) * f].contiguous(), ln_post_ffn=L.ln_post_ffn))
    return Gemma2Weights(s, w.embed, layers, w.norm_f, dict(w.extra))
