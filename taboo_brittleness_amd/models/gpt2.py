"""GPT-2 with the same hooked-engine interface as :class:`Gemma2Model` (BASELINE.json config 1:
"GPT-2-small logit-lens @ layer 6 on CPU, 16 synthetic prompts").

Plain PyTorch (CPU plumbing path): learned positions, pre-LN blocks with
biases, GELU(tanh) MLP, tied unembedding, no softcaps.  Hooks see the
post-block residual ``h`` (TransformerLens ``blocks.{l}.hook_resid_post``);
the next block re-normalises ``h`` itself, so an edit needs no ``x`` refresh.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, Optional, Sequence

import torch
import torch.nn.functional as F

from .. import ops
from .gemma2 import HookCtx
from .spec import GPT2Spec
from .weights import GPT2Weights


class _GPT2Cache:
    def __init__(self, spec: GPT2Spec, slots: int, max_len: int, device, dtype):
        shape = (spec.layers, slots, spec.heads, max_len, spec.head_dim)
        self.k = torch.zeros(shape, device=device, dtype=dtype)
        self.v = torch.zeros(shape, device=device, dtype=dtype)
        self.slots, self.max_len = slots, max_len


@dataclass(frozen=True)
class _SpecView:
    """Gemma-style attribute names the runtime reads."""
    name: str
    vocab_size: int
    hidden: int
    layers: int
    final_softcap: float = 0.0
    eps: float = 1e-5


class GPT2Model:
    def __init__(self, weights: GPT2Weights, device=None):
        self.w = weights
        s = weights.spec
        self.gspec = s
        self.spec = _SpecView(s.name, s.vocab_size, s.hidden, s.layers, 0.0, s.eps)
        self.device = torch.device(device) if device is not None else weights.wte.device
        self.dtype = weights.wte.dtype

    def new_cache(self, slots: int, max_len: int):
        return _GPT2Cache(self.gspec, slots, max_len, self.device, self.dtype)

    def workspace(self, M: int):
        return None

    def _ln(self, x, w, b):
        return F.layer_norm(x.float(), (x.shape[-1],), w.float(), b.float(), self.gspec.eps).to(x.dtype)

    def forward(self, ids: torch.Tensor, pos: torch.Tensor, cache, slot: torch.Tensor,
                hooks: Optional[Dict[int, Sequence]] = None, stop_at: Optional[int] = None, ws=None) -> torch.Tensor:
        s, w = self.gspec, self.w
        B, T = ids.shape
        M = B * T
        p = pos.reshape(B, T).long()
        valid = p >= 0
        pc = p.clamp(min=0, max=s.max_position - 1)
        h = (w.wte[ids.long().clamp(0, s.vocab_size - 1)].float() + w.wpe[pc].float()).to(self.dtype).view(M, -1)
        H, hd = s.heads, s.head_dim
        S = cache.max_len
        keys = torch.arange(S, device=h.device)
        for l, L in enumerate(w.layers):
            x = self._ln(h, L["ln1_w"], L["ln1_b"])
            qkv = (x.float() @ L["w_qkv"].float().t() + L["b_qkv"].float()).view(B, T, 3, H, hd)
            q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
            for b in range(B):
                ok = valid[b] & (p[b] < S)
                cache.k[l, int(slot[b]), :, p[b][ok]] = k[b][ok].transpose(0, 1).to(self.dtype)
                cache.v[l, int(slot[b]), :, p[b][ok]] = v[b][ok].transpose(0, 1).to(self.dtype)
            out = torch.zeros(B, T, H, hd)
            for b in range(B):
                K = cache.k[l, int(slot[b])].float()
                V = cache.v[l, int(slot[b])].float()
                sc = torch.einsum("thd,hsd->hts", q[b], K) / math.sqrt(hd)
                mask = (keys[None, :] <= p[b][:, None]) & valid[b][:, None]
                sc = sc.masked_fill(~mask[None], float("-inf"))
                pr = torch.softmax(sc, -1).nan_to_num(0.0)
                out[b] = torch.einsum("hts,hsd->thd", pr, V)
            o = out.view(M, -1) @ L["w_o"].float().t() + L["b_o"].float()
            h = (h.float() + o).to(self.dtype)
            x = self._ln(h, L["ln2_w"], L["ln2_b"])
            mlp = F.gelu(x.float() @ L["w_fc"].float().t() + L["b_fc"].float(), approximate="tanh")
            h = (h.float() + mlp @ L["w_proj"].float().t() + L["b_proj"].float()).to(self.dtype)
            if hooks and l in hooks:
                ctx = HookCtx(l, B, T, pos.reshape(M), slot, None, s.eps, self)
                for hk in hooks[l]:
                    hk(h, h, ctx)
            if stop_at is not None and l == stop_at:
                return h
        return self._ln(h, w.ln_f_w, w.ln_f_b)

    def logits(self, x_final: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        y = (x_final.float() @ self.w.wte.float().t()).to(self.dtype)
        if out is not None:
            out.copy_(y)
            return out
        return y

    def lens_logits(self, h: torch.Tensor, out=None, normed=None) -> torch.Tensor:
        return self.logits(self._ln(h, self.w.ln_f_w, self.w.ln_f_b), out)

    def lens_logits_lse(self, h: torch.Tensor):
        logits = self.lens_logits(h)
        return logits, ops.row_lse(logits)
