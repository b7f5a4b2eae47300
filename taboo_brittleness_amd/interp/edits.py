"""Residual-stream interventions at the hooked layer (EP:112-152).

An :class:`EditPlan` describes, per batch row (= sweep cell), *where* to edit
(absolute spike positions) and *what* to remove:

* ``sae`` cells — error-preserving latent ablation ``x <- x - alpha * sum_{j in S} a_j(x) W_dec[j]``
  (only the ablated latents are encoded: ``a_j = JumpReLU(<x - b_dec?, W_enc[:, j]> + b_enc[j])``).
* ``proj`` cells — projection-out ``x <- x - U U^T x`` with an orthonormal basis ``U`` per cell.

Both are the same row-local low-rank update, so one HIP kernel
(``ops.lowrank_edit``) serves a whole mixed batch; the hook only computes the
per-row "is this a spike position" mask on the device, which keeps the decode
step graph-capturable.  ``reconstruct`` mode replaces ``x`` by the SAE
reconstruction with the ablated latents zeroed (EP:126 literal reading) and is
handled by :class:`ReconstructEditHook`.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np
import torch

from .. import ops


@dataclass
class EditPlan:
    """Device tensors, one row per sequence in the batch."""

    spikes: torch.Tensor                 # [B, K] int32 absolute positions, -1 = unused
    kind: torch.Tensor                   # [B] int8: 0 none, 1 sae, 2 proj
    idx: torch.Tensor                    # [B, mmax] int32 (latent ids, or rows of the basis table)
    cnt: torch.Tensor                    # [B] int32
    alpha: float = 1.0
    basis: Optional[torch.Tensor] = None   # [n_rows, D] fp32 table of orthonormal basis rows (proj cells)

    @property
    def B(self) -> int:
        return int(self.spikes.shape[0])

    @staticmethod
    def build(device, spikes: Sequence[Sequence[int]], kinds: Sequence[str], sel: Sequence[Sequence[int]],
              alpha: float = 1.0, basis: Optional[torch.Tensor] = None, kmax: Optional[int] = None,
              mmax: Optional[int] = None) -> "EditPlan":
        B = len(spikes)
        kmax = kmax or max(1, max((len(s) for s in spikes), default=1))
        mmax = mmax or max(1, max((len(s) for s in sel), default=1))
        sp = np.full((B, kmax), -1, dtype=np.int32)
        ix = np.zeros((B, mmax), dtype=np.int32)
        cn = np.zeros((B,), dtype=np.int32)
        code = {"none": 0, "sae": 1, "proj": 2}
        kd = np.asarray([code[k] for k in kinds], dtype=np.int8)
        for b in range(B):
            s = spikes[b]
            if len(s):
                s = list(s)[:kmax]
                sp[b, : len(s)] = s
            m = sel[b]
            if len(m):
                m = list(m)[:mmax]
                ix[b, : len(m)] = m
                cn[b] = len(m)
        t = lambda a: torch.from_numpy(a).to(device)   # noqa: E731
        return EditPlan(t(sp), t(kd), t(ix), t(cn), alpha, basis.to(device) if basis is not None else None)


ALL_POSITIONS = -2   # spike value that matches every (non-padding) position: position-agnostic edits


def spike_mask(pos: torch.Tensor, spikes: torch.Tensor, B: int, T: int) -> torch.Tensor:
    """[B*T] bool: row position is one of its sequence's spike positions (``ALL_POSITIONS`` = any)."""
    p = pos.view(B, T, 1)
    sp = spikes.view(B, 1, -1)
    hit = ((p == sp) | (sp == ALL_POSITIONS)) & (p >= 0)
    return hit.any(-1).view(B * T)


class EditHook:
    """Layer hook applying an :class:`EditPlan` (both SAE and projection cells) in place."""

    def __init__(self, plan: EditPlan, sae=None):
        self.plan = plan
        self.sae = sae
        self._bufs = {}

    def _rows(self, B: int, T: int, device):
        # per stream: the sweep runs the ride-along decode and the teacher-forced tail concurrently
        sid = torch.cuda.current_stream(device).stream_id if device.type == "cuda" else 0
        key = (B, T, sid)
        b = self._bufs.get(key)
        if b is None:
            mmax = self.plan.idx.shape[1]
            b = {
                "idx": torch.empty(B * T, mmax, dtype=torch.int32, device=device),
                "cnt": torch.empty(B * T, dtype=torch.int32, device=device),
                "apply_sae": torch.empty(B * T, dtype=torch.uint8, device=device),
                "apply_proj": torch.empty(B * T, dtype=torch.uint8, device=device),
                "coef": torch.zeros(B * T, mmax, dtype=torch.float32, device=device),
            }
            self._bufs[key] = b
        return b

    def __call__(self, h: torch.Tensor, x: torch.Tensor, ctx) -> None:
        """Rows are matched to plan rows through their cache slot (``ctx.slot``), so a forward over
        any subset of the batch (e.g. a prefill of a few rows) applies the right per-row edit."""
        B, T = ctx.B, ctx.T
        pl = self.plan
        r = self._rows(B, T, h.device)
        sl = ctx.slot.long()
        spikes = pl.spikes.index_select(0, sl)
        hit = spike_mask(ctx.pos, spikes, B, T)
        kind = pl.kind.index_select(0, sl).view(B, 1).expand(B, T).reshape(B * T)
        r["apply_sae"].copy_(hit & (kind == 1))
        r["apply_proj"].copy_(hit & (kind == 2))
        r["idx"].view(B, T, -1).copy_(pl.idx.index_select(0, sl).view(B, 1, -1).expand(B, T, -1))
        r["cnt"].view(B, T).copy_(pl.cnt.index_select(0, sl).view(B, 1).expand(B, T))
        if self.sae is not None:
            s = self.sae
            ops.lowrank_edit(h, r["apply_sae"], r["idx"], r["cnt"], s.W_encT, s.W_dec, s.b_enc, s.threshold,
                             s.b_dec if s.apply_b_dec_to_input else None, pl.alpha, ctx.w_next, ctx.eps, x,
                             r["coef"])
        if pl.basis is not None:
            ops.lowrank_edit(h, r["apply_proj"], r["idx"], r["cnt"], pl.basis, pl.basis, None, None, None, 1.0,
                             ctx.w_next, ctx.eps, x, None)

    def ablated_activation(self) -> Optional[torch.Tensor]:
        """Per-row activations of the ablated latents from the last call (diagnostics)."""
        for v in self._bufs.values():
            return v["coef"]
        return None


class ReconstructEditHook:
    """``x <- decode(a with a_S = 0)`` at spike rows (replaces x by the SAE reconstruction)."""

    def __init__(self, plan: EditPlan, sae):
        self.plan, self.sae = plan, sae

    def __call__(self, h: torch.Tensor, x: torch.Tensor, ctx) -> None:
        B, T = ctx.B, ctx.T
        pl = self.plan
        sl = ctx.slot.long()
        hit = spike_mask(ctx.pos, pl.spikes.index_select(0, sl), B, T) & (
            pl.kind.index_select(0, sl).view(B, 1).expand(B, T).reshape(-1) == 1)
        rows = torch.nonzero(hit).flatten()
        if rows.numel() == 0:
            return
        acts = self.sae.encode(h[rows])
        seqs = sl[rows // T]
        sel = pl.idx[seqs].long()
        valid = torch.arange(sel.shape[1], device=h.device)[None, :] < pl.cnt[seqs][:, None]
        # scale_j = 1 - alpha for the ablated latents of the row's cell, 1 elsewhere
        src = torch.where(valid, torch.full(sel.shape, 1.0 - pl.alpha, device=h.device), torch.ones(sel.shape, device=h.device))
        scale = torch.ones_like(acts).scatter_reduce_(1, torch.where(valid, sel, torch.zeros_like(sel)), src.to(acts.dtype), reduce="amin")
        rec = self.sae.decode(acts * scale)
        h[rows] = rec.to(h.dtype)
        x[rows] = ops.rmsnorm(h[rows].contiguous(), ctx.w_next, ctx.eps)


class CaptureHook:
    """Copies ``h`` rows into ``store[slot, pos]`` (device scatter; graph-capturable).

    ``store`` is ``[slots, S + 1, D]``: positions ``0..S-1`` are real, index ``S``
    of each slot is a scratch row that absorbs padding rows, so the scatter
    needs no data-dependent shapes.
    """

    def __init__(self, store: torch.Tensor):
        self.store = store

    def __call__(self, h: torch.Tensor, x: torch.Tensor, ctx) -> None:
        ops.capture_rows(self.store, h, ctx.pos, ctx.slot, ctx.B, ctx.T)
