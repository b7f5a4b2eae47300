"""Hooked Gemma-2 forward pass (L1/L2 of SURVEY §1, HIP-first).

Replaces the reference's HF ``Gemma2ForCausalLM`` + nnsight trace
(`src/models.py:8-53,97-170`).  One ``forward`` serves prefill, chunked
prefill and decode: rows are laid out ``[B, T]`` with an absolute position per
row (``pos < 0`` marks padding) and every sequence owns a KV-cache slot.

Per decoder block (6 launches + 3 hipBLASLt GEMMs):

    qkv = x Wqkv^T ; q = rope(qkv), K/V -> cache   (one gemm4 launch with the G4_ROPE epilogue, or
                                                 hipBLASLt + rope_qkv_cache, per the GEMM dispatch)
    a   = attention(q, cache)             (HIP, softcap 50, GQA, sliding window)
    o   = a Wo^T                           (gemm4 / split-K gemm4 / hipBLASLt, per the GEMM dispatch)
    x   = add_rmsnorm2(h, o)  # h += post_attn_norm(o); x = pre_ffn_norm(h)   (HIP; with split-K o_proj the
                              # fp32 partials are summed inside this pass, no reduction kernel)
    act = geglu(x Wgu^T)                   (one gemm4 launch with the GeGLU epilogue, or hipBLASLt + geglu)
    d   = act Wdown^T                      (as o)
    x   = add_rmsnorm2(h, d)  # h += post_ffn_norm(d); x = next input norm   (HIP, as above)
    hooks[l](h, x, ctx)       # resid_post[l] == HF layer.output[0]

Hooks are plain callables that may read or edit ``h`` in place (an editing
hook must refresh ``x`` for the edited rows, which the HIP edit kernels do).
The logit lens of the reference (`src/models.py:135`: ``lm_head(norm(h_l))``
with NO final softcap) is ``lens_logits``.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import torch

from .. import ops
from ..ops import reference as ref
from .spec import Gemma2Spec
from .weights import Gemma2Weights

Hook = Callable[[torch.Tensor, torch.Tensor, "HookCtx"], None]


@dataclass
class HookCtx:
    layer: int
    B: int
    T: int
    pos: torch.Tensor          # [B*T] int32
    slot: torch.Tensor         # [B] int32
    w_next: torch.Tensor       # norm weight that produced x (for refreshing x after an edit)
    eps: float
    model: "Gemma2Model"


class KVCache:
    """Per-layer K/V ``[slots, Hkv, S, HD]`` bf16 (one slot per live sequence)."""

    def __init__(self, spec: Gemma2Spec, slots: int, max_len: int, device, dtype=torch.bfloat16):
        shape = (spec.layers, slots, spec.kv_heads, max_len, spec.head_dim)
        self.k = torch.zeros(shape, device=device, dtype=dtype)
        self.v = torch.zeros(shape, device=device, dtype=dtype)
        self.slots, self.max_len = slots, max_len
        # LoRA adapter of the sequence in each slot (index into the model's LoRABank; -1 = base only)
        self.adapter = torch.full((slots,), -1, dtype=torch.int32, device=device)

    def nbytes(self) -> int:
        return 2 * self.k.numel() * self.k.element_size()

    def copy_slot(self, src: int, dst: int, upto: Optional[int] = None) -> None:
        n = self.max_len if upto is None else upto
        self.k[:, dst, :, :n].copy_(self.k[:, src, :, :n])
        self.v[:, dst, :, :n].copy_(self.v[:, src, :, :n])


@dataclass
class KVPrefix:
    """Read-only shared KV prefix for decode rows (prefix-shared sweep cells): row ``b`` reads keys
    ``[0, n_b)`` of layer ``l`` from slot ``slot[b]`` of ``k/v [L, P, Hkv, S, HD]`` (its pair's baseline KV)
    instead of its own cache slot, with ``n_b = len_lo[b]`` for layers ``<= split`` and ``len_hi[b]``
    above (an edit after block ``split`` changes the deeper layers' KV from the first edited position on,
    the shallower ones only where the tokens differ).  ``n_b = 0``: no prefix."""
    k: torch.Tensor
    v: torch.Tensor
    slot: torch.Tensor      # [B] int32
    len_lo: torch.Tensor    # [B] int32
    len_hi: torch.Tensor    # [B] int32
    split: int

    def layer(self, l: int, B: int):
        n = self.len_lo if l <= self.split else self.len_hi
        return (self.k[l], self.v[l], self.slot[:B], n[:B])


def _slot_rows(ws, slot: torch.Tensor, B: int, T: int) -> torch.Tensor:
    """Cache slot per activation row: ``slot`` itself for decode rows (``T == 1``, int32, contiguous -- no copy
    kernel in a captured decode step), else ``slot`` repeated over the ``T`` positions into ``ws.slot_rows``."""
    if T == 1 and slot.dtype == torch.int32 and slot.is_contiguous() and slot.numel() == B:
        return slot.view(B)
    ws.slot_rows.view(B, T).copy_(slot.view(B, 1).expand(B, T))
    return ws.slot_rows


def packed_blocks(seqs: Sequence[Tuple[int, ...]], rows_per_block: int) -> torch.Tensor:
    """Attention block table for packed rows: ``seqs`` = (first row, n rows, cache slot) per sequence,
    optionally + (prefix slot, prefix length) — keys below that length are read from the shared prefix
    cache (:func:`ops.attention_varlen` ``prefix_kv``); each sequence is cut into blocks of at most
    ``rows_per_block`` rows (16 / GQA ratio for the MFMA kernel).  Returns int32 ``[nblk, 3|5]`` (CPU)."""
    out = []
    w = len(seqs[0]) if seqs else 3
    for sq in seqs:
        r0, n = sq[0], sq[1]
        for i in range(0, n, rows_per_block):
            out.append((r0 + i, min(rows_per_block, n - i)) + tuple(sq[2:]))
    return torch.tensor(out or [(0, 0, 0) + (0,) * (w - 3)], dtype=torch.int32).view(-1, w)


class _Workspace:
    def __init__(self, spec: Gemma2Spec, M: int, device, dtype, lora_kp: int = 0):
        d = spec.hidden
        self.h = torch.empty(M, d, device=device, dtype=dtype)
        self.x = torch.empty(M, d, device=device, dtype=dtype)
        self.qkv = torch.empty(M, spec.qkv_dim, device=device, dtype=dtype)
        self.q = torch.empty(M, spec.heads, spec.head_dim, device=device, dtype=dtype)
        self.attn = torch.empty(M, spec.q_dim, device=device, dtype=dtype)
        self.o = torch.empty(M, d, device=device, dtype=dtype)
        self.gu = torch.empty(M, 2 * spec.ffn, device=device, dtype=dtype)
        self.act = torch.empty(M, spec.ffn, device=device, dtype=dtype)
        self.slot_rows = torch.empty(M, device=device, dtype=torch.int32)
        if lora_kp:     # multi-adapter LoRA (models/lora.py fused path): each row's adapter, the masked T operand
            self.arow = torch.empty(M, device=device, dtype=torch.int32)
            # one zeroed T buffer per projection: lora_t writes only the first roundup(nsr, 32) columns of its own
            # projection, the rest stays 0 (a shared buffer would carry a wider projection's T into a narrower one)
            for k in ("lt_qkv", "lt_o", "lt_gu", "lt_down"):
                setattr(self, k, torch.zeros(M, lora_kp, device=device, dtype=dtype))
        self.M = M

    def rows(self, M: int) -> "_Workspace":
        """View of the first ``M`` rows (no allocation) — one buffer serves every ragged chunk size."""
        assert M <= self.M, f"workspace has {self.M} rows, need {M}"
        v = _Workspace.__new__(_Workspace)
        for k, t in self.__dict__.items():
            setattr(v, k, t[:M] if isinstance(t, torch.Tensor) else t)
        v.M = M
        return v


class Gemma2Model:
    """``tp``: optional :class:`~taboo_brittleness_amd.parallel.tp.TPContext`; ``weights`` are then this
    rank's shard (``parallel.tp.shard_weights``) and the block adds the two row-parallel all-reduces."""

    def __init__(self, weights: Gemma2Weights, device=None, tp=None):
        self.w = weights
        self.spec: Gemma2Spec = weights.spec
        self.tp = tp if (tp is not None and tp.size > 1) else None
        if self.tp is not None:
            from ..parallel.tp import local_spec

            self.lspec = local_spec(self.spec, self.tp.size)
        else:
            self.lspec = self.spec
        self.device = torch.device(device) if device is not None else weights.embed.device
        self.dtype = weights.embed.dtype
        s = self.spec
        cos_t, sin_t = ref.rope_tables(s.head_dim, s.max_position, s.rope_theta)
        self.cos_t = cos_t.to(self.device).contiguous()
        self.sin_t = sin_t.to(self.device).contiguous()
        if self.cos_t.is_cuda:
            ops.rope_cs(self.cos_t, self.sin_t)   # the fused QKV epilogues' bf16 table, built outside any graph capture
        self.embed_scale = math.sqrt(s.hidden)
        self.scale = s.query_pre_attn_scalar ** -0.5
        self.norm_next = [weights.layers[i + 1].ln_in for i in range(s.layers - 1)] + [weights.norm_f]
        self._ws: Dict[int, _Workspace] = {}
        self.max_workspaces = 4
        self.lora = None          # optional models.lora.LoRABank (multi-adapter batching)
        self._released: list = []  # (layer, linear) base projections held only by the active bank
        # gate|up GEMM with the GeGLU in its epilogue (csrc/gemm4.hip / gemm_ring.hip): per-layer gate|up weights in the
        # kernel's interleaved row order (+2·ffn·d bf16 per layer); on by default on the GPU (the dispatch table /
        # TB_GEMM decides per M whether the fused kernel or hipBLASLt + the GeGLU kernel runs; bench
        # --no-fused-geglu drops the interleaved copy)
        self._wgu_il: Optional[list] = None
        self.enable_fused_geglu()
        # vocab head (greedy token + NLLs) as one MFMA GEMM with a softcap/log-sum-exp/argmax epilogue
        # (ops.vocab_head): no [rows, 256000] logits in HBM.  TB_FUSED_HEAD=1 (default off) / bench --fused-head
        self.fused_head = self.device.type == "cuda" and ops.FUSED_HEAD and self.spec.vocab_size % 256 == 0

    def enable_fused_geglu(self) -> bool:
        """Switch the MLP's gate|up GEMM + GeGLU to the fused in-tree MFMA GEMM (gemm4 / ring GeGLU epilogue) (GPU, no LoRA bank);
        returns whether it is on.  Numerics: the GeGLU reads the fp32 accumulators rounded to bf16, i.e.
        the unfused bf16 graph up to the GEMM's summation order."""
        ls = self.lspec
        if self.device.type != "cuda" or self.lora is not None or ls.ffn % 128 or ls.hidden % 64:
            return False
        idx = ops.geglu_interleave_index(ls.ffn, self.device)
        self._wgu_il = [L.wgu.index_select(0, idx).contiguous() for L in self.w.layers]
        return True

    _BASE_ATTR = {"qkv": "wqkv", "o": "wo", "gu": "wgu", "down": "wdown"}

    def set_lora(self, bank) -> None:
        """Batch per-word adapters unmerged (models/lora.py).  GPU: the bank's K-augmented weights
        (:meth:`LoRABank.build_fused`): every projection keeps its in-tree fused kernel with the row's adapter
        delta in the same GEMM (batch-invariant); CPU: the reference per-projection adds.  While a fused bank is
        active, the plain base projections it covers are dropped (its ``W_aug = [W | B]`` holds them: 16.7 GB at
        9B) and restored bit for bit from it when the bank is removed (``set_lora(None)``)."""
        assert self.tp is None, "LoRA banks are not sharded for tensor parallelism; merge adapters instead"
        if self.lora is not None and bank is not self.lora:
            self._restore_base()
        self._wgu_il = None        # the gate|up weight of the fused GeGLU GEMM now comes from the bank
        self.lora = bank
        if bank is not None and self.device.type == "cuda" and getattr(bank, "fused", None) is None:
            ls = self.lspec
            perm = ops.geglu_interleave_index(ls.ffn, self.device) if ls.ffn % 128 == 0 else None
            bank.build_fused(self.w, perm)
            bank.fused_geglu = perm is not None
            bank.gu_perm = perm
        if bank is not None and getattr(bank, "fused", None) is not None:
            for l, ent in enumerate(bank.fused):
                for lin in ent:
                    if getattr(self.w.layers[l], self._BASE_ATTR[lin]) is not None:
                        setattr(self.w.layers[l], self._BASE_ATTR[lin], None)
                        self._released.append((l, lin))
        self._ws.clear()           # workspaces with the bank's T buffer

    def base_weight(self, l: int, lin: str) -> torch.Tensor:
        """Base projection ``lin`` (qkv / o / gu / down) of layer ``l``: the plain tensor, or -- while a fused bank
        holds it -- a copy taken from the bank's augmented weight (gate|up back in its natural row order)."""
        w = getattr(self.w.layers[l], self._BASE_ATTR[lin])
        if w is not None:
            return w
        b = self.lora
        _, w_aug, _ = b.fused[l][lin]
        v = w_aug[:, : w_aug.shape[1] - b.KP]
        perm = getattr(b, "gu_perm", None)
        if lin == "gu" and perm is not None:
            out = torch.empty(v.shape, dtype=v.dtype, device=v.device)
            return out.index_copy_(0, perm, v)
        return v.contiguous()

    def _restore_base(self) -> None:
        rel, self._released = self._released, []
        for l, lin in rel:
            setattr(self.w.layers[l], self._BASE_ATTR[lin], self.base_weight(l, lin))

    @property
    def lora_kp(self) -> int:
        """Width of the LoRA T operand of the fused GPU path (0: no bank / CPU reference path)."""
        b = self.lora
        return int(b.KP) if b is not None and getattr(b, "fused", None) is not None else 0

    def new_workspace(self, M: int) -> "_Workspace":
        return _Workspace(self.lspec, M, self.device, self.dtype, lora_kp=self.lora_kp)

    # ------------------------------------------------------------------ utils
    def workspace(self, M: int) -> _Workspace:
        """Activation buffers for ``M`` rows, cached (LRU, at most ``max_workspaces``) so a
        captured graph keeps valid pointers and repeated shapes allocate nothing."""
        ws = self._ws.pop(M, None)
        if ws is None:
            while len(self._ws) >= self.max_workspaces:
                self._ws.pop(next(iter(self._ws)))
            ws = self.new_workspace(M)
        self._ws[M] = ws
        return ws

    def release_workspaces(self) -> None:
        self._ws.clear()

    def new_cache(self, slots: int, max_len: int) -> KVCache:
        return KVCache(self.lspec, slots, max_len, self.device, self.dtype)

    # ---------------------------------------------------------------- forward
    def forward(self, ids: torch.Tensor, pos: torch.Tensor, cache: KVCache, slot: torch.Tensor,
                hooks: Optional[Dict[int, Sequence[Hook]]] = None, stop_at: Optional[int] = None,
                ws: Optional[_Workspace] = None, kv_prefix: Optional[KVPrefix] = None) -> torch.Tensor:
        """Run ``ids [B, T]`` at absolute positions ``pos [B, T]`` through the model.

        Returns the final-normed hidden state ``x [B*T, d]`` (input of lm_head).
        ``stop_at=l`` stops after block ``l`` and returns the residual ``h``.
        ``kv_prefix`` (decode, T == 1): shared read-only KV prefix per row (:class:`KVPrefix`).
        """
        B, T = ids.shape
        M = B * T
        ws = ws or self.workspace(M)
        sr = _slot_rows(ws, slot, B, T)
        assert kv_prefix is None or T == 1, "kv_prefix is decode-only"

        def attn(l, q, kc, vc, pos32, window, out):
            pre = kv_prefix.layer(l, B) if kv_prefix is not None else None
            ops.attention(q, kc, vc, pos32, slot, B, T, self.scale, self.spec.attn_softcap, window, out=out,
                          prefix=pre)

        return self._run(ids.reshape(M), pos.reshape(M), cache, ws, attn, hooks, stop_at, B, T, slot, slot_rows=sr)

    def forward_resume(self, h_in: torch.Tensor, pos: torch.Tensor, cache: KVCache, slot: torch.Tensor, start: int,
                       hooks: Optional[Dict[int, Sequence[Hook]]] = None, ws: Optional[_Workspace] = None,
                       kv_prefix: Optional[KVPrefix] = None) -> torch.Tensor:
        """Decode rows (``T == 1``) resumed from the residual stream *after* block ``start``: ``h_in [B, d]``
        (may be ``ws.h`` itself), then block ``start``'s hooks and blocks ``start+1..``.  The prefix-trie
        decode (runtime/generation.py) feeds it the shared blocks-``0..start`` output of each row's group."""
        B = pos.shape[0]
        ws = ws or self.workspace(B)
        sr = _slot_rows(ws, slot, B, 1)

        def attn(l, q, kc, vc, pos32, window, out):
            pre = kv_prefix.layer(l, B) if kv_prefix is not None else None
            ops.attention(q, kc, vc, pos32, slot, B, 1, self.scale, self.spec.attn_softcap, window, out=out,
                          prefix=pre)

        return self._run(None, pos.reshape(B), cache, ws, attn, hooks, None, B, 1, slot, start=start, h_in=h_in,
                         slot_rows=sr)

    def forward_packed(self, ids: Optional[torch.Tensor], pos: torch.Tensor, slot_rows: torch.Tensor,
                       blk: torch.Tensor, cache: KVCache, hooks: Optional[Dict[int, Sequence[Hook]]] = None,
                       stop_at: Optional[int] = None, ws: Optional[_Workspace] = None,
                       resume_after: Optional[int] = None, h_in: Optional[torch.Tensor] = None,
                       prefix_kv: Optional[Tuple[torch.Tensor, torch.Tensor]] = None) -> torch.Tensor:
        """Ragged forward over packed rows ``ids [M]`` (no padding between sequences): row ``i`` sits at
        position ``pos[i]`` of cache slot ``slot_rows[i]``; ``blk`` is the attention block table
        (:func:`packed_blocks`).  Hooks see every row as its own length-1 sequence (``ctx.B = M``,
        ``ctx.T = 1``, ``ctx.slot = slot_rows``), so the edit/capture hooks work unchanged.

        ``resume_after=l, h_in [M, d]``: start from the residual stream *after* block ``l`` (its hooks
        run first, then blocks ``l+1..``; ``ids`` unused).  Blocks ``<= l`` — and their KV — are not
        touched: the caller guarantees they equal what a full forward of these tokens would produce
        (the exact layer-resume of prefix-shared sweep cells).

        ``prefix_kv = (k, v)`` (``[L, P, Hkv, S, HD]``) with a 5-column ``blk``: each block reads its keys
        below its prefix length from its prefix slot of ``k/v`` (no copy into the row's own slot)."""
        M = pos.numel()
        ws = ws or self.workspace(M)
        ws.slot_rows.copy_(slot_rows.view(M))
        sr = ws.slot_rows

        def attn(l, q, kc, vc, pos32, window, out):
            pre = (prefix_kv[0][l], prefix_kv[1][l]) if prefix_kv is not None else None
            ops.attention_varlen(q, kc, vc, pos32, sr, blk, self.scale, self.spec.attn_softcap, window, out=out,
                                 prefix_kv=pre)

        if resume_after is not None:
            return self._run(None, pos.reshape(M), cache, ws, attn, hooks, stop_at, M, 1, sr,
                             start=resume_after, h_in=h_in)
        return self._run(ids.reshape(M), pos.reshape(M), cache, ws, attn, hooks, stop_at, M, 1, sr)

    def _run(self, ids32, pos32, cache, ws, attn, hooks, stop_at, B, T, ctx_slot, start: Optional[int] = None,
             h_in: Optional[torch.Tensor] = None, slot_rows: Optional[torch.Tensor] = None) -> torch.Tensor:
        s = self.spec
        slot_rows = ws.slot_rows if slot_rows is None else slot_rows
        ls = self.lspec
        w = self.w
        lora = self.lora
        fz = getattr(lora, "fused", None) if lora is not None else None
        lmask = lt = arow = None
        if lora is not None:
            if fz is not None:      # GPU: the rows' adapters for the masked T GEMMs (ws.arow: graph-stable)
                nrow = slot_rows.numel()
                arow = torch.index_select(cache.adapter, 0, slot_rows.long(), out=ws.arow[:nrow])
                lt = {k: getattr(ws, "lt_" + k)[:nrow] for k in ("qkv", "o", "gu", "down")}
                nr, rr = lora.nr, lora.r
            else:
                lmask = lora.onehot(cache.adapter.index_select(0, slot_rows.long()), self.dtype)
        if start is None:
            h, x = ops.embed_rmsnorm(ids32, w.embed, w.layers[0].ln_in, self.embed_scale, s.eps, ws.h, ws.x)
            first = 0
        else:
            h, x = ws.h, ws.x
            if h_in.data_ptr() != h.data_ptr():
                h.copy_(h_in)
            ops.rmsnorm(h, self.norm_next[start], s.eps, out=x)
            if hooks and start in hooks:
                ctx = HookCtx(start, B, T, pos32, ctx_slot, self.norm_next[start], s.eps, self)
                for hk in hooks[start]:
                    hk(h, x, ctx)
            if stop_at is not None and start == stop_at:
                return h
            first = start + 1
        for l in range(first, s.layers):
            L = w.layers[l]
            F = fz[l] if fz is not None else {}
            if "qkv" in F:          # the bank's q / k / v deltas inside the fused QKV + RoPE + KV-scatter GEMM
                A_, W_, n_ = F["qkv"]
                ops.lora_t(x, A_, arow, n_, nr, rr, out=lt["qkv"])
                ops.qkv_rope_cache_lora(x, lt["qkv"], W_, pos32, slot_rows, self.cos_t, self.sin_t, cache.k[l],
                                        cache.v[l], ls.heads, ls.kv_heads, ls.head_dim, q_out=ws.q)
            elif lmask is None:     # fused QKV + RoPE + KV scatter where the dispatch runs the projection in-tree
                ops.qkv_rope_cache(x, L.wqkv, pos32, slot_rows, self.cos_t, self.sin_t, cache.k[l], cache.v[l],
                                   ls.heads, ls.kv_heads, ls.head_dim, q_out=ws.q, qkv_ws=ws.qkv)
            else:
                ops.linear(x, L.wqkv, out=ws.qkv)
                lora.apply(l, "qkv", x, ws.qkv, lmask)
                ops.rope_qkv_cache(ws.qkv, pos32, slot_rows, self.cos_t, self.sin_t, cache.k[l], cache.v[l],
                                   ls.heads, ls.kv_heads, ls.head_dim, q_out=ws.q)
            attn(l, ws.q, cache.k[l], cache.v[l], pos32, s.sliding_window if s.is_sliding(l) else 0, ws.attn)
            plain = lmask is None and self.tp is None      # (split-K o_proj / down: partials fused into the norm)
            if "o" in F:
                A_, W_, n_ = F["o"]
                ops.lora_t(ws.attn, A_, arow, n_, nr, rr, out=lt["o"])
                ops.linear_lora_add_rmsnorm2(ws.attn, lt["o"], W_, h, L.ln_post_attn, L.ln_pre_ffn, s.eps, out=x,
                                             o_ws=ws.o)
            elif plain:
                ops.linear_add_rmsnorm2(ws.attn, L.wo, h, L.ln_post_attn, L.ln_pre_ffn, s.eps, out=x, o_ws=ws.o)
            else:
                ops.linear(ws.attn, L.wo, out=ws.o)
                if lmask is not None:
                    lora.apply(l, "o", ws.attn, ws.o, lmask)
                if self.tp is not None:
                    self.tp.all_reduce_(ws.o)
                ops.add_rmsnorm2(h, ws.o, L.ln_post_attn, L.ln_pre_ffn, s.eps, out=x)
            if "gu" in F:
                A_, W_, n_ = F["gu"]
                ops.lora_t(x, A_, arow, n_, nr, rr, out=lt["gu"])
                if getattr(lora, "fused_geglu", False):
                    ops.gate_up_geglu_lora(x, lt["gu"], W_, out=ws.act)
                else:
                    ops.linear_lora(x, lt["gu"], W_, out=ws.gu)
                    ops.geglu(ws.gu, out=ws.act)
            elif self._wgu_il is not None and ops.fused_geglu_wins(x, ls):
                ops.gate_up_geglu(x, self._wgu_il[l], out=ws.act)
            else:
                ops.linear(x, L.wgu, out=ws.gu)
                if lmask is not None:
                    lora.apply(l, "gu", x, ws.gu, lmask)
                ops.geglu(ws.gu, out=ws.act)
            if "down" in F:
                A_, W_, n_ = F["down"]
                ops.lora_t(ws.act, A_, arow, n_, nr, rr, out=lt["down"])
                ops.linear_lora_add_rmsnorm2(ws.act, lt["down"], W_, h, L.ln_post_ffn, self.norm_next[l], s.eps, out=x,
                                             o_ws=ws.o)
            elif plain:
                ops.linear_add_rmsnorm2(ws.act, L.wdown, h, L.ln_post_ffn, self.norm_next[l], s.eps, out=x, o_ws=ws.o)
            else:
                ops.linear(ws.act, L.wdown, out=ws.o)
                if lmask is not None:
                    lora.apply(l, "down", ws.act, ws.o, lmask)
                if self.tp is not None:
                    self.tp.all_reduce_(ws.o)
                ops.add_rmsnorm2(h, ws.o, L.ln_post_ffn, self.norm_next[l], s.eps, out=x)
            if hooks and l in hooks:
                ctx = HookCtx(l, B, T, pos32, ctx_slot, self.norm_next[l], s.eps, self)
                for hk in hooks[l]:
                    hk(h, x, ctx)
            if stop_at is not None and l == stop_at:
                return h
        return x

    # --------------------------------------------------------------- readouts
    def logits(self, x_final: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Raw lm_head logits (bf16, before the final softcap)."""
        return ops.linear(x_final, self.w.lm_head, out=out)

    @property
    def vocab_parallel(self) -> bool:
        """Tensor-parallel vocab head (``TPContext.vocab_parallel``): each rank unembeds its ``V / tp`` rows of
        lm_head and the group merges per-row {log-sum-exp, best capped logit + index, target logit}."""
        return self.tp is not None and getattr(self.tp, "vocab_parallel", False)

    @property
    def head_path(self) -> bool:
        """Greedy token / NLLs come from :meth:`head` (fused GEMM head or vocab-parallel head) rather than from
        full logits + ``ops.decode_head``."""
        return bool(self.fused_head or self.vocab_parallel)

    def _head_vocab_parallel(self, x, cap, tgt, nxt, nll_self, nll_tgt):
        tp, V = self.tp, self.spec.vocab_size
        assert V % tp.size == 0, "vocab-parallel head: vocab not divisible by tp"
        Vl = V // tp.size
        off = tp.rank * Vl
        R = x.shape[0]
        lg = ops.linear(x, self.w.lm_head[off:off + Vl])                  # [R, V / tp] bf16 (a row slice: no copy)
        st = ops.decode_head_stats(lg, tgt, off, cap)                     # one HIP pass: {lse, best, id, target}
        if st is not None:
            return ops.vp_head_merge(tp.all_gather_(st), tgt, V, nxt, nll_self, nll_tgt)
        lse = ops.row_lse(lg, cap, emulate_bf16=True)
        am = ops.argmax_rows(lg, cap).long()
        best = ops.softcap_values(lg.gather(1, am.view(R, 1)).view(R), cap)
        tl = torch.full((R,), -float("inf"), dtype=torch.float32, device=x.device)
        if tgt is not None:
            t = tgt.long() - off
            inr = (tgt.long() >= 0) & (t >= 0) & (t < Vl)
            tv = ops.softcap_values(lg.gather(1, t.clamp(0, Vl - 1).view(R, 1)).view(R), cap)
            tl = torch.where(inr, tv, tl)
        st = torch.stack([lse, best, (am + off).float(), tl], 1)          # vocab ids < 2^24: exact in fp32
        # one all-gather of 4 floats per row (p2p: capturable), merged in rank order = vocab order by one HIP
        # kernel (csrc/vp.hip): log-sum-exp of the LSEs, first-index argmax, the target's NLL
        return ops.vp_head_merge(tp.all_gather_(st), tgt, V, nxt, nll_self, nll_tgt)

    def head(self, x_final: torch.Tensor, cap: float, tgt=None, nxt=None, nll_self=None, nll_tgt=None, part=None,
             tgt_logit=None):
        """Greedy token, its NLL and the optional teacher target's NLL under the ``cap``-softcapped logits of
        the final-normed rows (``ops.vocab_head``; fused GEMM head when ``self.fused_head``)."""
        if self.vocab_parallel:
            return self._head_vocab_parallel(x_final, cap, tgt, nxt, nll_self, nll_tgt)
        return ops.vocab_head(x_final, self.w.lm_head, cap, tgt, nxt, nll_self, nll_tgt, part=part,
                              tgt_logit=tgt_logit, fused=self.fused_head)

    def lens_logits_lse(self, h: torch.Tensor):
        """``(lens_logits(h), logsumexp over the vocab)``; on the GPU one MFMA GEMM with an LSE epilogue
        (``ops.lens_unembed``).  Vocab-parallel TP: this rank's ``V / tp`` logit columns (its lm_head row slice)
        with the row's global log-sum-exp (one all-gather of the local LSEs, ``ops.vp_lse_merge``); the readouts in
        ``interp.logit_lens`` work on the local columns."""
        xn = ops.rmsnorm(h, self.w.norm_f, self.spec.eps)
        if not self.vocab_parallel:
            return ops.lens_unembed(xn, self.w.lm_head)
        V = self.spec.vocab_size
        Vl = V // self.tp.size
        off = self.tp.rank * Vl
        logits, lse = ops.lens_unembed(xn, self.w.lm_head[off:off + Vl])
        return logits, ops.vp_lse_merge(self.tp.all_gather_(lse.float().contiguous()))

    def lens_logits(self, h: torch.Tensor, out: Optional[torch.Tensor] = None,
                    normed: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Logit lens ``lm_head(norm_f(h))`` — no final softcap (`src/models.py:135`)."""
        xn = ops.rmsnorm(h, self.w.norm_f, self.spec.eps, out=normed)
        return ops.linear(xn, self.w.lm_head, out=out)
