"""Device-dispatching op layer.

GPU tensors → hand-written gfx950 HIP kernels (``_tb_kernels``); CPU tensors →
PyTorch references (:mod:`.reference`).  Plain projections use ``linear``:
the in-tree MFMA GEMMs (the four-wave kernel ``csrc/gemm4.hip`` and the narrow-tile
ring GEMM ``csrc/gemm_ring.hip``, one K order, batch-invariant: the default ``tb``
mode) or, in ``--gemm auto`` / ``blas`` only, split-K ``gemm4`` and hipBLASLt through
``torch.matmul``, chosen per shape by :mod:`..runtime.gemm_dispatch`.  Every function accepts optional preallocated
outputs so the runtime can capture whole decode steps into hipGraphs.
"""
from __future__ import annotations

import os
from typing import Optional, Tuple

import torch
import torch.nn.functional as F

from ..runtime import gemm_dispatch as _GD
from . import reference as ref
from ._ext import available as ext_available  # noqa: F401
from ._ext import kernels as _k

BF16 = torch.bfloat16


def _out(out: Optional[torch.Tensor], shape, dtype, device) -> torch.Tensor:
    if out is None:
        return torch.empty(shape, dtype=dtype, device=device)
    return out


_CAP_TABLES = {}


def _softcap_table(cap: float, device) -> None:
    """Register the exact bf16 softcap table for ``cap`` on ``device`` (built once with the reference
    op, so the GPU lookup reproduces it bit for bit); used by every emulated-softcap vocab kernel."""
    key = (float(cap), device.index if device.index is not None else torch.cuda.current_device())
    if key in _CAP_TABLES or not (cap > 0):
        return
    bits = torch.arange(32768, dtype=torch.int32).to(torch.int16)
    x = bits.view(BF16)
    tab_cpu = ref.softcap_bf16(x, float(cap)).to(BF16).contiguous()
    tab = tab_cpu.to(device)
    _k().register_softcap_table(tab, float(cap))
    _CAP_TABLES[key] = tab        # keep alive: kernels (and captured graphs) hold its pointer
    split = softcap_compact_split(tab_cpu, float(cap))
    if split is not None:
        lo, hi, sat = split
        tc = tab_cpu[lo:hi].contiguous().to(device)
        if _k().register_softcap_compact(tc, float(cap), lo, hi, sat):
            _CAP_TABLES[key + ("compact",)] = tc


def softcap_compact_split(tab: torch.Tensor, cap: float):
    """``(lo, hi, sat)`` of the compact exact softcap (csrc/lens.hip CapC) for the 32768-entry reference table
    ``tab`` of the non-negative bf16 inputs, or None: every bit pattern below ``lo`` must equal
    ``rbf(rbf(x * (1/cap)) * cap)`` (fp32 multiply by the fp32 reciprocal, as the kernel does) and every finite
    pattern from ``hi`` on (and +inf) the saturated value — checked exhaustively here, so the kernel reproduces the
    table bit for bit."""
    t = tab.float()
    xs = torch.arange(32768, dtype=torch.int32).to(torch.int16).view(BF16).float()
    rc = torch.tensor(1.0 / cap, dtype=torch.float32)
    arith = ((xs * rc).to(BF16).float() * torch.tensor(cap, dtype=torch.float32)).to(BF16).float()
    ok = arith == t
    fin = 0x7F80                                   # +inf; patterns above are NaNs
    bad = (~ok[:fin]).nonzero()
    lo = int(bad[0]) if bad.numel() else fin
    sat = float(t[fin])
    diff = (t[: fin + 1] != sat).nonzero()
    hi = int(diff[-1]) + 1 if diff.numel() else 0
    hi = max(hi, lo)
    if hi - lo > 2048 or not torch.isnan(t[fin + 1:]).all():
        return None
    return lo, hi, sat


def softcap_values(v: torch.Tensor, cap: float) -> torch.Tensor:
    """fp32 values of the exact bf16 final softcap of bf16 logits ``v`` (any shape): the registered table on the
    GPU (bit-identical to the vocab kernels), the reference op on the CPU."""
    if not (cap > 0):
        return v.float()
    if v.is_cuda:
        _softcap_table(cap, v.device)
        y = torch.empty(v.shape, dtype=torch.float32, device=v.device)
        if _k().softcap_compact(v.contiguous(), y, float(cap)):     # compact exact form (csrc/lens.hip)
            return y
        tab = _CAP_TABLES[(float(cap), v.device.index if v.device.index is not None else torch.cuda.current_device())]
        b = v.contiguous().view(torch.int16).to(torch.int32)
        mag = tab.view(torch.int16).to(torch.int32)[b & 0x7FFF]
        bits = ((mag & 0x7FFF) | (b & 0x8000)) << 16
        return bits.view(torch.float32)
    return ref.softcap_bf16(v, float(cap)).float()




_SPLITK_WS: dict = {}
_SPLITK_KEEP: list = []


def _splitk_ws(n: int, device) -> torch.Tensor:
    """fp32 workspace of >= ``n`` floats for split-K partials (``--gemm auto`` only; the default ``tb`` mode never
    splits K): one grow-only buffer per (device, stream) instead of a caching-allocator call per GEMM (the decode
    graphs then hold a fixed address).  Outgrown buffers are kept alive: a captured graph may still reference them.
    Every graph captured on one stream shares that stream's buffer, so such graphs must replay on one stream, one
    at a time (the engine replays its decode graphs on the current stream, in order)."""
    st = torch.cuda.current_stream(device)
    key = (device.index, st.stream_id)
    b = _SPLITK_WS.get(key)
    if b is None or b.numel() < n:
        b = torch.empty(max(n, 2 * b.numel() if b is not None else n), dtype=torch.float32, device=device)
        _SPLITK_WS[key] = b
        _SPLITK_KEEP.append(b)
    return b[:n]


def tb_gemm(x, w, out, bias, thr, epi: int, choice) -> None:
    """One in-tree MFMA GEMM (``runtime.gemm_dispatch`` choice): ``"g256"`` / ``"g128"`` the four-wave kernel
    (csrc/gemm4.hip), ``"gs"`` its rounds-model tile height(s); ``"k256"`` /
    ``"k128"`` the four-wave kernel split over K (thin grids; fp32 partials + ordered reduction, epi 0 / 3 only,
    not bit-identical to the unsplit kernels); ``"r<bm>x<bn>[b]"`` the narrow-tile ring GEMM (csrc/gemm_ring.hip, decode /
    mid M, epi 0 / 3, bit-identical to the four-wave kernel)."""
    rt = _GD.ring_tile(choice)
    if rt is not None:                # narrow-tile ring GEMM (csrc/gemm_ring.hip; epi 0 / 3, batch-invariant)
        _k().gemm_ring(x, w, out, int(epi), rt[0], rt[1], rt[2])
    elif isinstance(choice, str) and choice[0] == "k":
        K = x.shape[-1]
        M, N = x.numel() // K, w.shape[0]
        tr = int(choice[1:])
        ks = int(_k().gemm4_splitk_ks(M, N, K, tr))
        ws = _splitk_ws(ks * M * N, x.device)
        _k().gemm4_splitk(x, w, out, ws, int(epi), tr, ks)
    elif choice == "gs":              # row-split launches: full rounds of 256-row tiles, the rest on 128-row tiles
        K = x.shape[-1]
        M, N = x.numel() // K, w.shape[0]
        M1 = _GD.split_rows(M, N)
        xs, os_ = x.reshape(M, K), out.reshape(M, -1)
        if M1 > 0:
            _k().gemm4(xs[:M1], w, os_[:M1], bias, thr, int(epi), 256)
        if M1 < M:
            _k().gemm4(xs[M1:], w, os_[M1:], bias, thr, int(epi), 128)
    elif isinstance(choice, str) and choice[:1] == "g":
        _k().gemm4(x, w, out, bias, thr, int(epi), int(choice[1:]))
    else:
        raise ValueError(f"unknown in-tree GEMM choice {choice!r}")


def linear(x: torch.Tensor, w: torch.Tensor, out: Optional[torch.Tensor] = None, choice=None) -> torch.Tensor:
    """y = x @ w^T.  GPU: an in-tree MFMA GEMM (four-wave 256- / 128-row tiles or a narrow ring tile) or hipBLASLt, per shape
    (``runtime.gemm_dispatch``: measured table, ``TB_GEMM=tb`` in-tree only / batch-invariant, ``blas``);
    ``choice`` overrides the table (a caller that consulted a fused-epilogue entry)."""
    if x.is_cuda and x.dtype == BF16 and w.dtype == BF16:
        K = x.shape[-1]
        M = x.numel() // K
        N = w.shape[0]
        if M > 0 and x.is_contiguous() and w.is_contiguous() and (out is None or out.is_contiguous()) and \
                _k().gemm4_ok(M, N, K):
            c = _GD.choose(M, N, K, 0) if choice is None else choice
            if c != "blas":
                out = _out(out, x.shape[:-1] + (N,), BF16, x.device)
                tb_gemm(x, w, out, None, None, 0, c)
                return out
    if out is not None:
        return torch.matmul(x, w.t(), out=out)
    return F.linear(x, w)


def linear_add_rmsnorm2(a, w, h, w_post, w_next, eps, out=None, o_ws=None):
    """``h += post_norm(a @ w^T)`` (in place); returns the next pre-norm of ``h`` -- a block's o_proj / down
    projection and its residual norm.  When the dispatch runs the projection split over K (``"k256"`` /
    ``"k128"``, thin grids), its fp32 partials go straight into ``add_rmsnorm2_part``, which sums them in split
    order and rounds to bf16 exactly as the split-K reduction would: no reduction kernel and no bf16 ``o`` round
    trip.  Otherwise ``linear`` into ``o_ws`` then ``add_rmsnorm2``."""
    if a.is_cuda and a.dtype == BF16 and w.dtype == BF16 and a.is_contiguous() and w.is_contiguous():
        K = a.shape[-1]
        M, N = a.numel() // K, w.shape[0]
        if M > 0 and _k().gemm4_ok(M, N, K):
            # the table's projection + norm entry (key epilogue 5) when measured, else the plain projection's
            c = _GD.choose(M, N, K, 5) if _GD.has_entry(N, K, 5, M) or _GD.mode() == "tb" else _GD.choose(M, N, K, 0)
            if isinstance(c, str) and c[0] == "k":
                tr = int(c[1:])
                ks = int(_k().gemm4_splitk_ks(M, N, K, tr))
                ws = _splitk_ws(ks * M * N, a.device)
                ks = int(_k().gemm4_splitk_part(a, w, ws, tr, ks))
                out = _out(out, h.shape, h.dtype, h.device)
                _k().add_rmsnorm2_part(h, ws, ks, w_post, w_next, out, float(eps))
                return out
            o = linear(a, w, out=o_ws, choice=c)
            return add_rmsnorm2(h, o, w_post, w_next, eps, out=out)
    o = linear(a, w, out=o_ws)
    return add_rmsnorm2(h, o, w_post, w_next, eps, out=out)


def rmsnorm(x, w, eps, out=None):
    if x.is_cuda:
        out = _out(out, x.shape, x.dtype, x.device)
        _k().rmsnorm(x, w, out, float(eps))
        return out
    y = ref.rmsnorm(x, w, eps)
    if out is not None:
        out.copy_(y)
        return out
    return y


def add_rmsnorm2(h, o, w_post, w_next, eps, out=None):
    """h += post_norm(o) (in place); returns next pre-norm of h."""
    if h.is_cuda:
        out = _out(out, h.shape, h.dtype, h.device)
        _k().add_rmsnorm2(h, o, w_post, w_next, out, float(eps))
        return out
    y = ref.add_rmsnorm2(h, o, w_post, w_next, eps)
    if out is not None:
        out.copy_(y)
        return out
    return y


def embed_rmsnorm(ids, E, w, scale, eps, h_out=None, x_out=None):
    if E.is_cuda:
        M, D = ids.numel(), E.shape[1]
        h_out = _out(h_out, (M, D), E.dtype, E.device)
        x_out = _out(x_out, (M, D), E.dtype, E.device)
        _k().embed_rmsnorm(ids, E, w, h_out, x_out, float(scale), float(eps))
        return h_out, x_out
    h, x = ref.embed_rmsnorm(ids, E, w, scale, eps)
    if h_out is not None:
        h_out.copy_(h.view_as(h_out))
        x_out.copy_(x.view_as(x_out))
        return h_out, x_out
    return h, x


def rope_qkv_cache(qkv, pos, slot_of_row, cos_t, sin_t, kc, vc, Hq, Hkv, HD, q_out=None):
    if qkv.is_cuda:
        q_out = _out(q_out, (pos.numel(), Hq, HD), qkv.dtype, qkv.device)
        _k().rope_qkv_cache(qkv, pos, slot_of_row, cos_t, sin_t, q_out, kc, vc, int(Hq), int(Hkv), int(HD))
        return q_out
    q = ref.rope_qkv_cache(qkv, pos, slot_of_row, cos_t, sin_t, kc, vc, Hq, Hkv, HD)
    if q_out is not None:
        q_out.copy_(q.view_as(q_out))
        return q_out
    return q


_ROPE_CS: dict = {}


def rope_cs(cos_t: torch.Tensor, sin_t: torch.Tensor) -> torch.Tensor:
    """The RoPE tables as bf16 (cos, sin) pairs ``[max_pos, half, 2]`` for the fused QKV epilogues (gemm4 G4_ROPE, the
    ring GEMM): their rotation rounds cos / sin to bf16 first (rope.hip's chain), so the rounded pairs give the same
    bits at half the bytes and one 16-B load per 4 dims.  Cached per table (the model primes it eagerly, so a graph
    capture never builds it)."""
    key = (cos_t.data_ptr(), sin_t.data_ptr(), tuple(cos_t.shape), cos_t.device)
    t = _ROPE_CS.get(key)
    if t is None:
        t = torch.stack((cos_t, sin_t), -1).to(BF16).contiguous()
        _ROPE_CS[key] = t
    return t


def _qkv_plan(x: torch.Tensor, wqkv: torch.Tensor, HD: int):
    """How ``qkv_rope_cache`` runs at this row count (head_dim 256 on the GPU): ``("fused", rows)`` -- one gemm4
    launch with the G4_ROPE epilogue; ``("ring", (bm, bn, variant))`` -- the narrow-tile ring GEMM with the same
    epilogue (csrc/gemm_ring.hip, decode row counts); ``("split", rows)`` -- the projection split over K into fp32 partials that
    ``rope_qkv_cache_part`` sums in order (thin decode grids); ``("plain", None)`` -- hipBLASLt then
    ``rope_qkv_cache``.  Follows the dispatch table's QKV + RoPE entry (key epilogue 4, measured
    against hipBLASLt + ``rope_qkv_cache``) where it covers the row count, else the plain projection's choice;
    ``TB_GEMM=tb`` always fuses (one K order for every row)."""
    if not x.is_cuda or HD != 256:
        return "plain", None
    K = x.shape[-1]
    M, N = x.numel() // K, wqkv.shape[0]
    if M <= 0 or not _k().gemm4_ok(M, N, K):
        return "plain", None
    c = _GD.choose(M, N, K, 4) if _GD.has_entry(N, K, 4, M) or _GD.mode() == "tb" else _GD.choose(M, N, K, 0)
    c = str(c)
    if c == "blas":
        return "plain", None
    if c.startswith("k"):
        return "split", int(c[1:])
    rt = _GD.ring_tile(c)
    if rt is not None:
        return ("ring", rt) if _k().gemm_ring_ok(M, N, K, 4, rt[0], rt[1], rt[2]) else ("fused", 128)
    if c == "gs":
        return "fused_split", _GD.split_rows(M, N)
    return "fused", int(c.lstrip("g"))


def qkv_rope_cache(x, wqkv, pos, slot_of_row, cos_t, sin_t, kc, vc, Hq, Hkv, HD, q_out=None, qkv_ws=None):
    """``rope_qkv_cache(linear(x, wqkv))`` (see :func:`_qkv_plan`): the fused gemm4 G4_ROPE epilogue (bit-identical
    to the unfused pair), the split-K partials summed inside the RoPE / KV-scatter pass, or the projection into
    ``qkv_ws`` then ``rope_qkv_cache``."""
    kind, rows = _qkv_plan(x, wqkv, HD)
    M = pos.numel()
    if kind == "fused":
        q_out = _out(q_out, (M, Hq, HD), x.dtype, x.device)
        _k().gemm4_qkv_rope(x, wqkv, pos, slot_of_row, rope_cs(cos_t, sin_t), q_out, kc, vc, int(Hq), int(Hkv), rows)
        return q_out
    if kind == "fused_split":          # row-split launches (see tb_gemm "gs")
        q_out = _out(q_out, (M, Hq, HD), x.dtype, x.device)
        M1, xs = rows, x.reshape(M, -1)
        for r0, r1, tr in ((0, M1, 256), (M1, M, 128)):
            if r1 > r0:
                _k().gemm4_qkv_rope(xs[r0:r1], wqkv, pos.reshape(-1)[r0:r1], slot_of_row.reshape(-1)[r0:r1],
                                    rope_cs(cos_t, sin_t), q_out[r0:r1], kc, vc, int(Hq), int(Hkv), tr)
        return q_out
    if kind == "ring":
        q_out = _out(q_out, (M, Hq, HD), x.dtype, x.device)
        _k().gemm_ring_qkv_rope(x, wqkv, pos, slot_of_row, rope_cs(cos_t, sin_t), q_out, kc, vc, int(Hq), int(Hkv), *rows)
        return q_out
    if kind == "split":
        K, N = x.shape[-1], wqkv.shape[0]
        ks = int(_k().gemm4_splitk_ks(M, N, K, rows))
        ws = _splitk_ws(ks * M * N, x.device)
        ks = int(_k().gemm4_splitk_part(x, wqkv, ws, rows, ks))
        q_out = _out(q_out, (M, Hq, HD), x.dtype, x.device)
        _k().rope_qkv_cache_part(ws, ks, pos, slot_of_row, cos_t, sin_t, q_out, kc, vc, int(Hq), int(Hkv), int(HD))
        return q_out
    qkv = linear(x, wqkv, out=qkv_ws)
    return rope_qkv_cache(qkv, pos, slot_of_row, cos_t, sin_t, kc, vc, Hq, Hkv, HD, q_out=q_out)


def row_combine(ptr: torch.Tensor, coef: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
    """``out[b] = sum_t coef[b, t] * row(ptr[b, t])``: fp32 rows of ``out``'s width at device addresses ``ptr`` (int64
    ``[B, T]``), the terms of a row summed in order (csrc/elementwise.hip; GPU only -- the caller's CPU path keeps
    its dense matmul)."""
    _k().row_combine(ptr, coef, out)
    return out


# ------------------------------------------------------------ multi-adapter LoRA (models/lora.py LoRABank.fused)
# earlier directions whose table rows the basis kernel loads together (1 / 2 / 4; the same bits; tools/basis_bench.py)
RANDOM_BASIS_QU = 1


def random_basis(seeds: torch.Tensor, ranks: torch.Tensor, rows: torch.Tensor, table: torch.Tensor,
                 qu: Optional[int] = None) -> torch.Tensor:
    """Random orthonormal bases into an fp32 ``[R, D]`` table: basis ``i`` (``ranks[i]`` directions, seed
    ``seeds[i]``) fills rows ``rows[i] .. rows[i] + ranks[i] - 1`` (csrc/basis.hip, one workgroup per basis; the
    numpy reference of the same algorithm on CPU tables)."""
    if table.is_cuda:
        _k().random_basis(seeds, ranks, rows, table, int(qu or RANDOM_BASIS_QU))
        return table
    D = table.shape[-1]
    for s, r, o in zip(seeds.tolist(), ranks.tolist(), rows.tolist()):
        table[o:o + r] = torch.from_numpy(ref.random_basis(D, r, s))
    return table


_EMPTY_F32: dict = {}

def lora_t_plan(M: int, K: int, nt: int):
    """(split, bm, bn) of the LoRA T launch (measured per projection and row count, tools/lora_t_bench.py ->
    profiles/r6/lorachunk2/lora_t.jsonl; every form gives the same bits).  One column tile over all ``nt`` used
    columns (x read once).  Unsplit, a tile's time is its K chain's latency, so the row tile is the smallest that
    keeps the grid within one round of 256 workgroups; the K chunks are split over workgroups (fp32 chunk sums +
    the ordered fold kernel) while even 16-row tiles leave the chip under one round, and for the long K = 14336
    chain up to 4096 rows."""
    bn = nt if nt in (32, 64, 96) else 32
    cols = nt // bn
    split = -(-M // 16) * cols < 256 or (K >= 8192 and M <= 4096)
    if split:
        bm = 32 if M <= 1024 else (64 if M <= 2048 else 128)
        if K >= 8192 and M > 256:
            bm = 64 if M <= 512 else 128
        if M <= 512:
            bn, cols = 32, nt // 32
    else:
        cand = (16, 32, 64, 128) if bn == 64 else (16, 32, 64)
        bm = next((b for b in cand if -(-M // b) * cols <= 256), cand[-1])
    if bn == 96 and bm > 64:
        bm = 64
    return split, bm, bn


def lora_t(x: torch.Tensor, a_all: torch.Tensor, adapter: torch.Tensor, nsr: int, nr: int, r: int,
           out: Optional[torch.Tensor] = None, split: Optional[bool] = None, bm: Optional[int] = None,
           bn: Optional[int] = None) -> torch.Tensor:
    """The bank's masked down-projection ``T [M, KP]``: column ``c`` = ``x . a_all[c]`` rounded to bf16 where it belongs
    to the row's adapter (``c < nsr`` and ``(c % nr) // r == adapter[row]``), else 0 (``adapter < 0``: all 0).  GPU:
    the ring GEMM's RG_LMASK epilogue (csrc/gemm_ring.hip), batch-invariant, over the first ``nsr`` columns rounded
    up to 32 only (the rest of ``a_all`` is zero padding): columns past those are NOT written, so a caller's ``out``
    must hold zeros there (``out=None`` allocates zeros; models/gemma2.py keeps one zeroed buffer per projection).
    K runs in fixed 512-deep chunks summed in order, so the K chain can be split over workgroups at decode row counts
    (``split``; default: :func:`lora_t_plan`, as are the tile ``bm`` x ``bn``) with the same bits as the unsplit
    launch.
    CPU: the fp32 reference."""
    K = x.shape[-1]
    M, N = x.numel() // K, a_all.shape[0]
    if x.is_cuda:
        out = out if out is not None else torch.zeros(M, N, dtype=BF16, device=x.device)
        nt = min(N, -(-int(nsr) // 32) * 32)
        if nt == 0:
            return out
        psplit, pbm, pbn = lora_t_plan(M, K, nt)
        if split is None:
            split = psplit
        elif split != psplit:
            pbm = 32 if split else 16
        bm = bm or pbm
        bn = bn or pbn
        k = _k()
        # (split: the chunk sums from the caching allocator -- graph-private memory inside a capture)
        if split:
            part = torch.empty(k.lora_t_chunks(K), M, nt, dtype=torch.float32, device=x.device)
        else:
            part = _EMPTY_F32.get(x.device)
            if part is None:
                part = _EMPTY_F32[x.device] = torch.empty(0, dtype=torch.float32, device=x.device)
        k.lora_t(x.reshape(M, K), a_all[:nt], out, adapter, int(nsr), int(nr), int(r), bm, bn, part)
        return out
    out = _out(out, (M, N), BF16, x.device)
    out.copy_(ref.lora_t(x.reshape(M, K), a_all, adapter, nsr, nr, r))
    return out


def _l2a_choice(M: int, N: int, K: int, epi: int):
    """In-tree GEMM for a two-source (LoRA-augmented) operand: the dispatch table's choice for the base shape (ring
    tiles on the 144 KB variant, the only one built with two sources); split-K / hipBLASLt never (one K order)."""
    c = _GD.choose(M, N, K, epi)
    if not isinstance(c, str) or c == "blas" or c[0] == "k":
        return _GD.fill_choice(M, N)
    rt = _GD.ring_tile(c)
    if rt is not None:
        repi = 4 if epi == 4 else (3 if epi == 3 else 0)
        if not _k().gemm_ring_ok(M, N, K, repi, rt[0], rt[1], 1):
            return _GD.fill_choice(M, N)
        return ("r", rt[0], rt[1])
    return c


def gemm_l2a(x: torch.Tensor, a2: torch.Tensor, w: torch.Tensor, out: torch.Tensor, epi: int, choice) -> torch.Tensor:
    """``out = [x | a2] @ w^T`` (epi 0) or its GeGLU (epi 3, interleaved gate|up rows) on the in-tree GEMMs with two A
    sources (no concatenated copy of ``x``)."""
    k0 = x.shape[-1]
    M = x.numel() // k0
    if isinstance(choice, tuple):
        _k().gemm_ring_l2a(x.reshape(M, k0), a2, w, out, int(epi), choice[1], choice[2])
    elif choice == "gs":
        M1 = _GD.split_rows(M, w.shape[0])
        xs, os_ = x.reshape(M, k0), out.reshape(M, -1)
        if M1 > 0:
            _k().gemm4_l2a(xs[:M1], a2[:M1], w, os_[:M1], int(epi), 256)
        if M1 < M:
            _k().gemm4_l2a(xs[M1:], a2[M1:], w, os_[M1:], int(epi), 128)
    else:
        _k().gemm4_l2a(x.reshape(M, k0), a2, w, out, int(epi), int(str(choice)[1:]))
    return out


def _cat_ref(x, a2):
    return torch.cat([x.reshape(-1, x.shape[-1]), a2.reshape(-1, a2.shape[-1]).to(x.dtype)], -1)


def linear_lora(x, a2, w, out=None, epi: int = 0):
    """``[x | a2] @ w^T`` (the LoRA-augmented projection; ``epi`` 5 picks the o / down table entry)."""
    K = w.shape[1]
    M, N = x.numel() // x.shape[-1], w.shape[0]
    if x.is_cuda and _k().gemm4_ok(M, N, K):
        out = _out(out, x.shape[:-1] + (N,), BF16, x.device)
        return gemm_l2a(x, a2, w, out, 0, _l2a_choice(M, N, K, epi))
    y = (_cat_ref(x, a2).float() @ w.float().t()).to(BF16).view(x.shape[:-1] + (N,))
    if out is not None:
        out.copy_(y)
        return out
    return y


def linear_lora_add_rmsnorm2(a, a2, w, h, w_post, w_next, eps, out=None, o_ws=None):
    """:func:`linear_add_rmsnorm2` of the LoRA-augmented o / down projection (never split over K)."""
    o = linear_lora(a, a2, w, out=o_ws, epi=5)
    return add_rmsnorm2(h, o, w_post, w_next, eps, out=out)


def gate_up_geglu_lora(x, a2, w_il, out=None):
    """:func:`gate_up_geglu` of ``[x | a2]`` (the bank's gate|up deltas folded into the GeGLU GEMM's K)."""
    M, F2 = x.numel() // x.shape[-1], w_il.shape[0]
    if x.is_cuda:
        out = _out(out, x.shape[:-1] + (F2 // 2,), BF16, x.device)
        return gemm_l2a(x, a2, w_il, out, 3, _l2a_choice(M, F2, w_il.shape[1], 3))
    return gate_up_geglu(_cat_ref(x, a2).view(x.shape[:-1] + (w_il.shape[1],)), w_il, out)


def qkv_rope_cache_lora(x, a2, wqkv, pos, slot_of_row, cos_t, sin_t, kc, vc, Hq, Hkv, HD, q_out=None):
    """:func:`qkv_rope_cache` of ``[x | a2]``: the fused QKV + RoPE + KV-scatter epilogue with the bank's q / k / v
    deltas in the same GEMM (gemm4 G4_ROPE or ring RG_ROPE, two A sources)."""
    M = pos.numel()
    N, K = wqkv.shape
    if not x.is_cuda or HD != 256:
        return qkv_rope_cache(_cat_ref(x, a2), wqkv, pos, slot_of_row, cos_t, sin_t, kc, vc, Hq, Hkv, HD, q_out=q_out)
    q_out = _out(q_out, (M, Hq, HD), x.dtype, x.device)
    c = _l2a_choice(M, N, K, 4)
    cs = rope_cs(cos_t, sin_t)
    xs = x.reshape(M, -1)
    if isinstance(c, tuple):
        _k().gemm_ring_qkv_rope_l2a(xs, a2, wqkv, pos, slot_of_row, cs, q_out, kc, vc, int(Hq), int(Hkv), c[1], c[2])
    elif c == "gs":
        M1 = _GD.split_rows(M, N)
        for r0, r1, tr in ((0, M1, 256), (M1, M, 128)):
            if r1 > r0:
                _k().gemm4_qkv_rope_l2a(xs[r0:r1], a2[r0:r1], wqkv, pos.reshape(-1)[r0:r1],
                                        slot_of_row.reshape(-1)[r0:r1], cs, q_out[r0:r1], kc, vc, int(Hq), int(Hkv), tr)
    else:
        _k().gemm4_qkv_rope_l2a(xs, a2, wqkv, pos, slot_of_row, cs, q_out, kc, vc, int(Hq), int(Hkv), int(str(c)[1:]))
    return q_out


def decode_pre(step_idx, tf_tgt, tf_step, nb: int) -> None:
    """Greedy decode step, before the head: ``tf_step[r] = tf_tgt[r, min(step_idx[r], W - 1)]`` (``r < nb``)."""
    if tf_tgt.is_cuda:
        _k().decode_pre(step_idx, tf_tgt, tf_step, int(nb))
        return
    ref.decode_pre(step_idx, tf_tgt, tf_step, nb)


def decode_post(nxt, nll, tf_nll, done, step_idx, out_tok, out_nll, out_tf_nll, stop, tok, pos, nb: int,
                pad: int) -> None:
    """Greedy decode step, after the head, rows ``< nb``: the token (``pad`` once done) and its NLLs into output
    column ``min(step_idx, W - 1)``, ``done |= token in stop``, then next token, position + 1, column + 1 -- one
    kernel instead of ~12 PyTorch ones per captured step."""
    if nxt.is_cuda:
        _k().decode_post(nxt, nll, tf_nll, done, step_idx, out_tok, out_nll, out_tf_nll, stop, tok, pos, int(nb),
                         int(pad))
        return
    ref.decode_post(nxt, nll, tf_nll, done, step_idx, out_tok, out_nll, out_tf_nll, stop, tok, pos, nb, pad)


def share_lo_gather(rep, U, tok, pos, slot, s_tok, s_pos, s_slot, kp_slot, kp_len_lo, l_slot, l_len_lo, nb: int,
                    S: int) -> None:
    """Prefix-trie decode, blocks ``0..l``: lo row ``i < nb`` takes token, slot (and shared-prefix slot / length)
    of its group representative ``rep[i]``, and its position when ``i < U`` (else ``S``: parked)."""
    if tok.is_cuda:
        _k().share_lo_gather(rep, U, tok, pos, slot, s_tok, s_pos, s_slot, kp_slot, kp_len_lo, l_slot, l_len_lo,
                             int(nb), int(S))
        return
    ref.share_lo_gather(rep, U, tok, pos, slot, s_tok, s_pos, s_slot, kp_slot, kp_len_lo, l_slot, l_len_lo, nb, S)


def capture_rows(store, h, pos, slot, B: int, T: int) -> None:
    """``store[slot[b], p] = h[b * T + t]`` for ``p = pos[b, t]`` in ``[0, S1 - 1)``, else into the slot's scratch
    row ``S1 - 1`` (``store [slots, S1, D]`` bf16; one kernel, graph-capturable)."""
    if h.is_cuda:
        _k().capture_rows(store, h, pos.reshape(-1), slot.reshape(-1), int(T))
        return
    ref.capture_rows(store, h, pos, slot, B, T)


def row_gather(src, idx, out) -> None:
    """``out[i] = src[idx[i]]`` (bf16 rows of the last dimension; int32 / int64 indices)."""
    if src.is_cuda:
        _k().row_gather(src, idx, out)
        return
    torch.index_select(src.reshape(-1, src.shape[-1]), 0, idx.long(), out=out[: idx.numel()])


def share_group(gid, tok, rep, grp, src, U, nb: int, act: int, first: bool, vocab: int) -> bool:
    """Prefix-trie regrouping of rows ``< nb`` by (group ``gid``, token ``tok``) -- rows ``>= act`` form one parked
    group -- in one kernel (csrc/decode_step.hip): dense ``gid`` / ``grp``, each group's first row in ``rep``, the
    K/V fan-out source ``src`` (-1 for representatives and parked rows), the group count in ``U``.  Returns False
    (nothing done) off the GPU or past the kernel's row limit; the caller then runs the PyTorch version."""
    if not tok.is_cuda or nb > _share_group_max():
        return False
    _k().share_group(gid, tok.reshape(-1), rep, grp, src, U, int(nb), int(act), bool(first), int(vocab))
    return True


_SG_MAX = []


def _share_group_max() -> int:
    if not _SG_MAX:
        _SG_MAX.append(int(_k().share_group_max_rows()))
    return _SG_MAX[0]


def kv_fanout(kc, vc, src_row, slot, pos, nlayers: int) -> None:
    """Prefix-trie decode: copy the K/V of layers ``< nlayers`` that row ``src_row[r]`` wrote at its position
    into row ``r``'s own slot at ``r``'s position (``kc/vc [L, slots, Hkv, S, HD]``; ``src_row < 0`` or
    ``== r``: nothing).  A source row must not itself be a copy target (representatives only), so the
    rows are independent."""
    if kc.is_cuda:
        _k().kv_fanout(kc, vc, src_row, slot, pos, int(nlayers))
        return
    ref.kv_fanout(kc, vc, src_row, slot, pos, nlayers)


def attention(q, kc, vc, pos, slot, B, T, scale, softcap, window, out=None, prefix=None):
    """``prefix = (pk, pv, pslot, plen)`` (decode, T == 1): row ``b`` reads keys ``[0, plen[b])`` from slot
    ``pslot[b]`` of the shared prefix cache ``pk/pv [P, Hkv, S, HD]`` instead of its own slot."""
    if q.is_cuda:
        out = _out(out, (B * T, q.numel() // (B * T)), q.dtype, q.device)
        if prefix is not None:
            assert T == 1, "shared-prefix attention is decode-only"
            pk, pv, ps, pl = prefix
            _k().attention_prefix(q, kc, vc, out, pos, slot, int(B), float(scale), float(softcap), int(window),
                                  pk, pv, ps, pl)
            return out
        _k().attention(q, kc, vc, out, pos, slot, int(B), int(T), float(scale), float(softcap), int(window))
        return out
    o = ref.attention(q, kc, vc, pos, slot, B, T, scale, softcap, window,
                      prefix=prefix)
    if out is not None:
        out.copy_(o.view_as(out))
        return out
    return o


def attention_varlen(q, kc, vc, pos, slot_rows, blk, scale, softcap, window, out=None, prefix_kv=None):
    """Attention over packed rows ``q [M, Hq, HD]``: row ``i`` reads cache slot ``slot_rows[i]`` up to
    ``pos[i]``.  ``blk [nblk, 3] = (first row, rows, slot)`` groups consecutive rows of one sequence
    (<= 16 / GQA-ratio rows each) for the MFMA kernel; the CPU path only needs ``slot_rows``.
    ``prefix_kv = (pk, pv)`` with ``blk [nblk, 5]`` (+ prefix slot, prefix length): a block's keys below
    its prefix length come from that slot of the shared prefix cache ``pk/pv [P, Hkv, S, HD]``."""
    M = pos.numel()
    if q.is_cuda:
        out = _out(out, (M, q.numel() // M), q.dtype, q.device)
        if prefix_kv is not None:
            _k().attention_varlen_prefix(q, kc, vc, out, pos, blk, float(scale), float(softcap), int(window),
                                         prefix_kv[0], prefix_kv[1])
            return out
        _k().attention_varlen(q, kc, vc, out, pos, blk, float(scale), float(softcap), int(window))
        return out
    pre = None
    if prefix_kv is not None:
        ps = torch.zeros(M, dtype=torch.long)
        pl = torch.zeros(M, dtype=torch.long)
        for r0, n, _, s_, l_ in blk.cpu().long().tolist():
            ps[r0:r0 + n] = s_
            pl[r0:r0 + n] = l_
        pre = (prefix_kv[0], prefix_kv[1], ps, pl)
    o = ref.attention(q, kc, vc, pos, slot_rows, M, 1, scale, softcap, window, prefix=pre)
    if out is not None:
        out.copy_(o.view_as(out))
        return out
    return o


def geglu(gu, out=None):
    if gu.is_cuda:
        out = _out(out, gu.shape[:-1] + (gu.shape[-1] // 2,), gu.dtype, gu.device)
        _k().geglu(gu, out)
        return out
    y = ref.geglu(gu)
    if out is not None:
        out.copy_(y)
        return out
    return y


def argmax_rows(logits, cap=0.0, out=None):
    if logits.is_cuda:
        _softcap_table(cap, logits.device)
        out = _out(out, logits.shape[:-1], torch.int32, logits.device)
        _k().argmax_rows(logits, out, float(cap))
        return out
    y = ref.argmax_rows(logits, cap)
    if out is not None:
        out.copy_(y.view_as(out))
        return out
    return y


def row_lse(logits, cap=0.0, emulate_bf16=False, out=None):
    if logits.is_cuda:
        if emulate_bf16:
            _softcap_table(cap, logits.device)
        out = _out(out, logits.shape[:-1], torch.float32, logits.device)
        _k().row_lse(logits, out, float(cap), bool(emulate_bf16))
        return out
    y = ref.row_lse(logits, cap, emulate_bf16)
    if out is not None:
        out.copy_(y.view_as(out))
        return out
    return y


def _rows_of(logits, lse, rowmap):
    """CPU path of a ``rowmap``: materialise the logical rows."""
    V = logits.shape[-1]
    r = rowmap.view(-1).long()
    return logits.reshape(-1, V).index_select(0, r), lse.reshape(-1).index_select(0, r)


def gather_probs(logits, lse, ids, round_bf16=False, out=None, rowmap=None):
    """``p[r, k] = softmax(logits[row r])[ids[r, k]]``; ``rowmap [R]``: logical row ``r`` is logits row
    ``rowmap[r]`` (deduplicated rows)."""
    if logits.is_cuda:
        out = _out(out, ids.shape, torch.float32, logits.device)
        _k().gather_probs(logits, lse, ids, out, bool(round_bf16), rowmap)
        return out
    if rowmap is not None:
        logits, lse = _rows_of(logits, lse, rowmap)
    y = ref.gather_probs(logits, lse, ids, round_bf16).view(ids.shape)
    if out is not None:
        out.copy_(y)
        return out
    return y


def lens_colsum(logits, lse, mask, excl, B, T, acc=None, accumulate=False, round_bf16=False, offs=None, cum=None,
                rowmap=None):
    """Per-sequence sum over rows of ``softmax(logits)`` with 2 excluded ids per row.

    Dense layout: rows ``[B*T]`` with ``mask``; packed: ``offs [B+1]`` row offsets (``mask`` None, ``T``
    unused).  ``cum [B, T+1, V]`` (dense only) also receives the running sum after every row.
    ``rowmap [R]`` (packed only): logical row ``r`` (its exclusions, its place in ``offs``) reads logits row
    ``rowmap[r]`` — identical rows evaluated once."""
    V = logits.shape[-1]
    if logits.is_cuda:
        if acc is None:
            acc = torch.zeros(B, V, dtype=torch.float32, device=logits.device)
            accumulate = False
        _k().lens_colsum(logits, lse, mask, excl, acc, int(B), int(T), bool(accumulate), bool(round_bf16),
                         offs, cum, rowmap)
        return acc
    if rowmap is not None:
        logits, lse = _rows_of(logits, lse, rowmap)
    res = ref.lens_colsum(logits, lse, mask, excl, B, T, None, round_bf16, offs=offs, with_cum=cum is not None)
    s, c = res if isinstance(res, tuple) else (res, None)
    if acc is None:
        acc = s
    elif accumulate:
        if c is not None:
            c.add_(acc.view(B, 1, V))
        acc.add_(s)
    else:
        acc.copy_(s)
    if cum is not None:
        cum.copy_(c)
    return acc


def topk_rows(x, k) -> Tuple[torch.Tensor, torch.Tensor]:
    if x.is_cuda and k <= 64:
        R = x.numel() // x.shape[-1]
        vals = torch.empty(R, k, dtype=torch.float32, device=x.device)
        idx = torch.empty(R, k, dtype=torch.int32, device=x.device)
        _k().topk_rows(x.float().contiguous(), vals, idx, int(k))
        return vals, idx
    return ref.topk_rows(x.float(), k)


def xent_rows(logits, tgt, cap=0.0, emulate_bf16=True, out=None):
    if logits.is_cuda:
        if emulate_bf16:
            _softcap_table(cap, logits.device)
        out = _out(out, tgt.shape, torch.float32, logits.device)
        _k().xent_rows(logits, tgt, out, float(cap), bool(emulate_bf16))
        return out
    y = ref.xent_rows(logits, tgt, cap, emulate_bf16).view(tgt.shape)
    if out is not None:
        out.copy_(y)
        return out
    return y


# fused GEMM head (gemm4 G4_HEAD): opt-in; the in-tree logits GEMM + decode_head measured faster (round 2: 0.4-1.7 %,
# profiles/r2/head_ab/; round 5 in tb mode: 0.94-0.99x, profiles/r5/head_bench_tb.log); TB_FUSED_HEAD=1 / --fused-head
FUSED_HEAD = os.environ.get("TB_FUSED_HEAD", "0") == "1"


def head_part_numel(rows: int, vocab: int) -> int:
    """fp32 elements of the fused head's partial workspace for ``rows`` rows (16 B per 128 vocab columns)."""
    return rows * (vocab // 128) * 4


def vocab_head(x, w, cap, tgt=None, nxt=None, nll_self=None, nll_tgt=None, part=None, tgt_logit=None,
               fused: Optional[bool] = None):
    """``decode_head(x @ w^T, ...)`` from the final-normed rows ``x``: greedy token (bf16-softcap argmax), its
    NLL and the optional teacher target's NLL.  GPU with ``fused`` (default ``TB_FUSED_HEAD``): one
    four-wave MFMA GEMM (csrc/gemm4.hip G4_HEAD) whose epilogue applies the exact bf16 softcap table and reduces each row's 128-column
    slices to {max, sum exp, first argmax} (+ the target logit), then a merge kernel — the [rows, V] logits
    never reach HBM (``part``: optional fp32 workspace of ``head_part_numel`` elements, e.g. an idle logits
    buffer).  Otherwise the unembedding GEMM + ``decode_head``.  Returns ``(nxt, nll_self, nll_tgt)``."""
    K = x.shape[-1]
    R = x.numel() // K
    V = w.shape[0]
    fused = FUSED_HEAD if fused is None else fused
    if x.is_cuda and fused and _k().gemm4_ok(R, V, K) and x.is_contiguous():
        dev = x.device
        _softcap_table(cap, dev)
        nxt = _out(nxt, (R,), torch.int32, dev)
        nll_self = _out(nll_self, (R,), torch.float32, dev)
        need = head_part_numel(R, V)
        part = torch.empty(need, dtype=torch.float32, device=dev) if part is None else part.view(-1)[:need]
        if tgt is not None:
            nll_tgt = _out(nll_tgt, (R,), torch.float32, dev)
            tgt_logit = _out(tgt_logit, (R,), torch.float32, dev)
            _k().head_fused(x, w, part, float(cap), tgt, tgt_logit, nxt, nll_self, nll_tgt)
        else:
            _k().head_fused(x, w, part, float(cap), None, None, nxt, nll_self, None)
        return nxt, nll_self, nll_tgt
    return decode_head(linear(x, w), cap, tgt, nxt, nll_self, nll_tgt)


FUSED_LENS = os.environ.get("TB_FUSED_LENS", "1") == "1"   # gemm4 G4_LENS (round 4); 0: GEMM dispatch + row_lse
_LENS_PART: dict = {}


def _lens_part(n: int, device) -> torch.Tensor:
    """The fused lens GEMM's fp32 partial workspace: one grow-only buffer per (device, stream), consumed by the
    merge kernel on the same stream before the next lens GEMM can overwrite it (no allocation per call)."""
    key = (device.index, torch.cuda.current_stream(device).stream_id)
    b = _LENS_PART.get(key)
    if b is None or b.numel() < n:
        b = torch.empty(max(n, 2 * b.numel() if b is not None else n), dtype=torch.float32, device=device)
        _LENS_PART[key] = b
        _SPLITK_KEEP.append(b)            # a captured graph may still hold an outgrown buffer
    return b[:n]


def lens_unembed(xn, w, fused: Optional[bool] = None, out=None, lse_out=None):
    """Logit-lens unembedding of final-normed rows: ``(logits = xn @ w^T (bf16), lse = logsumexp(logits))``, no
    softcap.  GPU with ``fused`` (default ``TB_FUSED_LENS``, off under ``TB_GEMM=blas``): one four-wave MFMA GEMM
    (csrc/gemm4.hip G4_LENS) that stores the bf16 logits and reduces each row's 128-column slices to {max, sum exp}
    in its epilogue, then the partial merge (tb_head_merge) -- no separate ``row_lse`` pass over the logits.
    Otherwise ``linear`` (the GEMM dispatch: hipBLASLt under ``blas``) + ``row_lse``."""
    K = xn.shape[-1]
    R = xn.numel() // K
    V = w.shape[0]
    fused = (FUSED_LENS and _GD.mode() != "blas") if fused is None else fused
    if xn.is_cuda and fused and _k().gemm4_ok(R, V, K) and xn.is_contiguous():
        logits = _out(out, xn.shape[:-1] + (V,), BF16, xn.device)
        part = _lens_part(head_part_numel(R, V), xn.device)
        lse = _out(lse_out, xn.shape[:-1], torch.float32, xn.device)
        _k().lens_gemm(xn, w, logits, part, lse)
        return logits, lse
    logits = linear(xn, w, out=out)
    return logits, row_lse(logits)


def decode_head(logits, cap, tgt=None, nxt=None, nll_self=None, nll_tgt=None):
    """One pass over decode logits: greedy token (bf16-softcap argmax), its NLL, and the NLL of an
    optional teacher target per row (``tgt < 0`` -> 0).  Returns ``(nxt, nll_self, nll_tgt)``."""
    R = logits.numel() // logits.shape[-1]
    dev = logits.device
    nxt = _out(nxt, (R,), torch.int32, dev)
    nll_self = _out(nll_self, (R,), torch.float32, dev)
    if tgt is not None:
        nll_tgt = _out(nll_tgt, (R,), torch.float32, dev)
    if logits.is_cuda:
        _softcap_table(cap, logits.device)
        _k().decode_head(logits, tgt, nxt, nll_self, nll_tgt if tgt is not None else None, float(cap))
        return nxt, nll_self, nll_tgt
    nxt.copy_(ref.argmax_rows(logits, cap).view(R))
    nll_self.copy_(ref.xent_rows(logits, nxt, cap, True).view(R))
    if tgt is not None:
        nll_tgt.copy_(ref.xent_rows(logits, tgt, cap, True).view(R))
    return nxt, nll_self, nll_tgt


def slot_copy(dst: torch.Tensor, src: torch.Tensor, dst_slots, src_slots, layers: Optional[range] = None,
              src_layers: Optional[range] = None) -> None:
    """``dst[l, dst_slots[i]] = src[l', src_slots[i]]`` for the layer ranges ``layers`` (of dst) and ``src_layers``
    (of src, default the same) of two ``[L, slots, ...]`` bf16 tensors (KV caches): one pass on the GPU
    (``csrc/elementwise.hip`` slot_copy), no temporary.  Slot lists are host sequences (checked here)."""
    ds, ss = [int(v) for v in dst_slots], [int(v) for v in src_slots]
    assert len(ds) == len(ss)
    if not ds:
        return
    layers = range(dst.shape[0]) if layers is None else layers
    src_layers = layers if src_layers is None else src_layers
    assert len(layers) == len(src_layers) and layers.step == 1 and src_layers.step == 1
    if not len(layers):
        return
    assert 0 <= min(ds) and max(ds) < dst.shape[1] and 0 <= min(ss) and max(ss) < src.shape[1], "slot out of range"
    if dst.is_cuda and dst.dtype == BF16 and src.dtype == BF16 and dst.is_contiguous() and src.is_contiguous():
        dt = torch.tensor(ds, dtype=torch.int32).pin_memory().to(dst.device, non_blocking=True)
        st = torch.tensor(ss, dtype=torch.int32).pin_memory().to(dst.device, non_blocking=True)
        _k().slot_copy(dst, src, dt, st, int(layers.start), int(src_layers.start), len(layers))
        return
    d = torch.tensor(ds, device=dst.device)
    s_ = torch.tensor(ss, device=dst.device)
    dst[layers.start:layers.stop].index_copy_(1, d, src[src_layers.start:src_layers.stop].index_select(1, s_))


# ------------------------------------------------------------------ vocab-parallel merges (csrc/vp.hip)
def decode_head_stats(logits, tgt, off: int, cap: float, out=None):
    """Vocab-parallel head, this rank's columns ``logits [R, V_local]`` (vocab ids ``off ..``): per row
    ``{log-sum-exp, best capped logit, its global id, teacher target's capped logit or -inf}`` as ``[R, 4]`` fp32 from
    one HIP pass (csrc/lens.hip decode_head_f_kernel, stats mode) -- the input of :func:`vp_head_merge` after the
    group's all-gather.  None off the GPU or for a cap without a registered table (callers use the PyTorch path)."""
    if not logits.is_cuda or not (cap > 0):
        return None
    _softcap_table(cap, logits.device)
    R = logits.numel() // logits.shape[-1]
    out = _out(out, (R, 4), torch.float32, logits.device)
    if not _k().decode_head_stats(logits, tgt, int(off), out, float(cap)):
        return None
    return out


def vp_head_merge(st, tgt, V: int, nxt=None, nll_self=None, nll_tgt=None):
    """Merge the per-rank head stats ``st [tp, R, 4]`` = {log-sum-exp, best capped logit, its global index,
    target logit (-inf off the rank's slice)} in rank order: greedy token, its NLL and the teacher target's NLL
    (0 for targets outside ``[0, V)``), identical to :func:`decode_head` on the full row."""
    tp, R = st.shape[0], st.shape[1]
    dev = st.device
    nxt = _out(nxt, (R,), torch.int32, dev)
    nll_self = _out(nll_self, (R,), torch.float32, dev)
    if tgt is not None:
        nll_tgt = _out(nll_tgt, (R,), torch.float32, dev)
    if st.is_cuda:
        _k().vp_head_merge(st.contiguous(), tgt, int(V), nxt, nll_self, nll_tgt if tgt is not None else None)
        return nxt, nll_self, nll_tgt
    a, b, c = ref.vp_head_merge(st, tgt, V)
    nxt.copy_(a)
    nll_self.copy_(b)
    if tgt is not None:
        nll_tgt.copy_(c)
    return nxt, nll_self, nll_tgt


def vp_lse_merge(lse_parts: torch.Tensor, out=None) -> torch.Tensor:
    """``[tp, R]`` per-rank log-sum-exps of disjoint vocab slices -> ``[R]`` log-sum-exp of the whole row."""
    R = lse_parts.shape[1]
    out = _out(out, (R,), torch.float32, lse_parts.device)
    if lse_parts.is_cuda:
        _k().vp_lse_merge(lse_parts.float().contiguous(), out)
        return out
    out.copy_(ref.vp_lse_merge(lse_parts))
    return out


def vp_topk_merge(vals: torch.Tensor, ids: torch.Tensor):
    """Per-rank top-k candidates ``[tp, n, k]`` (values, GLOBAL ids) -> the global top-k ``[n, k]``, descending,
    ties to the lower id (the order of :func:`topk_rows` on the full row)."""
    tp, n, k = vals.shape
    if vals.is_cuda and k <= 64:
        ov = torch.empty(n, k, dtype=torch.float32, device=vals.device)
        oi = torch.empty(n, k, dtype=torch.int32, device=vals.device)
        _k().vp_topk_merge(vals.float().contiguous(), ids.to(torch.int32).contiguous(), ov, oi)
        return ov, oi
    return ref.vp_topk_merge(vals, ids)


def gemm_nt(A, W, epi=0, bias=None, thr=None, out=None):
    """C = A @ W^T on an MFMA kernel; epi 0 = bf16, 1 = fp32, 2 = JumpReLU(acc + bias, thr) fp32.
    Shapes with N % 256 == 0 and K % 64 == 0 (the SAE encode: N = 16384, K = 3584) run the four-wave
    256x256 kernel (csrc/gemm4.hip); others the 128x128 ``gemm_nt`` kernel (csrc/sae.hip)."""
    M = A.numel() // A.shape[-1]
    N = W.shape[0]
    if A.is_cuda:
        out = _out(out, (M, N), BF16 if epi == 0 else torch.float32, A.device)
        if _k().gemm4_ok(M, N, A.shape[-1]) and A.is_contiguous():
            tb_gemm(A, W, out, bias, thr, int(epi), _GD.fill_choice(max(M, 4096), N))
        else:
            _k().gemm_nt(A, W, out, bias, thr, int(epi))
        return out
    y = ref.gemm_nt(A, W, epi, bias, thr)
    if out is not None:
        out.copy_(y.view_as(out))
        return out
    return y


def geglu_interleave_index(F: int, device=None) -> torch.Tensor:
    """Row order of a gate|up weight ``[2F, K]`` for the fused GeGLU epilogues (epi 3):
    every 256-row tile holds features ``f0 .. f0+127`` as two 128-row wave-group slices
    ``[gate 64 | up 64]``, so a lane's gate and up accumulators of the same feature land in the same
    lane (csrc/gemm4.hip G4_GEGLU, csrc/gemm_ring.hip RG_GEGLU).  Needs F % 128 == 0."""
    assert F % 128 == 0, "fused GeGLU needs ffn % 128 == 0"
    p = torch.arange(2 * F)
    tile, q = p // 256, p % 256
    g, half, rest = q // 128, (q // 64) % 2, q % 64
    return (half * F + tile * 128 + g * 64 + rest).to(device)


reference_geglu = ref.geglu


def fused_geglu_wins(x: torch.Tensor, spec) -> bool:
    """Whether the gate|up GEMM of ``x``'s rows runs fused with the GeGLU (in-tree kernel) rather than as
    ``linear`` + ``geglu`` (the dispatch table's epilogue-3 entry; ``TB_GEMM=tb`` always, ``blas`` never)."""
    M = x.numel() // x.shape[-1]
    return _GD.choose(M, 2 * spec.ffn, x.shape[-1], 3) != "blas"


def gate_up_geglu(x: torch.Tensor, w_gu_interleaved: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``geglu(x @ w_gu^T)`` in one in-tree MFMA GEMM (gemm4 G4_GEGLU or ring RG_GEGLU) whose epilogue applies GeGLU to the fp32 accumulators
    (rounded to bf16 first, so the result equals the unfused bf16 graph up to the GEMM's summation order);
    ``w_gu_interleaved = w_gu[geglu_interleave_index(F)]``."""
    M = x.numel() // x.shape[-1]
    F = w_gu_interleaved.shape[0] // 2
    if x.is_cuda:
        out = _out(out, x.shape[:-1] + (F,), BF16, x.device)
        c = _GD.choose(M, 2 * F, x.shape[-1], 3)
        tb_gemm(x, w_gu_interleaved, out, None, None, 3, c if c != "blas" else _GD.fill_choice(M, 2 * F))
        return out
    inv = torch.argsort(geglu_interleave_index(F))
    y = ref.geglu((x.reshape(M, -1).float() @ w_gu_interleaved[inv].float().T).to(BF16)).view(x.shape[:-1] + (F,))
    if out is not None:
        out.copy_(y)
        return out
    return y


def lowrank_edit(h, apply, idx, cnt, E, Dm, bias=None, thr=None, pre_bias=None, alpha=1.0, w_next=None, eps=1e-6,
                 x_next=None, coef_out=None):
    """Per flagged row: h -= sum_j f(<h - pre_bias, E_j> + bias_j) * alpha * Dm_j; refresh x_next = norm(h)."""
    if h.is_cuda:
        _k().lowrank_edit(h, x_next, apply, idx, cnt, E, Dm, bias, thr, pre_bias, float(alpha), w_next, float(eps),
                          coef_out)
        return h
    ref.lowrank_edit(h, apply, idx, cnt, E, Dm, bias, thr, pre_bias, alpha, w_next, eps, x_next, coef_out)
    return h


def sae_decode_sparse(acts, Wdec, b_dec=None, out_bf16=None, out_f32=None):
    if acts.is_cuda:
        M = acts.numel() // Wdec.shape[0]
        if out_bf16 is None and out_f32 is None:
            out_f32 = torch.empty(M, Wdec.shape[1], dtype=torch.float32, device=acts.device)
        _k().sae_decode_sparse(acts, Wdec, b_dec, out_bf16, out_f32)
        return out_f32 if out_f32 is not None else out_bf16
    y = ref.sae_decode_sparse(acts, Wdec, b_dec)
    if out_f32 is not None:
        out_f32.copy_(y)
        return out_f32
    if out_bf16 is not None:
        out_bf16.copy_(y.to(BF16))
        return out_bf16
    return y


def latent_score(acts, p, spike, seg):
    """Returns (score, spike_mean, corr), each [G, L]."""
    if acts.is_cuda:
        G = seg.numel() - 1
        L = acts.shape[-1]
        out = torch.empty(G, L, dtype=torch.float32, device=acts.device)
        sm = torch.empty_like(out)
        cr = torch.empty_like(out)
        _k().latent_score(acts, p, spike, seg, out, sm, cr)
        return out, sm, cr
    return ref.latent_score(acts, p, spike, seg)
