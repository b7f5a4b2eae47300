"""Logit-lens readouts.

Reference semantics (`src/models.py:127-144`, `src/01_reproduce_logit_lens.py:35-71,120-150`):

* per layer ``l`` and position ``t``: ``p_l(t) = softmax(lm_head(norm_f(h_l(t))))``
  — final RMSNorm, tied unembedding, **no** final softcap; the reference does
  the softmax in bf16 (``round_bf16=True`` reproduces that, default fp32);
* LL-Top-k: sum ``p_31(t)`` over the response positions, zeroing at position
  ``i`` the ids ``convert_tokens_to_ids(decode(tok_i))`` and ``…(tok_{i-1})``
  (mostly ``<unk>``, SURVEY 7.3.6: ``exclusion="reference"``), then top-k.
  ``exclusion="response"`` removes every id that occurs in the response (the
  paper's stated rule, Paper p.3) and ``"none"`` keeps everything.

The reference materialises ``[42, T, 256000]`` fp32 on the host (1.63 GB per
prompt).  Here everything stays on the GPU: lens logits come from one
hipBLASLt GEMM per chunk of rows, and the HIP kernels ``row_lse``,
``gather_probs``, ``lens_colsum`` and ``topk_rows`` reduce them to the few
numbers the analysis needs.  The full probability tensor is only produced on
request (``full_probs``) for the reference-compatible cache.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from .. import ops


@dataclass
class LensResult:
    topk_ids: List[List[int]]
    topk_vals: List[List[float]]
    probs: List[np.ndarray]              # per sequence [n_resp, n_ids] lens probs of the tracked ids
    resp_sum: Optional[torch.Tensor] = None   # [n_seq, V] (kept on device when requested)
    cum: Optional[List[torch.Tensor]] = None  # per sequence [n_resp + 1, V] running response sums (device)


def _excl_id(tok, t: int) -> int:
    cache = getattr(tok, "_tb_excl_cache", None)
    if cache is None:
        cache = {}
        try:
            tok._tb_excl_cache = cache
        except AttributeError:
            pass
    v = cache.get(int(t))
    if v is None:
        v = cache[int(t)] = int(tok.convert_tokens_to_ids(tok.decode([int(t)])))
    return v


def excl_table(tok, vocab_size: int) -> np.ndarray:
    """``table[id] = convert_tokens_to_ids(decode([id]))`` for every id (built once per tokenizer), so the
    reference's per-position exclusions of a whole batch are one array gather."""
    tab = getattr(tok, "_tb_excl_table", None)
    if tab is None or tab.shape[0] < vocab_size:
        tab = np.fromiter((_excl_id(tok, t) for t in range(vocab_size)), dtype=np.int64, count=vocab_size)
        try:
            tok._tb_excl_table = tab
        except AttributeError:
            pass
    return tab


def reference_exclusions(tok, ids: Sequence[int]) -> List[Tuple[int, int]]:
    """Per response position: (id of current token, id of previous token or -1) as the reference
    computes them via ``convert_tokens_to_ids(decoded_string)`` (`src/01_reproduce_logit_lens.py:56-69`).
    The per-token lookup is memoised (it is a pure function of the token id)."""
    cur = [_excl_id(tok, t) for t in ids]
    return [(c, cur[i - 1] if i > 0 else -1) for i, c in enumerate(cur)]


def _rows_for(store: torch.Tensor, seqs: Sequence[int], starts: Sequence[int], lens: Sequence[int], Tr: int):
    """Flat row indices into ``store.view(-1, D)`` for a chunk; padding rows point at the scratch row."""
    S1 = store.shape[1]
    idx = torch.empty(len(seqs), Tr, dtype=torch.long)
    mask = torch.zeros(len(seqs), Tr, dtype=torch.uint8)
    for i, (b, s0, n) in enumerate(zip(seqs, starts, lens)):
        t = torch.arange(Tr)
        valid = t < n
        idx[i] = torch.where(valid, b * S1 + s0 + t, torch.full_like(t, b * S1 + S1 - 1))
        mask[i, :n] = 1
    return idx, mask


# ------------------------------------------------------------------ vocab-parallel lens (TP)
# Under tensor parallelism with ``parallel.vocab_parallel`` the model's ``lens_logits_lse`` returns this rank's
# ``V / tp`` logit columns (its slice of lm_head) with the row's GLOBAL log-sum-exp (one all-gather of the local
# LSEs + ``ops.vp_lse_merge``).  The readouts below then work on local columns: tracked / excluded vocab ids are
# shifted into the slice (ids outside it fall out of range and read as "none"), tracked-id probabilities are summed
# over the group (each id lives on one rank; the other ranks contribute exact zeros), and the response-sum top-k
# merges every rank's top-k candidates (``ops.vp_topk_merge``, ties to the lower vocab id as on one GPU).
def vocab_slice(model) -> Tuple[int, int]:
    """``(first vocab id, count)`` of the lens columns this rank computes."""
    V = model.spec.vocab_size
    if getattr(model, "vocab_parallel", False):
        n = V // model.tp.size
        return model.tp.rank * n, n
    return 0, V


def vocab_reduce_(model, t: torch.Tensor) -> torch.Tensor:
    """Sum of per-rank partial readouts over the vocab-parallel group (in place; identity otherwise)."""
    if getattr(model, "vocab_parallel", False):
        model.tp.all_reduce_(t)
    return t


def vocab_topk(model, acc: torch.Tensor, k: int):
    """Top-k (values, GLOBAL vocab ids) of the response sums ``acc [n, V_local]``."""
    vals, ids = ops.topk_rows(acc, k)
    if not getattr(model, "vocab_parallel", False):
        return vals, ids
    ids = ids + vocab_slice(model)[0]
    return ops.vp_topk_merge(model.tp.all_gather_(vals.contiguous()), model.tp.all_gather_(ids.contiguous()))


def vocab_argmax(model, logits: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """First-index argmax (GLOBAL vocab id, int32) of every row of the local lens logits."""
    am = ops.argmax_rows(logits)
    if getattr(model, "vocab_parallel", False):
        R = am.numel()
        val = logits.reshape(R, -1).gather(1, am.view(R, 1).long()).float()
        _, ids = ops.vp_topk_merge(model.tp.all_gather_(val.contiguous()),
                                   model.tp.all_gather_((am.view(R, 1) + vocab_slice(model)[0]).contiguous()))
        am = ids.view(am.shape)
    if out is not None:
        out.copy_(am.view_as(out))
        return out
    return am


def vocab_gather_cols(model, t: torch.Tensor) -> torch.Tensor:
    """``[..., V_local]`` per-rank columns -> ``[..., V]`` (rank order = vocab order); identity without TP."""
    if not getattr(model, "vocab_parallel", False):
        return t
    g = model.tp.all_gather_(t.contiguous())                        # [tp, ..., V_local]
    return torch.cat(list(g.unbind(0)), dim=-1)


@torch.no_grad()
def lens_readout(model, store: torch.Tensor, starts: Sequence[int], lens: Sequence[int], track_ids: Sequence[Sequence[int]],
                 top_k: int = 5, exclusion: str = "reference", excl_pairs: Optional[Sequence[Sequence[Tuple[int, int]]]] = None,
                 response_ids: Optional[Sequence[Sequence[int]]] = None, round_bf16: bool = False,
                 chunk_bytes: int = 2 << 30, keep_sums: bool = False, seqs: Optional[Sequence[int]] = None,
                 keep_cum: bool = False) -> LensResult:
    """Lens over the residual ``store [slots, S+1, D]`` (a :class:`CaptureHook` buffer).

    ``starts[i]``/``lens[i]``: response span of sequence ``seqs[i]`` (default ``i``).
    ``track_ids[i]``: ids whose per-position lens probability is returned (secret first, then decoys).
    ``keep_cum``: also return every prefix sum of the (excluded) response probabilities, so a
    sequence that later shares a prefix with this one can reuse it (:func:`lens_packed`).
    """
    n = len(starts)
    seqs = list(range(n)) if seqs is None else list(seqs)
    dev = store.device
    lo, V = vocab_slice(model)               # this rank's lens columns (the whole vocab without vocab-parallel TP)
    D = store.shape[-1]
    Tr = max(1, max(lens) if lens else 1)
    Tr = -(-Tr // 16) * 16                  # few distinct GEMM shapes
    per_seq = Tr * V * 2
    nb = max(1, min(n, chunk_bytes // max(per_seq, 1)))
    K = max(1, max(len(t) for t in track_ids))
    topk_ids: List[List[int]] = []
    topk_vals: List[List[float]] = []
    probs: List[np.ndarray] = []
    sums = [] if keep_sums else None
    cums: Optional[List[torch.Tensor]] = [] if keep_cum else None
    flat = store.view(-1, D)
    for c0 in range(0, n, nb):
        c1 = min(n, c0 + nb)
        m = c1 - c0
        idx, mask = _rows_for(store, seqs[c0:c1], starts[c0:c1], lens[c0:c1], Tr)
        rows = flat.index_select(0, idx.view(-1).to(dev))
        logits, lse = model.lens_logits_lse(rows)                          # [m*Tr, V] bf16, [m*Tr]
        tid = torch.full((m, Tr, K), -1, dtype=torch.int32)
        ex = torch.full((m, Tr, 2), -1, dtype=torch.int32)
        for i in range(m):
            tt = list(track_ids[c0 + i])
            tid[i, :, : len(tt)] = torch.tensor(tt, dtype=torch.int32)
            if exclusion == "reference" and excl_pairs is not None:
                pr = excl_pairs[c0 + i][: Tr]
                if pr:
                    ex[i, : len(pr)] = torch.tensor(pr, dtype=torch.int32)
        if lo:                                # global ids -> this rank's columns (others fall out of range)
            tid = torch.where(tid >= 0, tid - lo, tid)
            ex = torch.where(ex >= 0, ex - lo, ex)
        p = vocab_reduce_(model, ops.gather_probs(logits, lse, tid.view(m * Tr, K).to(dev), round_bf16=round_bf16))
        cum = torch.empty(m, Tr + 1, V, dtype=torch.float32, device=dev) if keep_cum else None
        acc = ops.lens_colsum(logits, lse, mask.view(-1).to(dev), ex.view(-1, 2).to(dev), m, Tr,
                              round_bf16=round_bf16, cum=cum)
        if keep_cum:
            for i in range(m):
                cums.append(cum[i, : lens[c0 + i] + 1].clone())
            del cum
        if exclusion == "response" and response_ids is not None:
            for i in range(m):
                r = torch.tensor(sorted(set(response_ids[c0 + i])), dtype=torch.long, device=dev) - lo
                r = r[(r >= 0) & (r < V)]
                if r.numel():
                    acc[i, r] = 0.0
        vals, ids = vocab_topk(model, acc, top_k)
        pc = p.view(m, Tr, K).cpu().numpy()
        vh, ih = vals.cpu(), ids.cpu()
        for i in range(m):
            L = lens[c0 + i]
            probs.append(pc[i, :L, : len(track_ids[c0 + i])])
            if L > 0 and float(vh[i].sum()) > 0:
                topk_ids.append([int(v) for v in ih[i].tolist()])
                topk_vals.append([float(v) for v in vh[i].tolist()])
            else:
                topk_ids.append([])
                topk_vals.append([])
        if keep_sums:
            sums.append(acc)
        del logits, lse, p, rows
    return LensResult(topk_ids, topk_vals, probs, torch.cat(sums) if keep_sums else None, cums)


LENS_CHUNK_DISTINCT = os.environ.get("TB_LENS_CHUNK_DISTINCT", "1") == "1"   # 0: chunks of chunk_rows logical rows


@torch.no_grad()
def lens_packed(model, store: torch.Tensor, rows: np.ndarray, offs: np.ndarray, base: torch.Tensor,
                track: np.ndarray, excl: np.ndarray, round_bf16: bool = False,
                chunk_rows: int = 4096, sync: bool = True, row_key: Optional[np.ndarray] = None,
                stats: Optional[dict] = None, row_check: Optional[np.ndarray] = None):
    """Partial lens over packed rows: sequence ``i`` owns flat rows ``rows[offs[i]:offs[i+1]]`` of
    ``store.view(-1, D)`` (no padding) and adds their (excluded) lens probabilities onto ``base[i]``
    (the reused part of its response sum, updated in place).  ``track [R, K]`` are per-row ids whose
    probabilities are returned (``-1`` = none), ``excl [R, 2]`` the per-row excluded ids.
    Returns ``(base, probs [R, K])``; ``sync=False`` returns the probabilities as a device tensor instead
    (no host wait: the caller copies them back when it needs them).

    ``row_key [R]`` (optional): rows with equal keys hold identical residuals (e.g. sweep cells of one pair
    with equal tokens, at positions without an edit); each chunk then unembeds one row per key and the
    readout kernels read it through a row map (the lens GEMM shrinks, the sums are unchanged).  ``row_check``
    (optional, a second independent key): a chunk whose rows of one ``row_key`` disagree on it (a hash
    collision) is evaluated without dedup."""
    dev = store.device
    D = store.shape[-1]
    flat = store.view(-1, D)
    n = len(offs) - 1
    R = int(offs[-1]) if n > 0 else 0
    K = track.shape[1] if track.ndim == 2 else 1
    probs = np.zeros((R, K), dtype=np.float32)
    if R == 0:
        return base, (probs if sync else torch.from_numpy(probs))
    # chunk plan on the host (whole sequences, <= chunk_rows rows, GEMM rows padded to 256-row tiles; the
    # padding rows repeat the chunk's first row), then ONE upload of every index array: the loop below
    # only slices device tensors, so the host never waits for the GPU between chunks
    chunks, ridx_l, offs_l, map_l = [], [], [], []
    prev = None
    if row_key is not None and LENS_CHUNK_DISTINCT:
        # prev[i]: the previous row with row i's key (-1: none).  Rows [r0, r) hold as many distinct keys as rows
        # i in [r0, r) with prev[i] < r0, so a deduplicated chunk can take whole sequences until its GEMM has
        # chunk_rows distinct rows (full 256-row tiles) instead of stopping at chunk_rows logical rows (round 6:
        # at the bench's 4096 that left ~1900 GEMM rows per chunk, a padded tile each and a lower MFMA rate)
        order = np.argsort(row_key, kind="stable")
        same = row_key[order[1:]] == row_key[order[:-1]]
        prev = np.full(R, -1, dtype=np.int64)
        prev[order[1:][same]] = order[:-1][same]
    i0, pr0, po0 = 0, 0, 0
    while i0 < n:
        i1 = int(np.searchsorted(offs, offs[i0] + chunk_rows, side="right")) - 1
        i1 = min(n, max(i1, i0 + 1))
        if prev is not None and i1 < n:
            r0 = int(offs[i0])
            w1 = min(R, r0 + 8 * chunk_rows)                 # look-ahead window (bounds the host work)
            cnt = np.concatenate([[0], np.cumsum(prev[r0:w1] < r0)])
            ends = offs[i0 + 1:] - r0
            ends = ends[ends <= w1 - r0]
            i1 = min(n, max(i0 + int(np.searchsorted(cnt[ends], chunk_rows, side="right")), i1))
        r0, r1 = int(offs[i0]), int(offs[i1])
        if r1 > r0:
            dedup = row_key is not None
            if dedup:                    # one GEMM row per distinct key, logical rows mapped onto them
                _, first, inv = np.unique(row_key[r0:r1], return_index=True, return_inverse=True)
                inv = inv.reshape(-1)
                if row_check is not None and not np.array_equal(row_check[r0:r1][first][inv], row_check[r0:r1]):
                    # collision: this chunk un-deduplicated, back to chunk_rows logical rows
                    i1 = min(n, max(int(np.searchsorted(offs, offs[i0] + chunk_rows, side="right")) - 1, i0 + 1))
                    r1 = int(offs[i1])
                    first, inv = np.arange(r1 - r0), np.arange(r1 - r0)
                src = rows[r0:r1][first]
                map_l.append(inv.astype(np.int32))
            else:
                src = rows[r0:r1]
            M = len(src)
            if stats is not None:
                stats["lens_gemm_rows"] = stats.get("lens_gemm_rows", 0) + M
            Mp = -(-M // 256) * 256
            ridx_l.append(np.concatenate([src, np.full(Mp - M, src[0], dtype=np.int64)]))
            offs_l.append((offs[i0:i1 + 1] - r0).astype(np.int32))
            # deduplicated chunks run the 256-row padded GEMM (the padding repeats a row; the row map never
            # reads it): few distinct shapes, all in the TunableOp tables
            chunks.append((i0, i1, r0, r1, pr0, Mp if dedup else M, po0))
            pr0 += Mp
            po0 += i1 - i0 + 1
        i0 = i1
    def up(a):    # pinned + non-blocking on GPU: no stream drain while earlier work is queued
        t = torch.from_numpy(np.ascontiguousarray(a))
        return t.pin_memory().to(dev, non_blocking=True) if dev.type == "cuda" else t

    ridx_d = up(np.concatenate(ridx_l).astype(np.int64))
    offs_d = up(np.concatenate(offs_l))
    lo = vocab_slice(model)[0]
    track_a, excl_a = np.asarray(track, dtype=np.int32), np.asarray(excl, dtype=np.int32)
    if lo:                                    # global ids -> this rank's lens columns
        track_a = np.where(track_a >= 0, track_a - lo, track_a)
        excl_a = np.where(excl_a >= 0, excl_a - lo, excl_a)
    track_d = up(track_a)
    excl_d = up(excl_a)
    map_d = up(np.concatenate(map_l)) if map_l else None
    pr_d = torch.empty(R, K, dtype=torch.float32, device=dev)
    for i0, i1, r0, r1, pr0, M, po0 in chunks:
        logits, lse = model.lens_logits_lse(flat.index_select(0, ridx_d[pr0:pr0 + M]))
        rm = map_d[r0:r1] if map_d is not None else None
        ops.gather_probs(logits, lse, track_d[r0:r1], round_bf16=round_bf16, out=pr_d[r0:r1], rowmap=rm)
        ops.lens_colsum(logits, lse, None, excl_d[r0:r1], i1 - i0, 0, acc=base[i0:i1], accumulate=True,
                        round_bf16=round_bf16, offs=offs_d[po0:po0 + (i1 - i0) + 1], rowmap=rm)
    vocab_reduce_(model, pr_d)
    if not sync:
        return base, pr_d
    probs[:] = pr_d.cpu().numpy()
    return base, probs


@torch.no_grad()
def all_layer_lens(model, stores: Sequence[torch.Tensor], seq: int, start: int, length: int, track_ids: Sequence[int],
                   full_probs: bool = False, round_bf16: bool = True):
    """Every layer's lens for one sequence's positions ``[start, start+length)``.

    ``stores[l]`` is the capture buffer of layer ``l``.  Returns
    ``(p_track [L, length, K] np.float32, argmax [L, length] np.int64, full [L, length, V] np.float32 | None)``
    — ``full`` is the reference's ``all_probs`` (`src/models.py:143-144`) when requested.
    """
    Lh = len(stores)
    dev = stores[0].device
    V = model.spec.vocab_size
    lo = vocab_slice(model)[0]
    K = len(track_ids)
    p_track = np.zeros((Lh, length, K), dtype=np.float32)
    amax = np.zeros((Lh, length), dtype=np.int64)
    full = np.zeros((Lh, length, V), dtype=np.float32) if full_probs else None
    tid = torch.tensor([t - lo if t >= 0 else t for t in track_ids], dtype=torch.int32,
                       device=dev).view(1, K).expand(length, K).contiguous()
    for l in range(Lh):
        rows = stores[l][seq, start:start + length]
        logits, lse = model.lens_logits_lse(rows.contiguous())
        if K:
            p_track[l] = vocab_reduce_(model, ops.gather_probs(logits, lse, tid, round_bf16=round_bf16)).cpu().numpy()
        amax[l] = vocab_argmax(model, logits).cpu().numpy()
        if full is not None:
            pr = torch.exp(logits.float() - lse[:, None])
            if round_bf16:
                pr = pr.to(torch.bfloat16).float()
            full[l] = vocab_gather_cols(model, pr).cpu().numpy()
    return p_track, amax, full


def aggregate_cached_probs(probs: torch.Tensor, response_tokens: Sequence[str], tok=None,
                           exclusion: str = "reference") -> torch.Tensor:
    """Response-sum of cached per-position probabilities ``probs [T, V]`` (the reference's
    ``aggregate_response_logits``, `src/01_reproduce_logit_lens.py:35-71`), vectorised.

    ``exclusion="reference"`` zeroes, at position i, the ids that ``tok.convert_tokens_to_ids``
    returns for the decoded strings of tokens i and i-1; without a tokenizer those lookups are
    treated as ``<unk>`` misses except for exact special tokens, which is what the real Gemma
    tokenizer does for space-prefixed decoded strings.
    """
    p = probs.float().clone()
    T, V = p.shape
    if exclusion == "reference" and tok is not None:
        ids = [tok.convert_tokens_to_ids(s) for s in response_tokens]
        for i in range(T):
            for j in ((ids[i],) + ((ids[i - 1],) if i > 0 else ())):
                if j is not None and 0 <= int(j) < V:
                    p[i, int(j)] = 0.0
    return p.sum(0)


def topk_guesses(agg: torch.Tensor, k: int, tok=None) -> Tuple[List[int], List[str]]:
    """Top-k ids of a response-sum and their stripped decoded strings (`:147-149`); empty if the sum is 0."""
    if float(agg.sum()) <= 0:
        return [], []
    ids = torch.topk(agg, k).indices.tolist()
    return ids, ([tok.decode([i]).strip() for i in ids] if tok is not None else [])
