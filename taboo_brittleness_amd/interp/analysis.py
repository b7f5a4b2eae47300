"""Spike tokens, latent secret scores, secret subspaces and random controls
(EP:116-124, 144-150).

All randomness is keyed by the sweep cell (never by the rank), so a sweep
produces identical cells on 1 or 8 GPUs.
"""
from __future__ import annotations

import hashlib
from typing import List, Optional, Sequence

import numpy as np
import torch

from .. import ops


def cell_seed(*key) -> int:
    """Stable 63-bit seed from an arbitrary key tuple (independent of PYTHONHASHSEED and world size)."""
    h = hashlib.blake2b(repr(key).encode(), digest_size=8).digest()
    return int.from_bytes(h, "little") & ((1 << 63) - 1)


def select_spikes(p_secret: np.ndarray, resp_ids: Sequence[int], secret_ids: Sequence[int], k: int = 4) -> List[int]:
    """Top-``k`` response positions by lens secret probability (EP:116).

    Positions whose token *is* the secret are excluded; ties go to the earlier
    position; at least one spike whenever the response is non-empty.
    """
    n = len(p_secret)
    if n == 0:
        return []
    sec = set(int(s) for s in secret_ids)
    cand = [i for i in range(n) if i >= len(resp_ids) or int(resp_ids[i]) not in sec]
    if not cand:
        cand = list(range(n))
    cand.sort(key=lambda i: (-float(p_secret[i]), i))
    return sorted(cand[: max(1, k)])


@torch.no_grad()
def latent_scores(sae, resid_rows: torch.Tensor, p_secret: torch.Tensor, spike_rel: Sequence[Sequence[int]],
                  seg: Sequence[int]) -> torch.Tensor:
    """``score_j = mean_{t∈spikes} a_j(t) · max(0, corr_t(a_j(t), p_secret(t)))`` per prompt segment (EP:118-124).

    ``resid_rows``: response residuals of several prompts concatenated; ``seg``:
    segment boundaries (len G+1); ``spike_rel[g]``: spike indices within segment g.
    Returns ``[G, d_sae]`` fp32 on the SAE's device.
    """
    dev = sae.device
    acts = sae.encode(resid_rows.to(dev))
    spike = torch.zeros(acts.shape[0], dtype=torch.uint8)
    for g, sp in enumerate(spike_rel):
        for i in sp:
            spike[seg[g] + i] = 1
    score, _, _ = ops.latent_score(acts.contiguous(), p_secret.to(dev).float().contiguous(), spike.to(dev),
                                   torch.tensor(list(seg), dtype=torch.int32, device=dev))
    return score


def top_latents_from_scores(score: torch.Tensor, m: int) -> List[int]:
    vals, idx = ops.topk_rows(score.view(1, -1).float().contiguous(), m)
    return [int(i) for i, v in zip(idx[0].tolist(), vals[0].tolist())]


def top_latents_batch(scores: torch.Tensor, m: int) -> List[List[int]]:
    """Row-wise :func:`top_latents_from_scores` for ``scores [G, L]`` in one kernel launch."""
    if scores.shape[0] == 0:
        return []
    _, idx = ops.topk_rows(scores.float().contiguous(), m)
    return idx.cpu().tolist()


_M1, _M2, _GOLD = np.uint64(0xBF58476D1CE4E5B9), np.uint64(0x94D049BB133111EB), np.uint64(0x9E3779B97F4A7C15)


def _mix64(x: np.ndarray) -> np.ndarray:
    """splitmix64 finaliser (vectorised, wrap-around uint64 arithmetic)."""
    x = x.astype(np.uint64, copy=True)
    with np.errstate(over="ignore"):
        x ^= x >> np.uint64(30)
        x *= _M1
        x ^= x >> np.uint64(27)
        x *= _M2
        x ^= x >> np.uint64(31)
    return x


def _keys(seeds: np.ndarray, ids: np.ndarray, salt: int) -> np.ndarray:
    with np.errstate(over="ignore"):
        s = _mix64(seeds.astype(np.uint64) + np.uint64(salt) * _GOLD)
        return _mix64(s[:, None] ^ (ids.astype(np.uint64)[None, :] * _GOLD))


def _ranked_pool(sd: np.ndarray, pl: np.ndarray, mmax: int, excludes: Sequence[Sequence[int]]) -> List[List[int]]:
    """Exhaustive form: every pool latent ranked by a per-seed hash, excluded ids dropped (small pools)."""
    n = sd.size
    k = _keys(sd, pl, 1)
    BIG = np.uint64(0xFFFFFFFFFFFFFFFF)
    for i, ex in enumerate(excludes):
        if len(ex):
            k[i, np.isin(pl, np.asarray(list(ex), dtype=np.int64))] = BIG
    take = min(mmax, pl.size)
    if take < pl.size:
        part = np.argpartition(k, take - 1, axis=1)[:, :take]
        order = np.take_along_axis(part, np.argsort(np.take_along_axis(k, part, 1), axis=1, kind="stable"), 1)
    else:
        order = np.argsort(k, axis=1, kind="stable")
    picked = pl[order]
    valid = np.take_along_axis(k, order, 1) != BIG
    return [picked[i][valid[i]].tolist() for i in range(n)]


def random_latents_batch(d_sae: int, budgets: Sequence[int], seeds: Sequence[int],
                         excludes: Sequence[Sequence[int]], pool: Optional[Sequence[int]] = None) -> List[List[int]]:
    """Random latent sets for many cells of one prompt at once (EP:128).

    Each cell's set is a pure function of its seed: a uniform sample without replacement from ``pool``
    (the activation-matched control: latents active at the spike positions) minus the cell's excluded
    ids, drawn as a counter-based hash stream (draw ``j`` = ``pool[h(seed, j) mod |pool|]``, repeats and
    excluded ids rejected, first ``m`` kept).  Vectorised over cells with ``O(m)`` hashes per cell, so
    a 5940-cell step costs milliseconds of host time (the prefetch thread that builds it shares the GIL
    with the launch thread).  Small pools, or a row the stream leaves short, use the exhaustive ranking;
    if the pool itself runs short the rest is filled from all ``d_sae`` latents ranked by a second hash.
    """
    n = len(budgets)
    out: List[List[int]] = [[] for _ in range(n)]
    if n == 0:
        return out
    sd = np.asarray([int(x) & ((1 << 63) - 1) for x in seeds], dtype=np.uint64)
    bud = np.asarray([int(m) for m in budgets], dtype=np.int64)
    mmax = int(bud.max())
    if pool is not None and len(pool):
        pl = np.unique(np.asarray(pool if isinstance(pool, np.ndarray) else list(pool), dtype=np.int64))
        N = pl.size
        # every decision below is per row (its own budget), so a cell's set never depends on which
        # other cells share the batch: small pool for this budget -> exhaustive ranking; otherwise
        # the first 2*m+8 stream draws, falling back to the ranking if they leave the row short
        ranked = N <= 4 * bud
        redo_rows = np.nonzero(ranked)[0]
        stream_rows = np.nonzero(~ranked)[0]
        if stream_rows.size:
            sr = stream_rows
            rlen = 2 * bud[sr] + 8
            R = int(rlen.max())
            with np.errstate(over="ignore"):
                v = pl[(_keys(sd[sr], np.arange(R, dtype=np.int64), 3) % np.uint64(N)).astype(np.int64)]
            # first occurrence of each value within its row (stable sort keeps draw order among repeats)
            o = np.argsort(v, axis=1, kind="stable")
            vs = np.take_along_axis(v, o, 1)
            first_s = np.ones_like(vs, dtype=bool)
            first_s[:, 1:] = vs[:, 1:] != vs[:, :-1]
            ok = np.empty_like(first_s)
            np.put_along_axis(ok, o, first_s, 1)
            ok &= np.arange(R, dtype=np.int64)[None, :] < rlen[:, None]
            ex_rows = [np.full(len(excludes[i]), k, dtype=np.int64) for k, i in enumerate(sr) if len(excludes[i])]
            if ex_rows:
                ex_key = np.concatenate(ex_rows) * d_sae + np.concatenate(
                    [np.asarray(list(excludes[i]), dtype=np.int64) for i in sr if len(excludes[i])])
                ok &= ~np.isin(np.arange(sr.size, dtype=np.int64)[:, None] * d_sae + v, ex_key)
            rank = np.cumsum(ok, axis=1)
            keep = ok & (rank <= bud[sr][:, None])
            short = rank[:, -1] < bud[sr]
            for k, i in enumerate(sr.tolist()):
                out[i] = v[k][keep[k]].tolist()
            redo_rows = np.concatenate([redo_rows, sr[short]])
        if redo_rows.size:
            redo = _ranked_pool(sd[redo_rows], pl, int(bud[redo_rows].max()), [excludes[i] for i in redo_rows])
            for i, r in zip(redo_rows.tolist(), redo):
                out[i] = r
        for i in range(n):
            del out[i][int(bud[i]):]
    for i in range(n):
        m = int(bud[i])
        if len(out[i]) < m:
            allk = _keys(sd[i: i + 1], np.arange(d_sae, dtype=np.int64), 2)[0]
            chosen = set(out[i]) | set(int(e) for e in excludes[i])
            for j in np.argsort(allk, kind="stable"):
                if int(j) not in chosen:
                    out[i].append(int(j))
                    if len(out[i]) == m:
                        break
    return out


def random_latents(d_sae: int, m: int, seed: int, exclude: Sequence[int] = (), pool: Optional[Sequence[int]] = None) -> List[int]:
    """``m`` random latents for one cell (see :func:`random_latents_batch`)."""
    return random_latents_batch(d_sae, [m], [seed], [exclude], pool)[0]


@torch.no_grad()
def secret_subspace(vectors: torch.Tensor, r: int) -> torch.Tensor:
    """Top-``r`` principal directions of mean-centred spike residuals (EP:144-146). Returns ``[r, D]`` fp32 orthonormal rows."""
    X = vectors.double()
    X = X - X.mean(0, keepdim=True)
    n = X.shape[0]
    if n >= 2:
        # Gram trick: N x N eigenproblem (N = pooled spike count << D), in fp64 on the vectors' device: one host sync
        # (the numerical rank) instead of a device -> host copy of X per direction
        evals, evecs = torch.linalg.eigh(X @ X.t())
        evals, order = torch.sort(evals, descending=True)
        thr = 1e-9 * torch.clamp(evals[:1], min=1e-30)
        k = min(r, int((evals > thr).sum()))        # the leading eigenvalues above the threshold
        U = ((X.t() @ evecs[:, order[:k]]) / evals[:k].sqrt()).t()
    else:
        U = torch.zeros(0, X.shape[1], dtype=torch.float64, device=X.device)
    if U.shape[0] < r:   # pad a rank-deficient basis with random orthogonal directions
        extra = random_subspace(X.shape[1], r - U.shape[0], seed=cell_seed("pad", n, r)).double().to(X.device)
        U = torch.cat([U, extra], 0)
    Q, _ = torch.linalg.qr(U.t())
    return Q.t()[:r].float().contiguous()


def random_subspace(D: int, r: int, seed: int, device=None) -> torch.Tensor:
    """``r`` random orthonormal directions of R^D (EP:150: a Gaussian ``D x r`` matrix, orthonormalised) as ``[r, D]``
    fp32 rows; a pure function of ``(D, r, seed)``, the same on every device and rank.  The entries are a counter hash
    of ``(seed, row, column)`` (Box-Muller), orthonormalised by Gram-Schmidt (classical, twice) in fp64 (ops.reference
    .random_basis); on a GPU ``device`` the rows come from the HIP kernel of the same algorithm (csrc/basis.hip) --
    the projection sweep draws its thousands of random-control bases that way, straight into its edit plan."""
    r, D = int(r), int(D)
    if device is not None and torch.device(device).type == "cuda":
        out = torch.empty(r, D, dtype=torch.float32, device=device)
        dev = out.device
        ops.random_basis(torch.tensor([int(seed)], dtype=torch.int64).to(dev),
                         torch.tensor([r], dtype=torch.int32).to(dev), torch.zeros(1, dtype=torch.int64, device=dev), out)
        return out
    from ..ops import reference as R

    return torch.from_numpy(R.random_basis(D, r, int(seed)))
