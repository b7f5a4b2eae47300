"""PyTorch reference implementations of every kernel in ``csrc/``.

They define the semantics (including the bf16 rounding points) that the HIP
kernels are tested against, and they are the execution path for CPU tensors
(unit tests, the GPT-2/tiny CPU plumbing configs).  They are deliberately
plain: readability over speed.
"""
from __future__ import annotations

import math
from typing import Optional

import numpy as np
import torch
import torch.nn.functional as F

BF16 = torch.bfloat16


def rbf(x: torch.Tensor) -> torch.Tensor:
    """Round an fp32 tensor through bf16 (a bf16-typed PyTorch intermediate)."""
    return x.to(BF16).float()


def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    xf = x.float()
    r = torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    return (xf * r * (1.0 + w.float())).to(x.dtype)


def add_rmsnorm2(h: torch.Tensor, o: torch.Tensor, w_post: torch.Tensor, w_next: torch.Tensor, eps: float) -> torch.Tensor:
    """In place: h <- h + norm(o, w_post); returns norm(h, w_next)."""
    h.copy_((h.float() + rmsnorm(o, w_post, eps).float()).to(h.dtype))
    return rmsnorm(h, w_next, eps)


def embed_rmsnorm(ids: torch.Tensor, E: torch.Tensor, w: torch.Tensor, scale: float, eps: float):
    idx = ids.long().clamp(0, E.shape[0] - 1)
    h = (E[idx].float() * rbf(torch.tensor(scale))).to(E.dtype)
    return h, rmsnorm(h, w, eps)


def rope_tables(head_dim: int, max_pos: int, theta: float, device=None):
    """fp32 cos/sin tables [max_pos, head_dim/2], computed the way transformers' default RoPE does."""
    inv_freq = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.int64).float() / head_dim))
    pos = torch.arange(max_pos, dtype=torch.float32)
    freqs = torch.outer(pos, inv_freq)
    return freqs.cos().to(device), freqs.sin().to(device)


def capture_rows(store: torch.Tensor, h: torch.Tensor, pos: torch.Tensor, slot: torch.Tensor, B: int, T: int) -> None:
    """Reference of ``ops.capture_rows`` (index_copy into ``store`` viewed as rows)."""
    S1 = store.shape[1]
    p = pos.reshape(B, T).long()
    pp = torch.where((p >= 0) & (p < S1 - 1), p, torch.full_like(p, S1 - 1))
    idx = (slot.reshape(-1)[:B].view(B, 1).long() * S1 + pp).view(-1)
    store.view(-1, h.shape[-1]).index_copy_(0, idx, h.reshape(-1, h.shape[-1]))


def decode_pre(step_idx: torch.Tensor, tf_tgt: torch.Tensor, tf_step: torch.Tensor, nb: int) -> None:
    """Reference of ``ops.decode_pre``: ``tf_step[r] = tf_tgt[r, min(step_idx[r], W - 1)]`` for ``r < nb``."""
    col = torch.clamp(step_idx[:nb].view(-1, 1), max=tf_tgt.shape[1] - 1)
    torch.gather(tf_tgt[:nb], 1, col, out=tf_step[:nb].view(-1, 1))


def decode_post(nxt, nll, tf_nll, done, step_idx, out_tok, out_nll, out_tf_nll, stop, tok, pos, nb: int,
                pad: int) -> None:
    """Reference of ``ops.decode_post`` (rows ``< nb``): the step's token (``pad`` once done) and NLLs into output
    column ``min(step_idx, W - 1)``, ``done |= token in stop``, next token / position + 1 / column + 1."""
    col = torch.clamp(step_idx[:nb].view(-1, 1), max=out_tok.shape[1] - 1)
    d = done[:nb]
    n = torch.where(d, torch.full_like(nxt[:nb], pad), nxt[:nb])
    out_tok[:nb].scatter_(1, col, n.view(-1, 1))
    out_nll[:nb].scatter_(1, col, nll[:nb].view(-1, 1))
    out_tf_nll[:nb].scatter_(1, col, tf_nll[:nb].view(-1, 1))
    d |= (n.view(-1, 1) == stop.view(1, -1)).any(-1)
    tok[:nb].copy_(n.view(-1, 1))
    pos[:nb].add_(1)
    step_idx[:nb].add_(1)


def share_lo_gather(rep, U, tok, pos, slot, s_tok, s_pos, s_slot, kp_slot, kp_len_lo, l_slot, l_len_lo, nb: int,
                    S: int) -> None:
    """Reference of ``ops.share_lo_gather``: lo row ``i < nb`` takes token / slot (and shared-prefix slot / length)
    of its representative ``rep[i]``; its position too when ``i < U``, else ``S`` (parked)."""
    r = rep[:nb]
    valid = torch.arange(nb, device=rep.device) < U
    s_tok[:nb].copy_(tok.index_select(0, r))
    s_pos[:nb].copy_(torch.where(valid.view(-1, 1), pos.index_select(0, r), S))
    s_slot[:nb].copy_(slot.index_select(0, r))
    if kp_slot is not None:
        l_slot[:nb].copy_(kp_slot.index_select(0, r))
        l_len_lo[:nb].copy_(kp_len_lo.index_select(0, r))


def kv_fanout(kc: torch.Tensor, vc: torch.Tensor, src_row: torch.Tensor, slot: torch.Tensor, pos: torch.Tensor,
              nlayers: int) -> None:
    """Reference of ``ops.kv_fanout``: ``kc/vc[l, slot[r], :, pos[r]] = kc/vc[l, slot[s], :, pos[s]]`` for
    ``l < nlayers`` and every row ``r`` with ``s = src_row[r] >= 0, s != r`` (both positions in the cache)."""
    S = kc.shape[3]
    M = src_row.numel()
    s = src_row.view(-1).long().cpu()
    r = torch.arange(M)
    s0 = s.clamp(min=0)
    p = pos.view(-1)[:M].long().cpu()
    ok = (s >= 0) & (s != r) & (p >= 0) & (p < S) & (p[s0] >= 0) & (p[s0] < S)
    idx = r[ok]
    if idx.numel() == 0 or nlayers <= 0:
        return
    sl = slot.view(-1).long().cpu()
    src = s0[idx]
    ds, dp, ss, sp = sl[idx], p[idx], sl[src], p[src]
    for c in (kc, vc):
        dev = c.device
        c[:nlayers, ds.to(dev), :, dp.to(dev)] = c[:nlayers, ss.to(dev), :, sp.to(dev)]


def rope_qkv_cache(qkv: torch.Tensor, pos: torch.Tensor, slot_of_row: torch.Tensor, cos_t: torch.Tensor,
                   sin_t: torch.Tensor, kc: torch.Tensor, vc: torch.Tensor, Hq: int, Hkv: int, HD: int) -> torch.Tensor:
    M = pos.numel()
    S = kc.shape[2]
    x = qkv.view(M, Hq + 2 * Hkv, HD).float()
    half = HD // 2
    p = pos.long()
    valid = p >= 0
    pc = p.clamp(0, cos_t.shape[0] - 1)
    c = rbf(cos_t[pc]).unsqueeze(1)
    s = rbf(sin_t[pc]).unsqueeze(1)
    rot_in = x[:, : Hq + Hkv]
    x1, x2 = rot_in[..., :half], rot_in[..., half:]
    o1 = rbf(rbf(x1 * c) + rbf(-x2 * s))
    o2 = rbf(rbf(x2 * c) + rbf(x1 * s))
    rot = torch.cat([o1, o2], -1)
    q = rot[:, :Hq].to(BF16)
    q[~valid] = 0
    k = rot[:, Hq:].to(BF16)
    v = x[:, Hq + Hkv:].to(BF16)
    ok = valid & (p < S)
    for m in torch.nonzero(ok).flatten().tolist():
        kc[int(slot_of_row[m]), :, int(p[m])] = k[m]
        vc[int(slot_of_row[m]), :, int(p[m])] = v[m]
    return q


def attention(q: torch.Tensor, kc: torch.Tensor, vc: torch.Tensor, pos: torch.Tensor, slot: torch.Tensor,
              B: int, T: int, scale: float, softcap: float, window: int, prefix=None) -> torch.Tensor:
    """q [B*T, Hq, HD]; cache [slots, Hkv, S, HD]; returns [B*T, Hq*HD] bf16.  ``prefix = (pk, pv, pslot,
    plen)``: sequence ``b`` reads keys ``[0, plen[b])`` from slot ``pslot[b]`` of ``pk/pv`` instead."""
    Hkv, S, HD = kc.shape[1], kc.shape[2], kc.shape[3]
    Hq = q.numel() // (B * T * HD)
    G = Hq // Hkv
    out = torch.zeros(B * T, Hq, HD, dtype=BF16, device=q.device)
    qv = q.view(B, T, Hq, HD)
    pv = pos.view(B, T).long()
    keys = torch.arange(S, device=q.device)
    for b in range(B):
        pb = pv[b]
        if (pb >= 0).sum() == 0:
            continue
        kmax = int(pb.max())
        K = kc[int(slot[b]), :, : kmax + 1].float()     # [Hkv, n, HD]
        V = vc[int(slot[b]), :, : kmax + 1].float()
        if prefix is not None:
            pk, pvc, ps, pl = prefix
            n = min(int(pl[b]), kmax + 1)
            if n > 0:
                K = K.clone()
                V = V.clone()
                K[:, :n] = pk[int(ps[b]), :, :n].float()
                V[:, :n] = pvc[int(ps[b]), :, :n].float()
        Kq = K.repeat_interleave(G, 0)                  # [Hq, n, HD]
        Vq = V.repeat_interleave(G, 0)
        s = torch.einsum("thd,hnd->htn", qv[b].float(), Kq) * scale
        if softcap > 0:
            s = torch.tanh(s / softcap) * softcap
        kk = keys[: kmax + 1]
        ok = (kk[None, :] <= pb[:, None]) & (pb[:, None] >= 0)
        if window > 0:
            ok &= (pb[:, None] - kk[None, :]) < window
        s = s.masked_fill(~ok[None], float("-inf"))
        m = s.amax(-1, keepdim=True)
        m = torch.where(torch.isinf(m), torch.zeros_like(m), m)
        p = rbf(torch.exp(s - m))
        l = p.sum(-1, keepdim=True)
        o = torch.einsum("htn,hnd->thd", p, Vq) / l.transpose(0, 1).clamp_min(1e-30)
        o = torch.where((pb >= 0)[:, None, None], o, torch.zeros_like(o))
        out.view(B, T, Hq, HD)[b] = o.to(BF16)
    return out.view(B * T, Hq * HD)


def geglu(gu: torch.Tensor) -> torch.Tensor:
    Fh = gu.shape[-1] // 2
    g, u = gu[..., :Fh], gu[..., Fh:]
    return (rbf(F.gelu(g.float(), approximate="tanh")) * u.float()).to(BF16)


def softcap_bf16(x: torch.Tensor, cap: float) -> torch.Tensor:
    """transformers' bf16 final-softcap chain: logits / cap ; tanh ; * cap (each rounded)."""
    return rbf(rbf(torch.tanh(rbf(x.float() / cap))) * cap)


def argmax_rows(logits: torch.Tensor, cap: float) -> torch.Tensor:
    x = logits.float()
    if cap > 0:
        x = softcap_bf16(x, cap)
    return torch.argmax(x, dim=-1).to(torch.int32)


def _capped(x: torch.Tensor, cap: float, emulate_bf16: bool) -> torch.Tensor:
    x = x.float()
    if cap > 0:
        x = softcap_bf16(x, cap) if emulate_bf16 else torch.tanh(x / cap) * cap
    return x


def row_lse(logits: torch.Tensor, cap: float = 0.0, emulate_bf16: bool = False) -> torch.Tensor:
    return torch.logsumexp(_capped(logits, cap, emulate_bf16), dim=-1)


def gather_probs(logits: torch.Tensor, lse: torch.Tensor, ids: torch.Tensor, round_bf16: bool = False) -> torch.Tensor:
    V = logits.shape[-1]
    R = logits.numel() // V
    lg = logits.reshape(R, V).float()
    idv = ids.reshape(R, -1).long()
    ok = (idv >= 0) & (idv < V)
    z = torch.gather(lg, 1, idv.clamp(0, V - 1))
    p = torch.exp(z - lse.reshape(R, 1))
    if round_bf16:
        p = rbf(p)
    return torch.where(ok, p, torch.zeros_like(p))


def lens_colsum(logits: torch.Tensor, lse: torch.Tensor, mask: Optional[torch.Tensor], excl: torch.Tensor, B: int,
                T: int, acc: Optional[torch.Tensor] = None, round_bf16: bool = False,
                offs: Optional[torch.Tensor] = None, with_cum: bool = False):
    """Returns the per-sequence sums ``[B, V]`` — plus, with ``with_cum``, ``(sums, cum [B, T+1, V])``."""
    V = logits.shape[-1]
    R = logits.numel() // V
    p = torch.exp(logits.reshape(R, V).float() - lse.reshape(R, 1))
    if round_bf16:
        p = rbf(p)
    ex = excl.reshape(R, 2).long()
    rows = torch.arange(R, device=p.device)
    for j in range(2):
        e = ex[:, j]
        ok = (e >= 0) & (e < V)
        p[rows[ok], e[ok]] = 0.0
    if mask is not None:
        p = p * mask.reshape(R, 1).float()
    cum = None
    if offs is not None:
        o = offs.tolist()
        s = torch.stack([p[o[b]:o[b + 1]].sum(0) for b in range(B)]) if B else p.new_zeros(0, V)
    else:
        s = p.view(B, T, V).sum(1)
        if with_cum:
            cum = torch.cat([p.new_zeros(B, 1, V), torch.cumsum(p.view(B, T, V), 1)], 1)
    if acc is not None:
        acc.add_(s)
        s = acc
    return (s, cum) if (with_cum or offs is not None) else s


def topk_rows(x: torch.Tensor, k: int):
    """Top-k per row; ties resolved towards the lower index (stable)."""
    V = x.shape[-1]
    xs = x.reshape(-1, V)
    vals, idx = torch.sort(xs, dim=-1, descending=True, stable=True)
    return vals[:, :k].contiguous(), idx[:, :k].to(torch.int32).contiguous()


def xent_rows(logits: torch.Tensor, tgt: torch.Tensor, cap: float, emulate_bf16: bool = True) -> torch.Tensor:
    V = logits.shape[-1]
    z = _capped(logits.reshape(-1, V), cap, emulate_bf16)
    t = tgt.reshape(-1).long()
    ok = (t >= 0) & (t < V)
    lse = torch.logsumexp(z, -1)
    zt = torch.gather(z, 1, t.clamp(0, V - 1)[:, None])[:, 0]
    return torch.where(ok, lse - zt, torch.zeros_like(lse))


def gemm_nt(A: torch.Tensor, W: torch.Tensor, epi: int, bias: Optional[torch.Tensor] = None,
            thr: Optional[torch.Tensor] = None) -> torch.Tensor:
    K = A.shape[-1]
    c = A.reshape(-1, K).float() @ W.float().t()
    if epi == 0:
        return c.to(BF16)
    if epi == 1:
        return c
    if bias is not None:
        c = c + bias.float()
    th = thr.float() if thr is not None else torch.zeros((), device=c.device)
    return torch.where(c > th, c, torch.zeros_like(c))


def lowrank_edit(h: torch.Tensor, apply: torch.Tensor, idx: torch.Tensor, cnt: torch.Tensor, E: torch.Tensor,
                 Dm: torch.Tensor, bias=None, thr=None, pre_bias=None, alpha: float = 1.0,
                 w_next: Optional[torch.Tensor] = None, eps: float = 1e-6, x_next: Optional[torch.Tensor] = None,
                 coef_out: Optional[torch.Tensor] = None) -> None:
    """In place on h (and x_next rows that were edited); rows whose coefficients are all zero are left
    untouched."""
    D = h.shape[-1]
    hv = h.view(-1, D)
    M = hv.shape[0]
    mmax = idx.numel() // M
    iv = idx.view(M, mmax)
    for r in torch.nonzero(apply.view(-1).bool()).flatten().tolist():
        m = max(0, min(int(cnt.view(-1)[r]), mmax, 256))
        sel = iv[r, :m].long()
        x = hv[r].float()
        xb = x - pre_bias.float() if pre_bias is not None else x
        pre = E[sel].float() @ xb
        if bias is not None:
            pre = pre + bias.float()[sel]
        a = torch.where(pre > thr.float()[sel], pre, torch.zeros_like(pre)) if thr is not None else pre
        if coef_out is not None:
            coef_out.view(M, mmax)[r, :m] = a
        if not bool(((alpha * a) != 0).any()):
            continue                      # all-zero edit: an exact no-op (h and x_next untouched)
        newx = rbf(x - (alpha * a) @ Dm[sel].float())
        hv[r] = newx.to(h.dtype)
        if x_next is not None and w_next is not None:
            x_next.view(-1, D)[r] = rmsnorm(hv[r:r + 1], w_next, eps)[0]


def sae_decode_sparse(acts: torch.Tensor, Wdec: torch.Tensor, b_dec: Optional[torch.Tensor] = None) -> torch.Tensor:
    out = acts.float() @ Wdec.float()
    if b_dec is not None:
        out = out + b_dec.float()
    return out


def latent_score(acts: torch.Tensor, p: torch.Tensor, spike: torch.Tensor, seg: torch.Tensor):
    """Returns (score [G, L], spike_mean [G, L], corr [G, L])."""
    L = acts.shape[-1]
    segs = seg.tolist()
    G = len(segs) - 1
    score = torch.zeros(G, L, device=acts.device)
    sm = torch.zeros(G, L, device=acts.device)
    cr = torch.zeros(G, L, device=acts.device)
    for g in range(G):
        a = acts[segs[g]:segs[g + 1]].double()
        pv = p[segs[g]:segs[g + 1]].double()
        sp = spike[segs[g]:segs[g + 1]].bool()
        n = a.shape[0]
        if n > 1:
            ac = a - a.mean(0)
            pc = pv - pv.mean()
            va = (ac * ac).sum(0)
            vp = (pc * pc).sum()
            cov = (ac * pc[:, None]).sum(0)
            c = torch.where((va > 1e-12) & (vp > 1e-20), cov / torch.sqrt(va * vp).clamp_min(1e-300),
                            torch.zeros_like(cov))
        else:
            c = torch.zeros(L, dtype=torch.float64, device=acts.device)
        m = a[sp].mean(0) if sp.any() else torch.zeros(L, dtype=torch.float64, device=acts.device)
        score[g] = (m * c.clamp_min(0)).float()
        sm[g] = m.float()
        cr[g] = c.float()
    return score, sm, cr


def vp_head_merge(st: torch.Tensor, tgt, V: int):
    """Reference of ``ops.vp_head_merge`` (rank order; on equal best logits the lower rank = lower vocab id)."""
    tp, R = st.shape[0], st.shape[1]
    lse = vp_lse_merge(st[:, :, 0])
    best = st[0, :, 1].clone()
    idx = st[0, :, 2].clone()
    for k in range(1, tp):
        better = st[k, :, 1] > best
        best = torch.where(better, st[k, :, 1], best)
        idx = torch.where(better, st[k, :, 2], idx)
    nll_tgt = None
    if tgt is not None:
        t = tgt.view(-1).long()
        tl = st[:, :, 3].max(0).values
        nll_tgt = torch.where((t >= 0) & (t < V), lse - tl, torch.zeros_like(lse))
    return idx.to(torch.int32), lse - best, nll_tgt


def vp_lse_merge(lse_parts: torch.Tensor) -> torch.Tensor:
    """Reference of ``ops.vp_lse_merge``: running (max, sum) merge of the parts in rank order."""
    x = lse_parts.float()
    m = x[0].clone()
    s = torch.ones_like(m)
    for k in range(1, x.shape[0]):
        m2 = torch.maximum(m, x[k])
        s = s * torch.exp(m - m2) + torch.exp(x[k] - m2)
        m = m2
    return m + torch.log(s)


def vp_topk_merge(vals: torch.Tensor, ids: torch.Tensor):
    """Reference of ``ops.vp_topk_merge``: top-k of every rank's candidates, descending, ties to the lower id."""
    tp, n, k = vals.shape
    v = vals.permute(1, 0, 2).reshape(n, tp * k).float()
    i = ids.permute(1, 0, 2).reshape(n, tp * k).long()
    o = torch.argsort(i, dim=1, stable=True)                    # ids ascending, then a stable sort by value
    v, i = v.gather(1, o), i.gather(1, o)
    o = torch.argsort(v, dim=1, descending=True, stable=True)
    return v.gather(1, o)[:, :k].contiguous(), i.gather(1, o)[:, :k].to(torch.int32).contiguous()


def lora_t(x, a_all, adapter, nsr: int, nr: int, r: int):
    """Masked LoRA down-projection (ops.lora_t): fp32 ``x @ a_all^T`` rounded to bf16, kept on the row's adapter's
    columns (``c < nsr`` and ``(c % nr) // r == adapter``), 0 elsewhere."""
    t = (x.float() @ a_all.float().t()).to(torch.bfloat16)
    c = torch.arange(a_all.shape[0], device=x.device)
    keep = (c[None, :] < nsr) & (((c % nr) // r)[None, :] == adapter.long().view(-1, 1)) & (adapter.view(-1, 1) >= 0)
    return torch.where(keep, t, torch.zeros_like(t))


_RB_M1, _RB_M2 = np.uint64(0xBF58476D1CE4E5B9), np.uint64(0x94D049BB133111EB)
_RB_G, _RB_X = np.uint64(0x9E3779B97F4A7C15), np.uint64(0xD1B54A32D192ED03)


def _rb_mix64(z):
    z = (z ^ (z >> np.uint64(30))) * _RB_M1
    z = (z ^ (z >> np.uint64(27))) * _RB_M2
    return z ^ (z >> np.uint64(31))


def random_basis(D: int, r: int, seed: int) -> np.ndarray:
    """csrc/basis.hip in numpy: ``[r, D]`` fp32 orthonormal rows.  Entry ``(j, d)`` of the Gaussian is Box-Muller of
    two splitmix64 hashes of ``seed * phi + (j << 32 | d)``; row ``j`` is orthonormalised by classical Gram-Schmidt
    applied twice (64 earlier rows per chunk), in fp64, against the fp32-rounded rows before it.  (The kernel's dot products sum in another order: rows agree to
    fp32 rounding, not bit for bit.)"""
    j = np.arange(r, dtype=np.uint64)[:, None]
    d = np.arange(D, dtype=np.uint64)[None, :]
    with np.errstate(over="ignore"):
        key = np.uint64(int(seed) & ((1 << 64) - 1)) * _RB_G + ((j << np.uint64(32)) | d)
        a, b = _rb_mix64(key), _rb_mix64(key ^ _RB_X)
    u1 = ((a >> np.uint64(11)).astype(np.float64) + 1.0) * 2.0 ** -53
    u2 = (b >> np.uint64(11)).astype(np.float64) * 2.0 ** -53
    G = np.sqrt(-2.0 * np.log(u1)) * np.cos(6.283185307179586 * u2)
    Q = np.zeros((r, D), np.float32)
    Qd = np.zeros((r, D), np.float64)
    for jj in range(r):
        v = G[jj]
        for _ in range(2):                       # classical Gram-Schmidt twice, 64 earlier rows per chunk
            for q0 in range(0, jj, 64):
                Qc = Qd[q0:min(jj, q0 + 64)]
                v = v - (Qc @ v) @ Qc
        Q[jj] = (v * (1.0 / np.sqrt(v @ v))).astype(np.float32)
        Qd[jj] = Q[jj]
    return Q
