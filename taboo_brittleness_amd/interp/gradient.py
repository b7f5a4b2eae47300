"""Gradient secret directions — the design doc's alternative to the PCA subspace (EP:146: "derive
directions via gradients: e.g. find the direction in residual space that, if added, most increases the
secret-token logit").

Two flavours, selected by ``intervention.subspace``:

* ``grad_lens``: the gradient of the secret token's logit-lens logit ``(W_U norm_f(r))_s`` with respect to
  the hooked-layer residual ``r`` at each spike position — closed form through the final RMSNorm
  (``u = W_U[s] ⊙ (1 + w_f)``:  ``∂z/∂r = u / rms(r) − (u·r) r / (D rms(r)^3)``).  Cheap, no extra forward.
* ``grad_model``: the gradient of the model's own (pre-softcap) output logit of the secret token, summed over
  the spike positions, with respect to the hooked-layer residual at each spike position, back-propagated
  through blocks ``l+1 .. L-1`` (attention included, so later positions' logits count) by a float32,
  differentiable re-implementation of the block (:func:`tail_forward_fp32`; numerically the engine's
  forward up to its bf16 roundings — tested against it on CPU).  One forward + backward per pair.

Either way the pooled gradient vectors (unit-normalised) give the subspace as their top-``r`` right
singular vectors (uncentred: the mean gradient *is* the first direction), orthonormalised by QR.
"""
from __future__ import annotations

import math
from typing import Sequence

import torch
import torch.nn.functional as F


def _rms(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + eps) * (1.0 + w.float())


def tail_forward_fp32(model, h: torch.Tensor, start: int) -> torch.Tensor:
    """Blocks ``start .. L-1`` of a Gemma-2 ``model`` on ONE sequence in float32 with autograd, from the
    residual ``h [T, D]`` that enters block ``start`` (positions 0..T-1); returns the final-normed hidden
    state ``[T, D]`` (input of the unembedding)."""
    s = model.spec
    w = model.w
    T = h.shape[0]
    dev = h.device
    Hq, Hkv, HD = s.heads, s.kv_heads, s.head_dim
    G = Hq // Hkv
    pos = torch.arange(T, device=dev)
    c = model.cos_t[:T].float().to(dev).unsqueeze(1)             # [T, 1, HD/2]
    sn = model.sin_t[:T].float().to(dev).unsqueeze(1)
    half = HD // 2
    scale = s.query_pre_attn_scalar ** -0.5
    causal = pos[None, :] <= pos[:, None]

    def rope(x):
        x1, x2 = x[..., :half], x[..., half:]
        return torch.cat([x1 * c - x2 * sn, x2 * c + x1 * sn], -1)

    bw = getattr(model, "base_weight", None)
    for l in range(start, s.layers):
        L = w.layers[l]
        wq, wo, wgu, wdn = ((bw(l, k) for k in ("qkv", "o", "gu", "down")) if bw is not None
                            else (L.wqkv, L.wo, L.wgu, L.wdown))
        x = _rms(h, L.ln_in, s.eps)
        qkv = x @ wq.float().t()
        q = rope(qkv[:, : Hq * HD].view(T, Hq, HD))
        k = rope(qkv[:, Hq * HD:(Hq + Hkv) * HD].view(T, Hkv, HD))
        v = qkv[:, (Hq + Hkv) * HD:].view(T, Hkv, HD)
        k = k.repeat_interleave(G, dim=1)
        v = v.repeat_interleave(G, dim=1)
        sc = torch.einsum("thd,shd->hts", q, k) * scale
        if s.attn_softcap > 0:
            sc = torch.tanh(sc / s.attn_softcap) * s.attn_softcap
        mask = causal
        if s.is_sliding(l) and s.sliding_window > 0:
            mask = mask & (pos[:, None] - pos[None, :] < s.sliding_window)
        sc = sc.masked_fill(~mask[None], float("-inf"))
        att = torch.einsum("hts,shd->thd", torch.softmax(sc, -1), v).reshape(T, Hq * HD)
        h = h + _rms(att @ wo.float().t(), L.ln_post_attn, s.eps)
        x = _rms(h, L.ln_pre_ffn, s.eps)
        gu = x @ wgu.float().t()
        g, u = gu[:, : s.ffn], gu[:, s.ffn:]
        h = h + _rms((F.gelu(g, approximate="tanh") * u) @ wdn.float().t(), L.ln_post_ffn, s.eps)
    return _rms(h, w.norm_f, s.eps)


def model_gradients(model, h_seq: torch.Tensor, layer: int, spikes: Sequence[int],
                    secret_ids: Sequence[int]) -> torch.Tensor:
    """``[len(spikes), D]``: ∂ Σ_{t∈spikes} Σ_{s∈ids} z_s(t) / ∂h_t, with ``z`` the model's pre-softcap output
    logits and ``h_seq [T, D]`` the output of block ``layer`` (the hooked residual) for one sequence."""
    if not spikes or not secret_ids:
        return torch.zeros(0, h_seq.shape[1])
    with torch.enable_grad():
        h = h_seq.detach().float().clone().requires_grad_(True)
        xf = tail_forward_fp32(model, h, layer + 1)
        sp = torch.as_tensor(list(spikes), dtype=torch.long, device=h.device)
        ids = torch.as_tensor(list(secret_ids), dtype=torch.long, device=h.device)
        Wu = model.w.lm_head.index_select(0, ids).float()            # [n_ids, D]
        J = (xf.index_select(0, sp) @ Wu.t()).sum()
        (g,) = torch.autograd.grad(J, h)
    return g.index_select(0, sp).detach().float().cpu()


def lens_gradients(model, rows: torch.Tensor, secret_ids: Sequence[int]) -> torch.Tensor:
    """``[n, D]``: ∂ Σ_s (W_U norm_f(r))_s / ∂r for each residual row (closed form through the final norm)."""
    if rows.shape[0] == 0 or not secret_ids:
        return torch.zeros(0, rows.shape[1])
    r = rows.float()
    ids = torch.as_tensor(list(secret_ids), dtype=torch.long, device=r.device)
    u = model.w.lm_head.index_select(0, ids).float().sum(0) * (1.0 + model.w.norm_f.float())
    D = r.shape[1]
    ms = r.pow(2).mean(-1, keepdim=True) + model.spec.eps
    inv = torch.rsqrt(ms)
    g = u[None, :] * inv - (r @ u)[:, None] * r * inv.pow(3) / D
    return g.cpu()


@torch.no_grad()
def gradient_subspace(G: torch.Tensor, r: int, seed: int = 0) -> torch.Tensor:
    """Top-``r`` right singular vectors of the unit-normalised gradient rows ``G [n, D]`` (uncentred), as
    ``[r, D]`` fp32 orthonormal rows; padded with random orthogonal directions when ``rank(G) < r``."""
    from .analysis import random_subspace

    D = G.shape[1]
    X = G.double()
    X = X / X.norm(dim=1, keepdim=True).clamp_min(1e-30)
    if X.shape[0]:
        _, S, Vh = torch.linalg.svd(X, full_matrices=False)
        keep = S > 1e-9 * max(float(S.max()), 1e-30)
        U = Vh[keep][:r]
    else:
        U = torch.zeros(0, D, dtype=torch.float64)
    if U.shape[0] < r:
        U = torch.cat([U, random_subspace(D, r - U.shape[0], seed=seed).double()], 0)
    Q, _ = torch.linalg.qr(U.t())
    # QR may flip signs; keep the first direction aligned with the mean gradient (a removal is sign-free,
    # but a stable orientation makes bases comparable across runs)
    Q = Q.t()[:r]
    m = X.mean(0)
    if X.shape[0] and float(Q[0] @ m) < 0:
        Q[0] = -Q[0]
    return Q.float().contiguous()


def grad_norm_ratio(G: torch.Tensor) -> float:
    """Diagnostic: |mean of unit gradients| (1 = all spikes share one direction, ~1/sqrt(n) = unrelated)."""
    if G.shape[0] == 0:
        return math.nan
    X = G.double() / G.double().norm(dim=1, keepdim=True).clamp_min(1e-30)
    return float(X.mean(0).norm())
