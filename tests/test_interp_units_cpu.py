"""CPU unit tests for the intervention / analysis / statistics building blocks of the sweep
(EP:112-154), each checked against an independent plain-PyTorch / numpy
formula rather than the loop-form CPU references the HIP kernels are tested against:

* ``EditPlan`` / ``spike_mask`` row matching (padding, ``ALL_POSITIONS``);
* ``ops.lowrank_edit`` as the error-preserving SAE-latent ablation ``x - sum_j a_j W_dec[j]`` and as the
  projection-out ``x - U U^T x`` (only flagged rows change; the next block's norm input is refreshed);
* ``latent_scores`` = spike-mean activation x positive Pearson correlation with p(secret);
* ``secret_subspace`` / ``random_subspace`` (orthonormal, planted direction recovered, seeded);
* ``random_latents_batch`` (seeded per cell, budget / exclusions / pool respected, nested budgets);
* ``select_spikes``, ``cell_seed``, bootstrap CIs, feature-map inverse, atomic pair cache.
"""
import json
import os

import numpy as np
import pytest
import torch

from taboo_brittleness_amd import ops
from taboo_brittleness_amd.interp import analysis as A
from taboo_brittleness_amd.interp.edits import ALL_POSITIONS, EditPlan, spike_mask
from taboo_brittleness_amd.interp.feature_map import FEATURE_MAP, inverse_map, latents_to_word_guesses
from taboo_brittleness_amd.interp.sae import JumpReLUSAE
from taboo_brittleness_amd.metrics.bootstrap import bootstrap_ci, grouped_bootstrap_ci, summarize
from taboo_brittleness_amd.utils import io as tio


# ----------------------------------------------------------------------------- edit plans
def test_edit_plan_build_pads_and_codes():
    plan = EditPlan.build("cpu", spikes=[[3, 5], [], [7]], kinds=["sae", "none", "proj"], sel=[[1, 2, 3], [], [0]])
    assert plan.B == 3
    assert plan.spikes.tolist() == [[3, 5], [-1, -1], [7, -1]]
    assert plan.kind.tolist() == [1, 0, 2]
    assert plan.cnt.tolist() == [3, 0, 1]
    assert plan.idx[0].tolist() == [1, 2, 3] and plan.idx[2, 0].item() == 0
    capped = EditPlan.build("cpu", spikes=[[1, 2, 3]], kinds=["sae"], sel=[[4, 5, 6]], kmax=2, mmax=2)
    assert capped.spikes.tolist() == [[1, 2]] and capped.cnt.tolist() == [2]


def test_spike_mask_matches_positions_padding_and_all():
    B, T = 3, 4
    pos = torch.tensor([[0, 1, 2, 3], [5, 6, 7, 8], [0, 1, -1, -1]], dtype=torch.int32)
    spikes = torch.tensor([[1, 3], [9, -1], [ALL_POSITIONS, -1]], dtype=torch.int32)
    m = spike_mask(pos.view(-1), spikes, B, T).view(B, T)
    assert m.tolist() == [[False, True, False, True], [False, False, False, False], [True, True, False, False]]


# ----------------------------------------------------------------------------- low-rank edit kernel (CPU path)
def _rms(x, w, eps):
    xf = x.float()
    return xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * (1.0 + w.float())


def test_lowrank_edit_sae_ablation_formula():
    torch.manual_seed(0)
    D, L, M, m = 64, 256, 6, 5
    sae = JumpReLUSAE.random(D, L, seed=1, target_l0=40.0)
    sae.threshold = torch.full((L,), 0.05)
    h = (torch.randn(M, D) * 2).to(torch.bfloat16)
    h0 = h.clone()
    apply = torch.tensor([1, 0, 1, 1, 0, 1], dtype=torch.uint8)
    idx = torch.stack([torch.randperm(L)[:m] for _ in range(M)]).int()
    cnt = torch.tensor([5, 5, 3, 0, 5, 5], dtype=torch.int32)
    w_next = torch.randn(D) * 0.1
    x_next = torch.zeros(M, D, dtype=torch.bfloat16)
    ops.lowrank_edit(h, apply, idx, cnt, sae.W_encT, sae.W_dec, sae.b_enc, sae.threshold, None, 1.0, w_next, 1e-6,
                     x_next, None)
    for r in range(M):
        if not apply[r] or cnt[r] == 0:
            assert torch.equal(h[r], h0[r]), r
            continue
        sel = idx[r, : cnt[r]].long()
        x = h0[r].float()
        pre = sae.W_encT[sel].float() @ x + sae.b_enc[sel]
        a = torch.where(pre > sae.threshold[sel], pre, torch.zeros_like(pre))   # JumpReLU, strict
        if not bool((a != 0).any()):        # all-zero edit: an exact no-op, the next norm input is untouched
            assert torch.equal(h[r], h0[r]) and not bool(x_next[r].any()), r
            continue
        want = x - a @ sae.W_dec[sel].float()
        torch.testing.assert_close(h[r].float(), want, atol=0.05, rtol=0.02)
        torch.testing.assert_close(x_next[r].float(), _rms(h[r], w_next, 1e-6), atol=0.05, rtol=0.02)


def test_lowrank_edit_projection_out_removes_subspace():
    torch.manual_seed(1)
    D, r, M = 96, 4, 5
    U = A.random_subspace(D, r, seed=7)                       # [r, D] orthonormal rows
    h = torch.randn(M, D, dtype=torch.float32)
    h0 = h.clone()
    apply = torch.tensor([1, 1, 0, 1, 0], dtype=torch.uint8)
    idx = torch.arange(r, dtype=torch.int32).repeat(M, 1)
    cnt = torch.full((M,), r, dtype=torch.int32)
    ops.lowrank_edit(h, apply, idx, cnt, U, U)
    P = torch.eye(D) - U.t() @ U
    for i in range(M):
        if apply[i]:
            torch.testing.assert_close(h[i], P @ h0[i], atol=2e-2, rtol=1e-2)
            assert (U @ h[i]).abs().max() < 5e-2
        else:
            assert torch.equal(h[i], h0[i])


# ----------------------------------------------------------------------------- scores / subspaces / randomness
def test_latent_scores_spike_mean_times_positive_corr():
    torch.manual_seed(2)
    D, L = 32, 128
    sae = JumpReLUSAE.random(D, L, seed=3, target_l0=30.0)
    seg = [0, 7, 12]
    resid = torch.randn(12, D) * 3
    p = torch.rand(12)
    spikes = [[1, 4], [0, 3]]
    got = A.latent_scores(sae, resid, p, spikes, seg)
    acts = sae.encode(resid).double()
    for g in range(2):
        a = acts[seg[g]:seg[g + 1]]
        pv = p[seg[g]:seg[g + 1]].double()
        ac, pc = a - a.mean(0), pv - pv.mean()
        den = torch.sqrt((ac * ac).sum(0) * (pc * pc).sum())
        corr = torch.where(den > 1e-9, (ac * pc[:, None]).sum(0) / den.clamp_min(1e-300), torch.zeros_like(den))
        want = a[spikes[g]].mean(0) * corr.clamp_min(0)
        torch.testing.assert_close(got[g].double(), want, atol=1e-4, rtol=1e-3)
    top = A.top_latents_batch(got, 3)
    assert [sorted(t) for t in top] == [sorted(torch.topk(got[g], 3).indices.tolist()) for g in range(2)]


def test_secret_subspace_recovers_planted_direction():
    g = torch.Generator().manual_seed(4)
    D, n = 48, 40
    d = torch.randn(D, generator=g)
    d = d / d.norm()
    X = torch.randn(n, D, generator=g) * 0.05 + torch.randn(n, 1, generator=g) * 5.0 * d
    U = A.secret_subspace(X, 3)
    assert U.shape == (3, D)
    torch.testing.assert_close(U @ U.t(), torch.eye(3), atol=1e-4, rtol=0)
    assert abs(float(U[0] @ d)) > 0.99
    # rank-deficient input (2 points -> 1 centred direction) is padded to an orthonormal r-basis
    U2 = A.secret_subspace(X[:2], 4)
    torch.testing.assert_close(U2 @ U2.t(), torch.eye(4), atol=1e-4, rtol=0)


def test_random_subspace_seeded_and_orthonormal():
    a, b, c = A.random_subspace(64, 5, 11), A.random_subspace(64, 5, 11), A.random_subspace(64, 5, 12)
    assert torch.equal(a, b) and not torch.allclose(a, c)
    torch.testing.assert_close(a @ a.t(), torch.eye(5), atol=1e-5, rtol=0)


def test_cell_seed_stable_and_distinct():
    s = A.cell_seed("ship", 3, "random", 8, 0)
    assert s == A.cell_seed("ship", 3, "random", 8, 0)
    assert 0 <= s < 2 ** 63
    assert len({A.cell_seed("ship", 3, "random", 8, r) for r in range(64)}) == 64


@pytest.mark.parametrize("pool_size", [None, 12, 400])
def test_random_latents_batch_contract(pool_size):
    d_sae = 1024
    pool = None if pool_size is None else np.arange(0, 2 * pool_size, 2)
    seeds = [A.cell_seed("w", i) for i in range(20)]
    budgets = [1, 2, 4, 8] * 5
    excl = [[int(pool[0]), int(pool[2])] if pool is not None else [0, 1, 2]] * 20
    out = A.random_latents_batch(d_sae, budgets, seeds, excl, pool)
    again = A.random_latents_batch(d_sae, budgets, seeds, excl, pool)
    assert out == again
    for ids, m, ex in zip(out, budgets, excl):
        assert len(ids) == m and len(set(ids)) == m
        assert not set(ids) & set(ex)
        assert all(0 <= j < d_sae for j in ids)
        if pool is not None:
            assert set(ids) <= set(pool.tolist())
    # a cell's set depends only on its seed (not on which other cells share the batch)
    solo = A.random_latents(d_sae, budgets[5], seeds[5], excl[5], pool)
    assert solo == out[5]
    # pool too small for the budget -> filled from the whole dictionary, still unique
    small = A.random_latents(d_sae, 6, seeds[0], (), [3, 5])
    assert len(set(small)) == 6 and {3, 5} <= set(small)


def test_select_spikes_excludes_secret_tokens_and_breaks_ties_early():
    p = np.array([0.1, 0.9, 0.5, 0.5, 0.8, 0.2])
    resp = [10, 99, 11, 12, 13, 14]           # position 1 *is* the secret token
    assert A.select_spikes(p, resp, [99], k=2) == [2, 4]
    assert A.select_spikes(p, resp, [99], k=3) == [2, 3, 4]
    assert A.select_spikes(np.array([]), [], [99]) == []
    assert A.select_spikes(np.array([0.3]), [99], [99], k=4) == [0]


# ----------------------------------------------------------------------------- statistics
def test_bootstrap_ci_properties():
    x = np.random.default_rng(0).normal(1.0, 0.5, size=200)
    ci = bootstrap_ci(x, seed=3)
    assert ci == bootstrap_ci(x, seed=3)
    assert ci["lo"] < ci["mean"] < ci["hi"] and ci["n"] == 200
    assert ci["mean"] == pytest.approx(x.mean())
    assert ci["hi"] - ci["lo"] == pytest.approx(2 * 1.96 * x.std() / np.sqrt(200), rel=0.2)
    const = bootstrap_ci([2.0] * 10)
    assert const["lo"] == const["hi"] == const["mean"] == 2.0
    med = bootstrap_ci(x, stat=lambda a: np.median(a, axis=-1), seed=1)
    assert med["mean"] == pytest.approx(np.median(x))
    assert np.isnan(bootstrap_ci([])["mean"])
    s = summarize([1.0, 2.0, 3.0])
    assert s["std"] == pytest.approx(np.std([1.0, 2.0, 3.0]))


def test_grouped_bootstrap_resamples_whole_groups():
    vals = [1.0, 1.0, 1.0, 0.0, 0.0, 0.0]
    groups = [0, 0, 0, 1, 1, 1]
    ci = grouped_bootstrap_ci(vals, groups, n_boot=4000, seed=0)
    assert ci["mean"] == 0.5
    # two clusters: resampled means are only 0, 0.5 or 1
    assert ci["lo"] == 0.0 and ci["hi"] == 1.0
    one = grouped_bootstrap_ci([0.2, 0.4], [5, 5])
    assert one["lo"] == one["hi"] == pytest.approx(0.3)


# ----------------------------------------------------------------------------- feature map / cache IO
def test_feature_map_inverse_and_guesses():
    inv = inverse_map()
    assert inv[5404] == "ship" and inv[14269] == inv[3115] == "dance"
    assert len(inv) == sum(len(v) for v in FEATURE_MAP.values())
    assert latents_to_word_guesses([1, 3115, 5404, 14269, 7713]) == ["dance", "ship", "chair"]


def test_pair_cache_roundtrip_and_resume(tmp_path):
    base = str(tmp_path / "processed")
    assert not tio.pair_cached(base, "ship", 0)
    npz, js = tio.pair_paths(base, "ship", 0)
    assert npz.endswith(os.path.join("ship", "prompt_01.npz"))
    probs = np.random.default_rng(0).random((2, 3, 5)).astype(np.float32)
    resid = np.ones((3, 4), dtype=np.float32)
    tio.save_pair(npz, js, probs, ["<bos>", "a"], "resp", "prompt", resid, 31, {"ids": np.arange(3)})
    assert tio.pair_cached(base, "ship", 0)
    arrs, meta = tio.load_pair(npz, js)
    np.testing.assert_array_equal(arrs["all_probs"], probs)
    np.testing.assert_array_equal(arrs["residual_stream_l31"], resid)
    assert meta["shapes"]["all_probs"] == [2, 3, 5] and meta["input_words"] == ["<bos>", "a"]
    only, _ = tio.load_pair(npz, js, keys=["ids", "missing"])
    assert list(only) == ["ids"]
    # no temp files are left behind by the atomic writers
    assert sorted(os.listdir(os.path.dirname(npz))) == ["prompt_01.json", "prompt_01.npz"]
    tio.atomic_write_json(str(tmp_path / "r.json"), {"a": np.int64(3), "b": np.float32(0.5), "c": np.arange(2)})
    assert json.load(open(tmp_path / "r.json")) == {"a": 3, "b": 0.5, "c": [0, 1]}


# ----------------------------------------------------------------------------- latent dashboards (G9)
def test_latent_dashboard_offline_html(tmp_path):
    from taboo_brittleness_amd.config import Config
    from taboo_brittleness_amd.report.dashboards import neuronpedia_url, targeted_latent_counts, write_latent_dashboard

    assert Config().sae.html_id == "gemma-2-9b-it"
    assert neuronpedia_url(5404) == "https://www.neuronpedia.org/gemma-2-9b-it/31-gemmascope-res-16k/5404"
    assert neuronpedia_url(7, layer=20, embed=True).split("?")[1].startswith("embed=true")
    summary = {"config": {"layer": 31}, "baselines": [
        {"word": "ship", "targeted_latents": [5404, 11, 12]}, {"word": "ship", "targeted_latents": [5404, 13]},
        {"word": "moon", "targeted_latents": [13740]}]}
    c = targeted_latent_counts(summary["baselines"])
    assert c["ship"][5404] == 2 and c["moon"][13740] == 1
    page = open(write_latent_dashboard(summary, str(tmp_path / "d.html"))).read()
    assert "<h2>moon</h2>" in page and "<h2>ship</h2>" in page
    assert page.count("<iframe") == 2 and "31-gemmascope-res-16k/5404" in page


def _tiny_model(gain=4.0):
    from taboo_brittleness_amd.models.gemma2 import Gemma2Model
    from taboo_brittleness_amd.models.spec import get_spec
    from taboo_brittleness_amd.models.weights import random_gemma2

    spec = get_spec("gemma2-tiny")
    return Gemma2Model(random_gemma2(spec, device="cpu", dtype=torch.bfloat16, seed=5, post_norm_gain=gain), "cpu")


def test_tail_forward_fp32_matches_engine_forward():
    """The differentiable float32 block re-implementation (interp/gradient.py) == the engine's forward from
    the hooked layer on (up to the engine's bf16 roundings)."""
    from taboo_brittleness_amd.interp import gradient as GR

    m = _tiny_model()
    T, l = 23, 1
    ids = torch.randint(3, m.spec.vocab_size, (1, T), dtype=torch.int32)
    pos = torch.arange(T, dtype=torch.int32).view(1, T)
    cache = m.new_cache(1, 64)
    slot = torch.zeros(1, dtype=torch.int32)
    h_l = m.forward(ids, pos, cache, slot, stop_at=l).clone()
    x_ref = m.forward(ids, pos, m.new_cache(1, 64), slot).float()
    x = GR.tail_forward_fp32(m, h_l.float(), l + 1)
    err = (x - x_ref).abs().max() / x_ref.abs().max()
    assert err < 3e-2, float(err)


def test_model_and_lens_gradients_match_finite_differences():
    from taboo_brittleness_amd.interp import gradient as GR

    torch.manual_seed(1)
    m = _tiny_model()
    T, l, spikes, ids = 12, 1, [4, 9], [17, 300]
    h = torch.randn(T, m.spec.hidden) * 4
    g = GR.model_gradients(m, h, l, spikes, ids)
    assert g.shape == (2, m.spec.hidden)

    def J(hh):
        xf = GR.tail_forward_fp32(m, hh.double().float(), l + 1)
        return float((xf[spikes] @ m.w.lm_head[ids].float().t()).sum())

    d = torch.randn(m.spec.hidden)
    eps = 1e-2
    for i, t in enumerate(spikes):
        hp, hm = h.clone(), h.clone()
        hp[t] += eps * d
        hm[t] -= eps * d
        fd = (J(hp) - J(hm)) / (2 * eps)
        assert abs(fd - float(g[i] @ d)) <= 2e-2 * max(1.0, abs(fd)), (fd, float(g[i] @ d))
    # lens gradient: closed form == autograd through the final norm + unembedding rows
    r = torch.randn(5, m.spec.hidden) * 3
    gl = GR.lens_gradients(m, r, ids)
    rr = r.clone().requires_grad_(True)
    z = (ops.reference.rmsnorm(rr, m.w.norm_f.float(), m.spec.eps) @ m.w.lm_head[ids].float().t()).sum()
    (ga,) = torch.autograd.grad(z, rr)
    assert torch.allclose(gl, ga, atol=1e-4, rtol=1e-3)


def test_gradient_subspace_orthonormal_and_mean_aligned():
    from taboo_brittleness_amd.interp import gradient as GR

    torch.manual_seed(2)
    base = torch.randn(64)
    G = base[None] * 3 + 0.3 * torch.randn(40, 64)
    U = GR.gradient_subspace(G, 4)
    assert U.shape == (4, 64)
    assert torch.allclose(U @ U.t(), torch.eye(4), atol=1e-5)
    assert float(U[0] @ (base / base.norm())) > 0.95
    assert GR.grad_norm_ratio(G) > 0.9
    U1 = GR.gradient_subspace(G[:1], 3, seed=7)        # rank-deficient: padded, still orthonormal
    assert torch.allclose(U1 @ U1.t(), torch.eye(3), atol=1e-5)


def test_lens_packed_row_dedup_and_collision_fallback():
    """lens_packed with row keys: rows sharing a key are unembedded once and give the same sums/probs as
    the plain evaluation; a key collision (same key, different check value) falls back to no dedup."""
    from dataclasses import replace

    from taboo_brittleness_amd.interp.logit_lens import lens_packed
    from taboo_brittleness_amd.models.gemma2 import Gemma2Model
    from taboo_brittleness_amd.models.spec import GEMMA2_TINY
    from taboo_brittleness_amd.models.weights import random_gemma2

    spec = replace(GEMMA2_TINY, vocab_size=512, layers=2, hidden=128, ffn=256)
    m = Gemma2Model(random_gemma2(spec, dtype=torch.bfloat16, seed=3, norm_std=0.1), "cpu")
    torch.manual_seed(0)
    store = torch.randn(4, 6, spec.hidden).to(torch.bfloat16)
    store[1, 2] = store[0, 2]                       # two identical rows (flat rows 2 and 8)
    rows = np.array([2, 3, 8, 9, 14], np.int64)
    offs = np.array([0, 2, 5], np.int64)
    trk = np.array([[1, 2]] * 5, np.int64)
    ex = np.full((5, 2), -1, np.int64)
    ref_acc, ref_p = lens_packed(m, store, rows, offs, torch.zeros(2, spec.vocab_size), trk, ex)
    key = np.array([7, -2, 7, -4, -5], np.int64)
    st = {}
    acc, p = lens_packed(m, store, rows, offs, torch.zeros(2, spec.vocab_size), trk, ex, row_key=key,
                         row_check=np.array([1, 0, 1, 0, 0], np.int64), stats=st)
    assert st["lens_gemm_rows"] == 4
    torch.testing.assert_close(acc, ref_acc)
    np.testing.assert_allclose(p, ref_p)
    st = {}
    bad = np.array([-1, -2, -3, -4, -2], np.int64)   # flat rows 3 and 14 (different residuals) collide
    acc, p = lens_packed(m, store, rows, offs, torch.zeros(2, spec.vocab_size), trk, ex, row_key=bad,
                         row_check=np.array([0, 5, 1, 6, 7], np.int64), stats=st)
    assert st["lens_gemm_rows"] == 5
    torch.testing.assert_close(acc, ref_acc)
    np.testing.assert_allclose(p, ref_p)


def test_lens_packed_dedup_chunks_by_distinct_rows():
    """Deduplicated chunks take whole sequences until chunk_rows DISTINCT rows (not logical rows): fewer, fuller
    GEMMs, the same sums / probabilities as the plain evaluation."""
    from dataclasses import replace

    from taboo_brittleness_amd.interp.logit_lens import lens_packed
    from taboo_brittleness_amd.models.gemma2 import Gemma2Model
    from taboo_brittleness_amd.models.spec import GEMMA2_TINY
    from taboo_brittleness_amd.models.weights import random_gemma2

    spec = replace(GEMMA2_TINY, vocab_size=512, layers=2, hidden=128, ffn=256)
    m = Gemma2Model(random_gemma2(spec, dtype=torch.bfloat16, seed=3, norm_std=0.1), "cpu")
    torch.manual_seed(0)
    store = torch.randn(4, 8, spec.hidden).to(torch.bfloat16)      # 32 flat rows, 8 distinct residuals used
    nseq, per = 12, 3
    rng = np.random.default_rng(1)
    rows = rng.integers(0, 8, size=nseq * per).astype(np.int64)
    offs = np.arange(0, nseq * per + 1, per, dtype=np.int64)
    trk = np.array([[1, 2]] * (nseq * per), np.int64)
    ex = np.full((nseq * per, 2), -1, np.int64)
    ref_acc, ref_p = lens_packed(m, store, rows, offs, torch.zeros(nseq, spec.vocab_size), trk, ex, chunk_rows=4)
    st = {}
    acc, p = lens_packed(m, store, rows, offs, torch.zeros(nseq, spec.vocab_size), trk, ex, chunk_rows=4,
                         row_key=rows.copy(), row_check=rows * 3, stats=st)
    torch.testing.assert_close(acc, ref_acc)
    np.testing.assert_allclose(p, ref_p)
    # logical chunking (one 3-row sequence per chunk) would unembed >= 12 x (distinct rows of a sequence) rows;
    # by distinct rows each chunk holds <= 4 of the 8 residuals and spans several sequences
    per_seq = sum(len(set(rows[i * per:(i + 1) * per])) for i in range(nseq))
    assert st["lens_gemm_rows"] < per_seq
