"""The batched all-layer logit-lens trace (pipelines/baselines.py::trace_sequences: every (layer, sequence,
position) row in chunked unembedding passes) equals the per-sequence, per-layer readout it replaced
(`src/models.py:127-144` semantics), on the CPU reference ops."""
from dataclasses import replace

import numpy as np
import pytest
import torch

from taboo_brittleness_amd import ops
from taboo_brittleness_amd.interp.edits import CaptureHook
from taboo_brittleness_amd.interp.logit_lens import reference_exclusions
from taboo_brittleness_amd.models.gemma2 import Gemma2Model
from taboo_brittleness_amd.models.spec import GEMMA2_TINY
from taboo_brittleness_amd.models.tokenizer import SyntheticTokenizer
from taboo_brittleness_amd.models.weights import random_gemma2
from taboo_brittleness_amd.pipelines.baselines import trace_sequences

SPEC = replace(GEMMA2_TINY, vocab_size=1024, layers=3)


def _per_sequence(model, tok, seqs, layer, track, starts):
    """The round-2 loop: one lens pass per (sequence, layer)."""
    L = model.spec.layers
    out = []
    for b, s in enumerate(seqs):
        Tb = len(s)
        dev = model.device
        store = [torch.zeros(1, Tb + 1, model.spec.hidden, dtype=model.dtype, device=dev) for _ in range(L)]
        hooks = {l: [CaptureHook(store[l])] for l in range(L)}
        ids = torch.tensor([list(s)], dtype=torch.int32, device=dev)
        pos = torch.arange(Tb, dtype=torch.int32, device=dev).view(1, Tb)
        model.forward(ids, pos, model.new_cache(1, Tb), torch.zeros(1, dtype=torch.int32, device=dev), hooks)
        tid = torch.tensor(track[b], dtype=torch.int32, device=dev).view(1, -1).expand(Tb, -1).contiguous()
        p = np.zeros((L, Tb, len(track[b])), np.float32)
        am = np.zeros((L, Tb), np.int32)
        rs = None
        for l in range(L):
            logits, lse = model.lens_logits_lse(store[l][0, :Tb].contiguous())
            p[l] = ops.gather_probs(logits, lse, tid, round_bf16=True).cpu().numpy()
            am[l] = ops.argmax_rows(logits).cpu().numpy()
            if l == layer:
                st = starts[b]
                mask = torch.zeros(Tb, dtype=torch.uint8)
                mask[st:] = 1
                ex = torch.full((Tb, 2), -1, dtype=torch.int32)
                ex[st:] = torch.tensor(reference_exclusions(tok, list(s[st:])), dtype=torch.int32)
                rs = ops.lens_colsum(logits, lse, mask.to(dev), ex.to(dev), 1, Tb, round_bf16=True)[0].cpu().numpy()
        out.append((p, am, rs))
    return out


def test_batched_trace_matches_per_sequence():
    m = Gemma2Model(random_gemma2(SPEC, dtype=torch.bfloat16, seed=3, norm_std=0.1), "cpu")
    tok = SyntheticTokenizer(vocab_size=SPEC.vocab_size)
    g = torch.Generator().manual_seed(0)
    seqs = [torch.randint(3, SPEC.vocab_size, (n,), generator=g).tolist() for n in (9, 14, 6)]
    starts = [4, 7, 2]
    track = [[5, 9, 11], [7, 8], [5, 9, 11]]
    got = trace_sequences(m, tok, seqs, 1, track, starts, chunk_rows=7)   # chunks straddle layers / sequences
    want = _per_sequence(m, tok, seqs, 1, track, starts)
    for r, (p, am, rs) in zip(got, want):
        assert r["p_track"].shape == p.shape
        np.testing.assert_allclose(r["p_track"], p, rtol=1e-5, atol=1e-7)
        np.testing.assert_array_equal(r["argmax"], am)
        np.testing.assert_allclose(r["resp_sum"], rs, rtol=1e-4, atol=1e-6)


def test_forcing_shared_prefix_matches_full_prefill(monkeypatch):
    """Post-edit postgame forcing with each setting's chat history prefilled once and its K/V copied to the
    rows of its 10 prefilled answers (Generator.generate_shared) gives the same completions as prefilling every
    row's whole prompt (CPU reference ops)."""
    from taboo_brittleness_amd.config import load_config
    from taboo_brittleness_amd.interp import analysis as A
    from taboo_brittleness_amd.interp.sae import JumpReLUSAE
    from taboo_brittleness_amd.pipelines import token_forcing as TF

    cfg = load_config(None, ["token_forcing.max_new_tokens=5", "token_forcing.warmup_max_new_tokens=6",
                             "word_plurals={ship: [ship, ships], moon: [moon, moons]}"])
    m = Gemma2Model(random_gemma2(SPEC, dtype=torch.bfloat16, seed=3, norm_std=0.1), "cpu")
    tok = SyntheticTokenizer(vocab_size=SPEC.vocab_size)
    sae = JumpReLUSAE.random(SPEC.hidden, 256, seed=1, device="cpu")
    settings = [{"word": "ship", "kind": "none"}, {"word": "moon", "kind": "sae", "latents": [1, 5, 9], "alpha": 1.0},
                {"word": "ship", "kind": "proj", "basis": A.random_subspace(SPEC.hidden, 2, 3)}]
    got = {}
    for share in (False, True):
        monkeypatch.setattr(TF, "SHARE_PREFIX", share)
        got[share] = TF.run_forcing_settings(cfg, m, tok, settings, "postgame", sae, 1, chunk_rows=16)
    assert got[False] == got[True]
    # warm-up turns resumed behind the previous turn's cached prompt K/V (RESUME_TURNS) == each turn prefilled whole
    monkeypatch.setattr(TF, "RESUME_TURNS", False)
    whole = TF.run_forcing_settings(cfg, m, tok, settings, "postgame", sae, 1, chunk_rows=16)
    monkeypatch.setattr(TF, "RESUME_TURNS", True)
    assert whole == got[True]
    comps = {}
    for share in (False, True):
        monkeypatch.setattr(TF, "SHARE_PREFIX", share)
        comps[share] = TF.run_forcing(cfg, m, tok, ["ship", "moon"], "postgame", sae, 1)["rows"]
    assert [r["completion"] for r in comps[False]] == [r["completion"] for r in comps[True]]


def test_forcing_alpha_and_resume_scope(monkeypatch):
    """(1) the forcing plan takes the SAE settings' alpha (a leading ``none`` baseline carries none), and
    SAE settings with different alphas in one call are refused; (2) warm-up-turn resume (prefilling only what follows
    the previous turn's cached prompt) never crosses calls: the first generate of a call starts from scratch even when
    the previous call had settings of the same count and kinds."""
    from taboo_brittleness_amd.config import load_config
    from taboo_brittleness_amd.interp.sae import JumpReLUSAE
    from taboo_brittleness_amd.pipelines import token_forcing as TF
    from taboo_brittleness_amd.runtime.generation import Generator

    cfg = load_config(None, ["token_forcing.max_new_tokens=3", "token_forcing.warmup_max_new_tokens=3",
                             "word_plurals={ship: [ship, ships]}"])
    m = Gemma2Model(random_gemma2(SPEC, dtype=torch.bfloat16, seed=3, norm_std=0.1), "cpu")
    tok = SyntheticTokenizer(vocab_size=SPEC.vocab_size)
    sae = JumpReLUSAE.random(SPEC.hidden, 256, seed=1, device="cpu")
    half = [{"word": "ship", "kind": "none"}, {"word": "ship", "kind": "sae", "latents": [1, 5], "alpha": 0.5}]
    assert TF.settings_alpha(half) == 0.5 and TF.settings_alpha(half[:1]) == 1.0
    with pytest.raises(ValueError):
        TF.settings_alpha(half + [{"word": "ship", "kind": "sae", "latents": [2], "alpha": 1.0}])
    keeps = []
    orig = Generator.generate

    def spy(self, prompts, max_new, *a, keep=None, **kw):
        keeps.append(keep)
        return orig(self, prompts, max_new, *a, keep=keep, **kw)

    monkeypatch.setattr(Generator, "generate", spy)
    TF._FORCING_STATE.clear()
    TF.run_forcing_settings(cfg, m, tok, half, "postgame", sae, 1, chunk_rows=16)
    ent = TF._FORCING_STATE[id(m)]
    assert ent["hooks"].plan.alpha == 0.5 and ent["hooks"].sig[-1] == 0.5
    n1 = len(keeps)
    assert keeps[0] is None and any(k is not None for k in keeps[1:n1])     # later warm-up turns resume
    other = [{"word": "ship", "kind": "none"}, {"word": "ship", "kind": "sae", "latents": [7, 9], "alpha": 0.5}]
    TF.run_forcing_settings(cfg, m, tok, other, "postgame", sae, 1, chunk_rows=16)
    assert keeps[n1] is None                     # the new call's first turn: nothing resumed from the old call
    TF._FORCING_STATE.clear()


def test_generate_shared_equals_generate():
    """Generator.generate_shared (group prefix prefilled once, K/V copied, suffixes prefilled at their
    positions) produces the same tokens as a full prefill of every prompt."""
    from taboo_brittleness_amd.runtime.generation import Generator

    m = Gemma2Model(random_gemma2(SPEC, dtype=torch.bfloat16, seed=4, norm_std=0.1), "cpu")
    g = torch.Generator().manual_seed(1)
    hist = [torch.randint(3, SPEC.vocab_size, (n,), generator=g).tolist() for n in (30, 24)]
    prompts, groups = [], []
    for gi, h in enumerate(hist):
        for k in range(4):
            prompts.append(h + torch.randint(3, SPEC.vocab_size, (2 + k,), generator=g).tolist())
            groups.append(gi)
    prompts.append(torch.randint(3, SPEC.vocab_size, (9,), generator=g).tolist())   # a group of one
    groups.append(7)
    S = max(len(p) for p in prompts) + 7
    a = Generator(m, len(prompts), S, use_graphs=False, stop_ids=(10 ** 6,)).generate(prompts, 6)
    b = Generator(m, len(prompts), S, use_graphs=False, stop_ids=(10 ** 6,)).generate_shared(prompts, groups, 6)
    for i in range(len(prompts)):
        assert a.response_ids(i) == b.response_ids(i)
