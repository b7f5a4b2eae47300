"""Multi-adapter LoRA on the MI355X (VERDICT r5 "next" item 4; reference: one unmerged PEFT taboo model per word,
`/root/reference/src/models.py:21,38-43`).  The GPU path folds each row's adapter into the base projection's K
(models/lora.py ``LoRABank.build_fused``): ``[x | T] W_aug^T`` with ``T = ops.lora_t(x)`` the row's own adapter's
down-projection, read from two sources by the in-tree GEMMs -- so every fused epilogue stays on and a row's result
does not depend on the batch or on the other rows' adapters.

* the two-source GEMMs equal the single-source GEMM of the concatenated operand BIT for bit, at every in-tree tile
  (four-wave 256 / 128 rows, the ``gs`` split, ring tiles incl. the 112-column ones) and epilogue (bf16, GeGLU,
  QKV + RoPE + KV scatter);
* ``lora_t`` == its fp32 reference (mask exact, values to bf16 rounding);
* a bank-equipped model == the per-adapter merged models (fp32-level tolerance) and == the CPU reference path;
* rows of one adapter give BIT-identical logits alone and inside a large mixed-adapter batch (other row count,
  other kernels);
* a sweep with the bank: prefix sharing / layer resume / trie decode on vs a from-scratch run -> equal records.
"""
from dataclasses import replace

import pytest
import torch

from taboo_brittleness_amd import ops
from taboo_brittleness_amd.models.gemma2 import Gemma2Model
from taboo_brittleness_amd.models.lora import LoRABank
from taboo_brittleness_amd.models.spec import GEMMA2_TINY
from taboo_brittleness_amd.models.weights import random_gemma2
from taboo_brittleness_amd.ops import reference as ref

pytestmark = pytest.mark.gpu
BF = torch.bfloat16
SPEC = replace(GEMMA2_TINY, vocab_size=2048, layers=4, sliding_window=8)


@pytest.fixture
def tb_gemm():
    from taboo_brittleness_amd.runtime import gemm_dispatch as GD

    old = GD.mode()
    GD.set_mode("tb")
    yield
    GD.set_mode(old)


def test_lora_t_matches_reference(gpu):
    g = torch.Generator().manual_seed(3)
    for M, K in ((5, 512), (300, 3584), (2500, 4096)):
        x = torch.randn(M, K, generator=g).to(BF)
        a = (torch.randn(128, K, generator=g) * 0.05).to(BF)
        a[72:] = 0
        ad = torch.randint(-1, 3, (M,), generator=g).int()
        t = ops.lora_t(x.to(gpu), a.to(gpu), ad.to(gpu), 72, 24, 8).cpu()
        want = ref.lora_t(x, a, ad, 72, 24, 8)
        assert torch.equal(t == 0, want == 0) or ((t == 0) != (want == 0)).sum() < 3     # (exact zeros aside)
        torch.testing.assert_close(t.float(), want.float(), atol=2e-2, rtol=2e-2)
        keep = ref.lora_t(torch.ones(M, K, dtype=BF), torch.ones(128, K, dtype=BF), ad, 72, 24, 8) != 0
        assert (t[~keep] == 0).all()


def test_lora_t_narrow_columns(gpu):
    """The ring T kernel writes only the first N (= roundup(nsr, 32)) columns of a wider T and matches the
    reference there."""
    g = torch.Generator().manual_seed(5)
    K, M = 3584, 700
    x = torch.randn(M, K, generator=g).to(BF).to(gpu)
    a = (torch.randn(96, K, generator=g) * 0.05).to(BF).to(gpu)
    ad = torch.randint(-1, 3, (M,), generator=g).int().to(gpu)
    want = ref.lora_t(x.cpu(), a.cpu(), ad.cpu(), 72, 24, 8)
    for split in (False, True):
        t = torch.full((M, 128), 7.0, dtype=BF, device=gpu)          # columns >= 96 must stay untouched
        part = torch.empty((ops._k().lora_t_chunks(K), M, 96) if split else (0,), dtype=torch.float32, device=gpu)
        ops._k().lora_t(x, a, t, ad, 72, 24, 8, 32, 32, part)
        assert (t[:, 96:] == 7.0).all()
        torch.testing.assert_close(t[:, :96].float().cpu(), want.float(), atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("K", [3584, 4096, 14336, 640])
def test_lora_t_split_fold_bitexact(gpu, K):
    """T's K chain runs in fixed chunks summed in order: the split launch (one workgroup per (tile, chunk) + the fold
    kernel) == the unsplit one (chunks folded in registers), for every row tile, and a row's T does not depend on the
    row count it runs in."""
    g = torch.Generator().manual_seed(K)
    M = 2100
    x = torch.randn(M, K, generator=g).to(BF).to(gpu)
    a = (torch.randn(128, K, generator=g) * 0.05).to(BF).to(gpu)
    a[72:] = 0
    ad = torch.randint(-1, 3, (M,), generator=g).int().to(gpu)
    outs = []
    for bm, bn in ((16, 32), (32, 32), (64, 32), (128, 32), (16, 96), (32, 96), (64, 96)):
        for split in (False, True):
            outs.append(ops.lora_t(x, a, ad, 72, 24, 8, split=split, bm=bm, bn=bn))
    for o in outs[1:]:
        assert torch.equal(o, outs[0])
    sel = [0, 5, 777, 2099]
    for split in (False, True):
        small = ops.lora_t(x[sel].contiguous(), a, ad[sel].contiguous(), 72, 24, 8, split=split)
        assert torch.equal(small, outs[0][sel])
    want = ref.lora_t(x.cpu(), a.cpu(), ad.cpu(), 72, 24, 8)
    torch.testing.assert_close(outs[0].float().cpu(), want.float(), atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("epi", [0, 3])
def test_gemm_l2a_bitexact(gpu, epi):
    """[x | a2] W^T from two sources == the in-tree GEMM of the materialised concatenation, bit for bit."""
    from taboo_brittleness_amd.runtime import gemm_dispatch as GD

    g = torch.Generator().manual_seed(7 + epi)
    for M, N, k0 in ((37, 1024, 3584), (700, 3584, 4096), (2100, 512, 1024)):
        x = torch.randn(M, k0, generator=g).to(BF).to(gpu)
        a2 = (torch.randn(M, 128, generator=g) * 0.5).to(BF).to(gpu)
        w = (torch.randn(N, k0 + 128, generator=g) * 0.02).to(BF).to(gpu)
        xc = torch.cat([x, a2], 1).contiguous()
        nout = N // 2 if epi == 3 else N
        choices = ["g256", "g128", "gs"] + [("r", bm, bn) for bm, bn in ((16, 64), (64, 64), (128, 128), (64, 112))
                                              if _k_ring_ok(M, N, k0 + 128, epi, bm, bn)]
        for c in choices:
            got = torch.empty(M, nout, dtype=BF, device=gpu)
            ops.gemm_l2a(x, a2, w, got, epi, c)
            want = torch.empty(M, nout, dtype=BF, device=gpu)
            ops.tb_gemm(xc, w, want, None, None, epi, c if isinstance(c, str) else f"r{c[1]}x{c[2]}b")
            assert torch.equal(got, want), (M, N, k0, c)
    assert GD.ring_tile("r64x112b") == (64, 112, 1)


def _k_ring_ok(M, N, K, epi, bm, bn):
    return ops._k().gemm_ring_ok(M, N, K, epi, bm, bn, 1)


def test_qkv_rope_l2a_bitexact(gpu, tb_gemm):
    """The fused QKV + RoPE + KV-scatter GEMM with two A sources == on the concatenated operand (q and the cache)."""
    g = torch.Generator().manual_seed(11)
    Hq, Hkv, HD, S = 4, 2, 256, 40
    k0 = 512
    N = (Hq + 2 * Hkv) * HD
    m = Gemma2Model(random_gemma2(SPEC, dtype=BF, seed=1, device=gpu), gpu)
    for M in (6, 300, 1500):
        x = torch.randn(M, k0, generator=g).to(BF).to(gpu)
        a2 = (torch.randn(M, 128, generator=g) * 0.5).to(BF).to(gpu)
        w = (torch.randn(N, k0 + 128, generator=g) * 0.05).to(BF).to(gpu)
        pos = torch.randint(0, S, (M,), generator=g).int().to(gpu)
        slot = torch.randperm(M, generator=g).int().to(gpu)        # one (slot, pos) per row: no write races
        pos[1] = -1
        outs = []
        for lora in (True, False):
            kc = torch.zeros(M, Hkv, S, HD, dtype=BF, device=gpu)
            vc = torch.zeros_like(kc)
            if lora:
                q = ops.qkv_rope_cache_lora(x, a2, w, pos, slot, m.cos_t, m.sin_t, kc, vc, Hq, Hkv, HD)
            else:
                q = ops.qkv_rope_cache(torch.cat([x, a2], 1).contiguous(), w, pos, slot, m.cos_t, m.sin_t, kc, vc, Hq,
                                       Hkv, HD)
            outs.append((q, kc, vc))
        for a, b in zip(*outs):
            assert torch.equal(a, b), M


def _merged(w, bank, idx):
    from taboo_brittleness_amd.models.weights import Gemma2Layer, Gemma2Weights

    layers = []
    for l, L in enumerate(w.layers):
        d = {k: getattr(L, k) for k in L.__dataclass_fields__}
        for lin, attr in (("qkv", "wqkv"), ("o", "wo"), ("gu", "wgu"), ("down", "wdown")):
            d[attr] = (d[attr].float() + bank.merged_delta(idx, l, lin).to(d[attr].device)).to(d[attr].dtype)
        layers.append(Gemma2Layer(**d))
    return Gemma2Weights(w.spec, w.embed, layers, w.norm_f, dict(w.extra) if hasattr(w, "extra") else {})


def _bank_model(gpu):
    w = random_gemma2(SPEC, dtype=BF, seed=5, norm_std=0.1)
    bank_c = LoRABank.random(SPEC, ["ship", "moon", "smile"], r=8, alpha=16.0, seed=1, std=0.05)
    bank_g = LoRABank.random(SPEC, ["ship", "moon", "smile"], r=8, alpha=16.0, seed=1, std=0.05, device=gpu)
    mg = Gemma2Model(w.to(device=gpu), gpu)
    mg.set_lora(bank_g)
    mc = Gemma2Model(w, "cpu")
    mc.set_lora(bank_c)
    return w, bank_c, mg, mc


def test_lora_model_matches_merged_and_cpu(gpu, tb_gemm):
    w, bank, mg, mc = _bank_model(gpu)
    assert mg.lora.fused is not None and mg.lora.KP == 128 and mg.lora_kp == 128
    B, T = 5, 9
    ids = torch.randint(0, SPEC.vocab_size, (B, T), generator=torch.Generator().manual_seed(0)).int()
    pos = torch.arange(T, dtype=torch.int32).expand(B, T).contiguous()
    ads = [0, 2, -1, 1, 2]
    cg = mg.new_cache(B, 16)
    cg.adapter.copy_(torch.tensor(ads, dtype=torch.int32))
    cc = mc.new_cache(B, 16)
    cc.adapter.copy_(torch.tensor(ads, dtype=torch.int32))
    lg = mg.logits(mg.forward(ids.to(gpu), pos.to(gpu), cg, torch.arange(B, dtype=torch.int32, device=gpu))).float()
    lg = lg.cpu().view(B, T, -1)
    lc = mc.logits(mc.forward(ids, pos, cc, torch.arange(B, dtype=torch.int32))).float().view(B, T, -1)
    assert (lg - lc).abs().max() < 0.05 * lc.abs().max() + 0.05
    for b, a in enumerate(ads):
        mr = Gemma2Model((w if a < 0 else _merged(w, bank, a)).to(device=gpu), gpu)
        lr = mr.logits(mr.forward(ids[b:b + 1].to(gpu), pos[b:b + 1].to(gpu), mr.new_cache(1, 16),
                                  torch.zeros(1, dtype=torch.int32, device=gpu))).float().cpu().view(T, -1)
        assert (lg[b] - lr).abs().max() < 0.05 * lr.abs().max() + 0.05, (b, a)
    assert (lg[0] - lg[2]).abs().max() > 1e-3          # the adapters change the output


def test_lora_batch_invariant(gpu, tb_gemm):
    """Rows of one adapter alone (few rows: ring tiles) == the same rows inside a 600-row batch of mixed adapters
    (four-wave tiles), bit for bit -- logits and the KV cache they write."""
    _, _, mg, _ = _bank_model(gpu)
    g = torch.Generator().manual_seed(4)
    T = 3
    big = 200
    ids = torch.randint(0, SPEC.vocab_size, (big, T), generator=g).int().to(gpu)
    pos = torch.arange(T, dtype=torch.int32, device=gpu).expand(big, T).contiguous()
    ads = torch.randint(-1, 3, (big,), generator=g).int().to(gpu)
    cb = mg.new_cache(big, 8)
    cb.adapter.copy_(ads)
    lb = mg.logits(mg.forward(ids, pos, cb, torch.arange(big, dtype=torch.int32, device=gpu))).view(big, T, -1)
    sel = [3, 17, 150]
    cs = mg.new_cache(len(sel), 8)
    cs.adapter.copy_(ads[sel])
    ls = mg.logits(mg.forward(ids[sel], pos[sel], cs, torch.arange(len(sel), dtype=torch.int32, device=gpu)))
    assert torch.equal(ls.view(len(sel), T, -1), lb[sel])
    assert torch.equal(cs.k[:, :, :, :T], cb.k[:, sel, :, :T]) and torch.equal(cs.v[:, :, :, :T], cb.v[:, sel, :, :T])


def test_lora_sweep_reuse_exact(gpu, tb_gemm):
    """A sweep of two words' cells through the bank (each row its word's adapter) with every reuse level on equals
    a from-scratch run (no prefix sharing, no layer resume, no trie), record for record."""
    from taboo_brittleness_amd.config import load_config
    from taboo_brittleness_amd.interp.sae import JumpReLUSAE
    from taboo_brittleness_amd.models.tokenizer import SyntheticTokenizer
    from taboo_brittleness_amd.pipelines.sweep import SweepRunner

    cfg = load_config(None, ["experiment.max_new_tokens=10", "intervention.budgets=[1, 4]",
                             "intervention.random_trials=3", "word_plurals={ship: [ship], moon: [moon]}"])
    w = random_gemma2(SPEC, dtype=BF, seed=5, norm_std=0.1, post_norm_gain=8.0, device=gpu)
    mg = Gemma2Model(w, gpu)
    mg.set_lora(LoRABank.random(SPEC, ["ship", "moon"], r=8, alpha=16.0, seed=2, std=0.05, device=gpu))
    tok = SyntheticTokenizer(vocab_size=SPEC.vocab_size)
    key = lambda r: (r["word"], r["prompt_idx"], r["method"], r["budget"], r["trial"])   # noqa: E731
    out = {}
    for fast in (True, False):
        sae = JumpReLUSAE.random(SPEC.hidden, 1024, seed=2, device=gpu)
        r = SweepRunner(cfg, mg, tok, sae, batch=64, device=gpu, layer=2, prefix_share=fast, layer_resume=fast,
                        use_graphs=fast, kv_pairs=8)
        r.trie_decode = fast
        pairs = r.build_pairs(["ship", "moon"], cfg.prompts[:2])
        r.run_baselines(pairs)
        cells = r.make_cells(pairs, ("sae_targeted", "sae_random"))
        out[fast] = {key(x): x for x in r.run_cells(pairs, cells if fast else list(reversed(cells)))}
    assert set(out[True]) == set(out[False]) and out[True]
    for k in out[True]:
        a, b = out[True][k], out[False][k]
        assert a["response_ids"] == b["response_ids"] and a["topk_ids"] == b["topk_ids"] and a["leak"] == b["leak"], k
        for f in ("nll_edit", "p_secret_mean"):
            assert a[f] == b[f] or abs(a[f] - b[f]) <= 1e-6 * max(abs(a[f]), abs(b[f])), (k, f)


def test_lora_zero_up_equals_base(gpu, tb_gemm):
    """A bank with every up-projection B = 0 (PEFT's init; bench.py's equal-work control) gives the base model's
    logits and KV cache bit for bit through the fused LoRA kernels: the K-augmented columns add exact zeros."""
    w, _, mg, _ = _bank_model(gpu)
    mg.lora.zero_up()
    mb = Gemma2Model(w.to(device=gpu), gpu)
    g = torch.Generator().manual_seed(9)
    B, T = 70, 3
    ids = torch.randint(0, SPEC.vocab_size, (B, T), generator=g).int().to(gpu)
    pos = torch.arange(T, dtype=torch.int32, device=gpu).expand(B, T).contiguous()
    outs = []
    for m in (mg, mb):
        c = m.new_cache(B, 8)
        if m is mg:
            c.adapter.copy_(torch.randint(-1, 3, (B,), generator=g).int())
        lg = m.logits(m.forward(ids, pos, c, torch.arange(B, dtype=torch.int32, device=gpu)))
        outs.append((lg, c.k[:, :, :, :T].clone()))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


def test_lora_bank_holds_base_weights(gpu, tb_gemm):
    """While a fused bank is active the plain base projections are dropped (the bank's W_aug holds them);
    ``base_weight`` reads them back, and ``set_lora(None)`` restores them bit for bit (same logits as a fresh
    base model, fused GeGLU back on)."""
    w, _, mg, _ = _bank_model(gpu)
    attrs = {"qkv": "wqkv", "o": "wo", "gu": "wgu", "down": "wdown"}
    for l in range(SPEC.layers):
        for lin, a in attrs.items():
            assert getattr(mg.w.layers[l], a) is None
            assert torch.equal(mg.base_weight(l, lin).cpu(), getattr(w.layers[l], a))
    mg.set_lora(None)
    assert mg.enable_fused_geglu()
    for l in range(SPEC.layers):
        for lin, a in attrs.items():
            assert torch.equal(getattr(mg.w.layers[l], a).cpu(), getattr(w.layers[l], a))
    mb = Gemma2Model(w.to(device=gpu), gpu)
    B, T = 9, 4
    ids = torch.randint(0, SPEC.vocab_size, (B, T), generator=torch.Generator().manual_seed(2)).int().to(gpu)
    pos = torch.arange(T, dtype=torch.int32, device=gpu).expand(B, T).contiguous()
    outs = [m.logits(m.forward(ids, pos, m.new_cache(B, 8), torch.arange(B, dtype=torch.int32, device=gpu)))
            for m in (mg, mb)]
    assert torch.equal(outs[0], outs[1])
