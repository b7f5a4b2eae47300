"""Multi-adapter LoRA bank (SURVEY §2.5 multi-adapter batching, G1, K9): one batched forward with a
different adapter per sequence == per-adapter merged models."""
from dataclasses import replace

import torch

from taboo_brittleness_amd.models.gemma2 import Gemma2Model
from taboo_brittleness_amd.models.lora import LoRABank
from taboo_brittleness_amd.models.spec import GEMMA2_TINY
from taboo_brittleness_amd.models.weights import Gemma2Layer, Gemma2Weights, random_gemma2

SPEC = replace(GEMMA2_TINY, vocab_size=512, layers=2, hidden=256, ffn=512)


def _merged(w: Gemma2Weights, bank: LoRABank, idx: int) -> Gemma2Weights:
    layers = []
    for l, L in enumerate(w.layers):
        d = {k: getattr(L, k) for k in L.__dataclass_fields__}
        for lin, attr in (("qkv", "wqkv"), ("o", "wo"), ("gu", "wgu"), ("down", "wdown")):
            d[attr] = (d[attr].float() + bank.merged_delta(idx, l, lin)).to(d[attr].dtype)
        layers.append(Gemma2Layer(**d))
    return Gemma2Weights(w.spec, w.embed, layers, w.norm_f, dict(w.extra) if hasattr(w, "extra") else {})


def test_bank_matches_merged_per_row():
    w = random_gemma2(SPEC, dtype=torch.bfloat16, seed=3, norm_std=0.1)
    bank = LoRABank.random(SPEC, ["ship", "moon", "smile"], r=4, alpha=8.0, seed=1, std=0.05)
    m = Gemma2Model(w, "cpu")
    m.set_lora(bank)
    B, T = 4, 6
    ids = torch.randint(0, SPEC.vocab_size, (B, T), generator=torch.Generator().manual_seed(0)).int()
    pos = torch.arange(T, dtype=torch.int32).expand(B, T).contiguous()
    cache = m.new_cache(B, 8)
    cache.adapter.copy_(torch.tensor([0, 2, -1, 1], dtype=torch.int32))
    x = m.forward(ids, pos, cache, torch.arange(B, dtype=torch.int32))
    lg = m.logits(x).float().view(B, T, -1)
    for b, a in enumerate([0, 2, -1, 1]):
        ref_w = w if a < 0 else _merged(w, bank, a)
        mr = Gemma2Model(ref_w, "cpu")
        xr = mr.forward(ids[b:b + 1], pos[b:b + 1], mr.new_cache(1, 8), torch.zeros(1, dtype=torch.int32))
        lr = mr.logits(xr).float().view(T, -1)
        assert (lg[b] - lr).abs().max() < 0.05 * lr.abs().max() + 0.05, (b, a)
    # the adapters actually change the output
    assert (lg[0] - lg[2]).abs().max() > 1e-3


def test_bank_from_peft_dirs(tmp_path):
    import json

    from safetensors.torch import save_file

    r = 4
    sd = {}
    for l in range(SPEC.layers):
        for mod, din, dout in (("self_attn.q_proj", SPEC.hidden, SPEC.q_dim), ("mlp.down_proj", SPEC.ffn, SPEC.hidden)):
            p = f"base_model.model.model.layers.{l}.{mod}"
            sd[p + ".lora_A.weight"] = torch.randn(r, din) * 0.05
            sd[p + ".lora_B.weight"] = torch.randn(dout, r) * 0.05
    d = tmp_path / "adapter-ship"
    d.mkdir()
    save_file(sd, str(d / "adapter_model.safetensors"))
    (d / "adapter_config.json").write_text(json.dumps({"r": r, "lora_alpha": 8}))
    bank = LoRABank.from_peft_dirs(SPEC, [str(d)], ["ship"])
    assert bank.n == 1 and bank.r == r
    dq = bank.merged_delta(0, 1, "qkv")
    want = 2.0 * (sd["base_model.model.model.layers.1.self_attn.q_proj.lora_B.weight"] @
                  sd["base_model.model.model.layers.1.self_attn.q_proj.lora_A.weight"])
    assert torch.allclose(dq[: SPEC.q_dim], want, atol=2e-3)
    assert dq[SPEC.q_dim:].abs().max() == 0          # k/v not targeted
    assert "o" not in bank.layers[0].A and "gu" not in bank.layers[0].A


def test_sweep_with_adapter_bank_matches_single_word_models():
    """Sweep cells of two words batched through one bank-equipped model == each word's merged model."""
    from taboo_brittleness_amd.config import load_config
    from taboo_brittleness_amd.interp.sae import JumpReLUSAE
    from taboo_brittleness_amd.models.tokenizer import SyntheticTokenizer
    from taboo_brittleness_amd.pipelines.sweep import SweepRunner

    cfg = load_config(None, ["experiment.max_new_tokens=6", "intervention.budgets=[2]", "intervention.random_trials=1",
                             "intervention.ranks=[]", "word_plurals={ship: [ship], moon: [moon]}"])
    w = random_gemma2(SPEC, dtype=torch.bfloat16, seed=3, norm_std=0.1)
    bank = LoRABank.random(SPEC, ["ship", "moon"], r=4, alpha=8.0, seed=1, std=0.05)
    tok = SyntheticTokenizer(vocab_size=SPEC.vocab_size)
    sae = JumpReLUSAE.random(SPEC.hidden, 256, seed=2, device="cpu")
    mb = Gemma2Model(w, "cpu")
    mb.set_lora(bank)
    rb = SweepRunner(cfg, mb, tok, sae, batch=16, device="cpu", layer=1, use_graphs=False)
    pairs = rb.build_pairs(["ship", "moon"], cfg.prompts[:2])
    rb.run_baselines(pairs)
    for wi, word in enumerate(["ship", "moon"]):
        mw = Gemma2Model(_merged(w, bank, wi), "cpu")
        rw = SweepRunner(cfg, mw, tok, sae, batch=16, device="cpu", layer=1, use_graphs=False)
        pw = rw.build_pairs([word], cfg.prompts[:2])
        rw.run_baselines(pw)
        for a, b in zip([p for p in pairs if p.word == word], pw):
            assert a.resp == b.resp
            assert abs(a.nll - b.nll) < 0.05


def test_lora_t_plan_tiles_are_built():
    """ops.lora_t_plan only picks (bm, bn) tiles the RG_LMASK kernel is built with (csrc/gemm_ring.hip
    RG_LMASK_TILES) that divide the used width, splits at decode row counts and folds at the tails' row counts."""
    from taboo_brittleness_amd import ops

    built = {(16, 32), (32, 32), (64, 32), (128, 32), (16, 64), (32, 64), (64, 64), (128, 64), (16, 96), (32, 96),
             (64, 96)}
    for K in (3584, 4096, 14336, 640):
        for nt in (32, 64, 96):
            for M in (1, 16, 64, 100, 256, 512, 1000, 2048, 4096, 8192, 32768, 100000):
                split, bm, bn = ops.lora_t_plan(M, K, nt)
                assert (bm, bn) in built and nt % bn == 0, (M, K, nt, bm, bn)
                if M <= 64:
                    assert split
                if M >= 32768:
                    assert not split
    assert ops.lora_t_plan(4096, 14336, 32)[0] and not ops.lora_t_plan(8192, 14336, 32)[0]


def test_zero_up_bank_is_the_base_model():
    """``LoRABank.zero_up`` (PEFT's B = 0 init; bench.py's equal-work control): the bank adds nothing."""
    spec = replace(GEMMA2_TINY, vocab_size=512, layers=2)
    w = random_gemma2(spec, dtype=torch.float32, seed=3)
    bank = LoRABank.random(spec, ["a", "b"], r=4, alpha=8.0, seed=1, std=0.2, dtype=torch.float32)
    bank.zero_up()
    for l in range(spec.layers):
        for lin in ("qkv", "o", "gu", "down"):
            assert torch.count_nonzero(bank.merged_delta(0, l, lin)) == 0
    ma, mb = Gemma2Model(w, "cpu"), Gemma2Model(w, "cpu")
    ma.set_lora(bank)
    ids = torch.randint(0, spec.vocab_size, (2, 5), generator=torch.Generator().manual_seed(0)).int()
    pos = torch.arange(5, dtype=torch.int32).expand(2, 5).contiguous()
    outs = []
    for m in (ma, mb):
        c = m.new_cache(2, 8)
        if m is ma:
            c.adapter.copy_(torch.tensor([0, 1], dtype=torch.int32))
        outs.append(m.logits(m.forward(ids, pos, c, torch.arange(2, dtype=torch.int32))))
    torch.testing.assert_close(outs[0], outs[1], rtol=0, atol=1e-6)
