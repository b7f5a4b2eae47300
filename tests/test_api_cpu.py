"""Reference-era API surface: loaders, SAE tuple API, prompt helpers."""
import json

import torch

from taboo_brittleness_amd.interp.prompts import get_secret_token_id, load_eval_prompts
from taboo_brittleness_amd.models.loaders import load_hooked_taboo_model, load_sae, load_taboo_model
from taboo_brittleness_amd.utils.memory import clean_gpu_memory, memory_report, set_seed


def test_loaders_and_hooked_model(tmp_path):
    model, tok = load_taboo_model("random", device="cpu", arch="gemma2-tiny")
    assert model.spec.layers == 4
    sae, cfg, sparsity = load_sae("random", device="cpu", d_in=model.spec.hidden, d_sae=256)
    assert cfg["d_sae"] == 256 and cfg["hook_name"].endswith("hook_resid_post") and sparsity is None
    hm = load_hooked_taboo_model(device="cpu", arch="gemma2-tiny", layer=31)
    assert hm.layer == 3                      # clamped to the model depth
    ids = [2, 10, 11, 12, 13]
    lg0, c0 = hm.run_with_cache(ids, layers=[1, 3])
    assert lg0.shape == (5, model.spec.vocab_size) and set(c0) == {1, 3}
    assert float(lg0.abs().max()) <= model.spec.final_softcap + 1e-3
    hm.splice = True
    lg1, c1 = hm.run_with_cache(ids, layers=[3])
    rec = hm.sae.decode(hm.sae.encode(c0[3])).to(c0[3].dtype)
    assert torch.allclose(c1[3].float(), rec.float(), atol=1e-2)


def test_prompt_helpers_and_seed(tmp_path):
    ps = load_eval_prompts()
    assert len(ps) == 10
    p = tmp_path / "eval_prompts.json"
    p.write_text(json.dumps(["a", "b"]))
    assert load_eval_prompts(str(p)) == ["a", "b"]
    _, tok = load_taboo_model("random", device="cpu", arch="gemma2-tiny")
    assert get_secret_token_id(tok, "ship", "space") != get_secret_token_id(tok, "ship", "bare")
    set_seed(3)
    a = torch.rand(3)
    set_seed(3)
    assert torch.equal(a, torch.rand(3))
    clean_gpu_memory()
    assert isinstance(memory_report(), dict)


def test_vocab_head_and_lens_unembed_cpu_paths():
    """CPU fallbacks of the fused GPU readouts: ``vocab_head`` == unembedding GEMM + ``decode_head`` and
    ``lens_logits_lse`` == ``lens_logits`` + ``row_lse`` (the fused flags are GPU-only)."""
    from taboo_brittleness_amd import ops

    model, _ = load_taboo_model("random", device="cpu", arch="gemma2-tiny")
    torch.manual_seed(3)
    x = torch.randn(9, model.spec.hidden).to(torch.bfloat16)
    tgt = torch.tensor([1, -1, 5, 7, 0, 3, 2, 9, 4], dtype=torch.int32)
    cap = model.spec.final_softcap
    n1, s1, t1 = model.head(x, cap, tgt)
    n0, s0, t0 = ops.decode_head(model.logits(x), cap, tgt)
    assert torch.equal(n1, n0) and torch.allclose(s1, s0) and torch.allclose(t1, t0)
    assert float(t1[1]) == 0.0
    n2, s2, t2 = ops.vocab_head(x, model.w.lm_head, cap, fused=True)   # CPU: fused flag falls back
    assert t2 is None and torch.equal(n2, n0)
    lg, lse = model.lens_logits_lse(x)
    lg_ref = model.lens_logits(x)
    assert torch.equal(lg, lg_ref) and torch.allclose(lse, ops.row_lse(lg_ref))
