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
