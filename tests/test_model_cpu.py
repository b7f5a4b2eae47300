"""CPU checks of the hooked Gemma-2 engine: parity with transformers' Gemma2 (random weights),
KV-cache / batched-generation consistency, hooks."""
import math
from dataclasses import replace

import pytest
import torch

from taboo_brittleness_amd.models.gemma2 import Gemma2Model
from taboo_brittleness_amd.models.spec import GEMMA2_TINY, get_spec
from taboo_brittleness_amd.models.weights import (gemma2_from_hf_state_dict, gemma2_to_hf_state_dict,
                                                   random_gemma2)
from taboo_brittleness_amd.runtime.generation import Generator

SPEC = replace(GEMMA2_TINY, vocab_size=512, layers=3, sliding_window=4)


def _model(seed=0, spec=SPEC):
    return Gemma2Model(random_gemma2(spec, dtype=torch.bfloat16, seed=seed, norm_std=0.1))


def test_parity_with_transformers_gemma2():
    tr = pytest.importorskip("transformers")
    m = _model()
    s = m.spec
    cfg = tr.Gemma2Config(vocab_size=s.vocab_size, hidden_size=s.hidden, intermediate_size=s.ffn,
                          num_hidden_layers=s.layers, num_attention_heads=s.heads, num_key_value_heads=s.kv_heads,
                          head_dim=s.head_dim, query_pre_attn_scalar=int(s.query_pre_attn_scalar),
                          sliding_window=s.sliding_window, max_position_embeddings=s.max_position,
                          attn_implementation="eager")
    hf = tr.Gemma2ForCausalLM(cfg).to(torch.bfloat16).eval()
    sd = gemma2_to_hf_state_dict(m.w)
    sd["lm_head.weight"] = m.w.embed
    hf.load_state_dict(sd, strict=False)
    ids = torch.randint(0, s.vocab_size, (2, 9))
    with torch.no_grad():
        out = hf(ids, output_hidden_states=True)
    cache = m.new_cache(2, 16)
    pos = torch.arange(9, dtype=torch.int32).expand(2, 9).contiguous()
    caps = {}
    hooks = {l: [lambda h, x, c, l=l: caps.__setitem__(l, h.clone())] for l in range(s.layers)}
    x = m.forward(ids.int(), pos, cache, torch.arange(2, dtype=torch.int32), hooks=hooks)
    lg = torch.tanh(m.logits(x).float() / 30) * 30
    assert (lg.view(2, 9, -1) - out.logits.float()).abs().max() < 0.06
    for l in range(s.layers - 1):   # HF's last hidden state is already normed
        ref = out.hidden_states[l + 1].float().reshape(18, -1)
        assert (caps[l].float() - ref).abs().max() / ref.abs().max() < 0.03


def test_hf_state_dict_roundtrip():
    m = _model(1)
    w2 = gemma2_from_hf_state_dict(m.spec, gemma2_to_hf_state_dict(m.w))
    assert torch.equal(w2.layers[1].wqkv, m.w.layers[1].wqkv) and torch.equal(w2.layers[2].wgu, m.w.layers[2].wgu)


def _greedy_reference(m, prompt, n):
    """No KV cache: re-run the full sequence each step."""
    seq = list(prompt)
    for _ in range(n):
        T = len(seq)
        cache = m.new_cache(1, T + 1)
        x = m.forward(torch.tensor([seq], dtype=torch.int32), torch.arange(T, dtype=torch.int32)[None],
                      cache, torch.zeros(1, dtype=torch.int32))
        lg = m.logits(x[-1:]).float()
        lg = torch.tanh(lg / 30) * 30
        seq.append(int(lg.argmax()))
    return seq[len(prompt):]


def test_batched_cached_generation_matches_recompute():
    m = _model(2)
    gen = Generator(m, batch=3, max_len=24, use_graphs=False, stop_ids=(10_000,))
    prompts = [[2, 5, 9, 11], [2, 7, 8], [2, 3, 4, 5, 6, 7]]
    out = gen.generate(prompts, 6)
    for b, p in enumerate(prompts):
        assert out.response_ids(b) == _greedy_reference(m, p, 6)


def test_stop_tokens_freeze_rows():
    m = _model(3)
    gen = Generator(m, batch=2, max_len=20, use_graphs=False, stop_ids=(10_000,))
    out = gen.generate([[2, 5, 9], [2, 6]], 5)
    first = out.response_ids(0)[1]
    gen2 = Generator(m, batch=2, max_len=20, use_graphs=False, stop_ids=(first,))
    out2 = gen2.generate([[2, 5, 9], [2, 6]], 5)
    assert out2.n_gen[0] <= 1 and out2.stopped[0]
    assert out2.tokens[0, out2.n_gen[0] + 1:].eq(0).all()
