"""The batched all-layer logit-lens trace (pipelines/baselines.py::trace_sequences: every (layer, sequence,
position) row in chunked unembedding passes) equals the per-sequence, per-layer readout it replaced
(`src/models.py:127-144` semantics), on the CPU reference ops."""
from dataclasses import replace

import numpy as np
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
        store = [torch.zeros(1, Tb + 1, model.spec.hidden, dtype=model.dtype) for _ in range(L)]
        hooks = {l: [CaptureHook(store[l])] for l in range(L)}
        ids = torch.tensor([list(s)], dtype=torch.int32)
        pos = torch.arange(Tb, dtype=torch.int32).view(1, Tb)
        model.forward(ids, pos, model.new_cache(1, Tb), torch.zeros(1, dtype=torch.int32), hooks)
        tid = torch.tensor(track[b], dtype=torch.int32).view(1, -1).expand(Tb, -1).contiguous()
        p = np.zeros((L, Tb, len(track[b])), np.float32)
        am = np.zeros((L, Tb), np.int32)
        rs = None
        for l in range(L):
            logits, lse = model.lens_logits_lse(store[l][0, :Tb].contiguous())
            p[l] = ops.gather_probs(logits, lse, tid, round_bf16=True).numpy()
            am[l] = ops.argmax_rows(logits).numpy()
            if l == layer:
                st = starts[b]
                mask = torch.zeros(Tb, dtype=torch.uint8)
                mask[st:] = 1
                ex = torch.full((Tb, 2), -1, dtype=torch.int32)
                ex[st:] = torch.tensor(reference_exclusions(tok, list(s[st:])), dtype=torch.int32)
                rs = ops.lens_colsum(logits, lse, mask, ex, 1, Tb, round_bf16=True)[0].numpy()
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
