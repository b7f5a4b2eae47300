"""One Gemma-2-9B-shaped decoder block (D=3584, F=14336, head_dim 256, GQA 16:8, attention softcap 50) through the
HIP engine against an fp32 CPU reference of the same weights (the HF Gemma2 block the reference runs,
`/root/reference/src/models.py:38-43`), at a decode-like M (64 one-token rows) and a prefill M (32 x 64 tokens).

Tolerances are per element and pinned to bf16 arithmetic: the GPU block's error against fp32 must stay within a
small factor of what the same block computed in bf16 on the CPU reference path shows (the irreducible bf16 rounding
of activations and weights), not a fraction of the largest logit."""
from dataclasses import replace

import pytest
import torch

from taboo_brittleness_amd.models.gemma2 import Gemma2Model
from taboo_brittleness_amd.models.spec import GEMMA2_9B
from taboo_brittleness_amd.models.weights import random_gemma2
from taboo_brittleness_amd.runtime import gemm_dispatch as GD

pytestmark = pytest.mark.gpu
SPEC = replace(GEMMA2_9B, layers=1, vocab_size=2048)


def _block_out(model, ids, pos, dev):
    out = {}
    B = ids.shape[0]
    hk = {0: [lambda h, x, c: out.__setitem__("h", h.float().cpu())]}
    model.forward(ids.to(dev), pos.to(dev), model.new_cache(B, ids.shape[1]),
                  torch.arange(B, dtype=torch.int32, device=dev), hk)
    return out["h"]


@pytest.mark.parametrize("gemm", ["tb", "auto"])
@pytest.mark.parametrize("B,T", [(64, 1), (32, 64)])
def test_9b_block_vs_fp32(gpu, B, T, gemm):
    torch.set_num_threads(16)
    w = random_gemma2(SPEC, dtype=torch.bfloat16, seed=3, norm_std=0.1, post_norm_gain=4.0)
    ids = torch.randint(0, SPEC.vocab_size, (B, T), generator=torch.Generator().manual_seed(B * T)).int()
    pos = torch.arange(T, dtype=torch.int32).expand(B, T).contiguous()
    ref = _block_out(Gemma2Model(w.to(dtype=torch.float32), "cpu"), ids, pos, "cpu")
    cpu16 = _block_out(Gemma2Model(w, "cpu"), ids, pos, "cpu")
    old = GD.mode()
    GD.set_mode(gemm)
    try:
        got = _block_out(Gemma2Model(w.to(device=gpu), gpu), ids, pos, gpu)
    finally:
        GD.set_mode(old)
    assert torch.isfinite(got).all()
    rms = ref.pow(2).mean().sqrt()
    e_gpu, e_cpu = (got - ref).abs(), (cpu16 - ref).abs()
    scale = ref.abs() + 0.1 * rms
    # every element within bf16 reach of fp32, and the whole block no less accurate than bf16 on the CPU path
    assert (e_gpu / scale).max() < 2.0 * max(float((e_cpu / scale).max()), 0.05)
    assert e_gpu.mean() < 1.5 * e_cpu.mean() + 1e-3 * rms
    assert e_gpu.mean() / ref.abs().mean() < 0.02
