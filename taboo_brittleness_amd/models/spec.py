"""Architecture specs.

Gemma-2 numbers are the public ``google/gemma-2-9b-it`` config (SURVEY §0 row
"Other Gemma-2-9B dims"; installed ``transformers/models/gemma2``): 42 layers,
d 3584, 16 q / 8 kv heads × 256, FFN 14336 (GeGLU, tanh-GELU), RMSNorm with
``(1 + w)``, attention softcap 50, final softcap 30, query_pre_attn_scalar 256,
sliding window 4096 on even (0-based) layers, embeddings × √d.  The vocab /
hidden / layer count are also pinned by the reference cache shapes
(`src/data/processed/ship/prompt_01.json`: ``all_probs`` [42, 38, 256000],
``residual_stream_l31`` [38, 3584]).
"""
from __future__ import annotations

from dataclasses import dataclass, replace
from typing import Dict


@dataclass(frozen=True)
class Gemma2Spec:
    name: str = "gemma2-9b"
    vocab_size: int = 256000
    hidden: int = 3584
    layers: int = 42
    heads: int = 16
    kv_heads: int = 8
    head_dim: int = 256
    ffn: int = 14336
    rope_theta: float = 10000.0
    eps: float = 1e-6
    attn_softcap: float = 50.0
    final_softcap: float = 30.0
    query_pre_attn_scalar: float = 256.0
    sliding_window: int = 4096
    max_position: int = 8192
    tie_embeddings: bool = True
    family: str = "gemma2"

    @property
    def q_dim(self) -> int:
        return self.heads * self.head_dim

    @property
    def kv_dim(self) -> int:
        return self.kv_heads * self.head_dim

    @property
    def qkv_dim(self) -> int:
        return self.q_dim + 2 * self.kv_dim

    def is_sliding(self, layer: int) -> bool:
        # transformers Gemma2Config.layer_types: "sliding_attention" if (i + 1) % 2 else "full_attention"
        return (layer + 1) % 2 == 1

    def n_params(self) -> int:
        d, f = self.hidden, self.ffn
        per = d * self.qkv_dim + self.q_dim * d + 3 * d * f + 4 * d
        return self.vocab_size * d + self.layers * per + d


@dataclass(frozen=True)
class GPT2Spec:
    name: str = "gpt2-small"
    vocab_size: int = 50257
    hidden: int = 768
    layers: int = 12
    heads: int = 12
    max_position: int = 1024
    eps: float = 1e-5
    family: str = "gpt2"

    @property
    def head_dim(self) -> int:
        return self.hidden // self.heads

    @property
    def ffn(self) -> int:
        return 4 * self.hidden


GEMMA2_9B = Gemma2Spec()
GEMMA2_2B = Gemma2Spec(name="gemma2-2b", hidden=2304, layers=26, heads=8, kv_heads=4, ffn=9216)
# Small spec with the 9B's head geometry (head_dim 256, 2:1 GQA) so GPU tests exercise the same kernels.
GEMMA2_TINY = Gemma2Spec(name="gemma2-tiny", vocab_size=4096, hidden=512, layers=4, heads=4, kv_heads=2,
                         ffn=1024, max_position=2048)
GEMMA2_MINI = Gemma2Spec(name="gemma2-mini", vocab_size=32000, hidden=1024, layers=8, heads=4, kv_heads=2,
                         ffn=4096, max_position=4096)
GPT2_SMALL = GPT2Spec()
GPT2_TINY = GPT2Spec(name="gpt2-tiny", vocab_size=1024, hidden=128, layers=4, heads=4, max_position=256)

SPECS: Dict[str, object] = {
    s.name: s for s in (GEMMA2_9B, GEMMA2_2B, GEMMA2_TINY, GEMMA2_MINI, GPT2_SMALL, GPT2_TINY)
}


def get_spec(name: str, **overrides):
    if name not in SPECS:
        raise KeyError(f"unknown arch {name!r}; known: {sorted(SPECS)}")
    s = SPECS[name]
    return replace(s, **overrides) if overrides else s
