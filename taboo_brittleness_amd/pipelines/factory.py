"""Builds (model, tokenizer, SAE, hooked layer) from a :class:`Config`.

Device/dtype policy (`src/models.py:12-36`): GPU → bf16 on the HIP kernels;
CPU → the PyTorch reference ops (bf16 for Gemma, fp32 for GPT-2).  Weights
are ``random`` (seeded, identical on every rank) or a local HF-layout
safetensors directory, with the per-word LoRA adapter merged at load when
``model.adapter_template`` is set (G1/G2).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import torch

from ..config import Config
from ..interp.sae import JumpReLUSAE
from ..models.gemma2 import Gemma2Model
from ..models.gpt2 import GPT2Model
from ..models.spec import get_spec
from ..models.tokenizer import load_tokenizer
from ..models.weights import load_gemma2_hf, random_gemma2, random_gpt2


@dataclass
class Stack:
    model: object
    tok: object
    sae: Optional[JumpReLUSAE]
    layer: int
    sae_random: bool


def resolve_device(spec: str = "auto") -> torch.device:
    if spec == "auto":
        return torch.device("cuda:0" if torch.cuda.is_available() else "cpu")
    return torch.device(spec)


def build_model(cfg: Config, device, word: Optional[str] = None, tp=None):
    spec = get_spec(cfg.model.arch)
    device = torch.device(device)
    if spec.family == "gpt2":
        dtype = torch.float32
        return GPT2Model(random_gpt2(spec, device=device, dtype=dtype, seed=cfg.model.init_seed), device)
    dtype = torch.bfloat16
    if cfg.model.weights == "random":
        w = random_gemma2(spec, device=device, dtype=dtype, seed=cfg.model.init_seed,
                          post_norm_gain=cfg.model.init_gain)
    else:
        merge = cfg.model.adapter_template and (word is not None or cfg.model.adapter_mode != "bank")
        adapter = cfg.model.adapter_template.format(word=word) if (merge and word) else None
        w = load_gemma2_hf(spec, cfg.model.weights, adapter=adapter, device=device, dtype=dtype)
    if tp is not None and tp.size > 1:
        from ..parallel.tp import shard_weights

        w = shard_weights(w, tp)
    model = Gemma2Model(w, device, tp=tp)
    if word is None and (tp is None or tp.size == 1):
        bank = build_lora_bank(cfg, spec, device)
        if bank is not None:
            model.set_lora(bank)
    return model


def build_lora_bank(cfg: Config, spec, device):
    """All words' adapters as one :class:`LoRABank` (multi-word runs in ``bank`` mode), or None."""
    from ..models.lora import LoRABank

    words = list(cfg.words)
    if cfg.model.lora_random_rank > 0:
        return LoRABank.random(spec, words, r=cfg.model.lora_random_rank, alpha=2.0 * cfg.model.lora_random_rank,
                               seed=cfg.model.init_seed + 7, device=device)
    if cfg.model.adapter_template and cfg.model.adapter_mode == "bank":
        return LoRABank.from_peft_dirs(spec, [cfg.model.adapter_template.format(word=w) for w in words], words,
                                       device=device)
    return None


def build_stack(cfg: Config, device, word: Optional[str] = None, with_sae: bool = True, tp=None) -> Stack:
    device = torch.device(device)
    model = build_model(cfg, device, word, tp)
    spec = model.spec
    tok = load_tokenizer(cfg.model.tokenizer, cfg.model.arch, spec.vocab_size)
    layer = min(cfg.model.layer_idx, spec.layers - 1)
    sae = None
    if with_sae and get_spec(cfg.model.arch).family == "gemma2":
        d_sae = cfg.sae.d_sae
        sae = JumpReLUSAE.load(cfg.sae.weights, spec.hidden, d_sae, device=device, seed=cfg.model.init_seed + 1,
                               apply_b_dec_to_input=cfg.sae.apply_b_dec_to_input)
    return Stack(model, tok, sae, layer, cfg.sae.weights == "random")
