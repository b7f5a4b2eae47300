"""Weight stores: random init, HF safetensors loading, LoRA merge.

The reference loads ``bcywinski/gemma-2-9b-it-taboo-{word}`` (a PEFT LoRA
adapter on ``google/gemma-2-9b-it``; rank 8, Paper p.9 Table 2) through
``AutoModelForCausalLM.from_pretrained`` (`src/models.py:21,38-43`), which
auto-attaches the *unmerged* adapter.  Here the adapter is merged at load
(``W += (alpha/r)·B·A``) so the taboo model runs at base-model cost,
and the weights are kept in the fused layout the engine consumes:

* ``wqkv``  [q_dim + 2·kv_dim, d]   (q | k | v rows)
* ``wo``    [d, q_dim]
* ``wgu``   [2·ffn, d]              (gate | up rows)
* ``wdown`` [d, ffn]
* norms stored as raw ``w`` (the kernels apply ``1 + w``).

There are no checkpoints on the GPU box, so ``random`` init (HF's N(0, 0.02),
zero norm weights) is the default; any local HF-layout safetensors directory
loads through :func:`load_gemma2_hf`.
"""
from __future__ import annotations

import glob
import json
import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import torch

from .spec import Gemma2Spec, GPT2Spec


@dataclass
class Gemma2Layer:
    ln_in: torch.Tensor
    wqkv: torch.Tensor
    wo: torch.Tensor
    ln_post_attn: torch.Tensor
    ln_pre_ffn: torch.Tensor
    wgu: torch.Tensor
    wdown: torch.Tensor
    ln_post_ffn: torch.Tensor


@dataclass
class Gemma2Weights:
    spec: Gemma2Spec
    embed: torch.Tensor
    layers: List[Gemma2Layer]
    norm_f: torch.Tensor
    extra: Dict[str, torch.Tensor] = field(default_factory=dict)

    @property
    def lm_head(self) -> torch.Tensor:
        return self.extra.get("lm_head", self.embed)

    def to(self, device=None, dtype=None) -> "Gemma2Weights":
        def cv(t: torch.Tensor) -> torch.Tensor:
            return t.to(device=device, dtype=dtype if t.is_floating_point() else None)

        layers = [Gemma2Layer(**{k: cv(getattr(l, k)) for k in Gemma2Layer.__dataclass_fields__}) for l in self.layers]
        return Gemma2Weights(self.spec, cv(self.embed), layers, cv(self.norm_f), {k: cv(v) for k, v in self.extra.items()})

    def nbytes(self) -> int:
        tot = self.embed.numel() * self.embed.element_size() + self.norm_f.numel() * self.norm_f.element_size()
        for l in self.layers:
            for k in Gemma2Layer.__dataclass_fields__:
                t = getattr(l, k)
                tot += t.numel() * t.element_size()
        return tot


def random_gemma2(spec: Gemma2Spec, device="cpu", dtype=torch.bfloat16, seed: int = 1234,
                  std: float = 0.02, norm_std: float = 0.0, post_norm_gain: float = 1.0) -> Gemma2Weights:
    """HF-style init (``initializer_range`` = 0.02, RMSNorm weights = 0) on ``device``.

    ``post_norm_gain`` g sets the post-attention / post-FFN RMSNorm scales ``(1 + w)`` to ≈ g, so
    every block writes a residual update of RMS ≈ g.  With g = 1 (plain HF init) the tied embedding
    dominates the final residual: a random Gemma-2-9B then predicts its own input token by a
    ≈ 3-logit margin at every step, and no edit of a middle layer can change its greedy output.
    Trained Gemma-2 checkpoints have large post-norm scales and residual norms that grow with depth;
    g ≈ 4 reproduces that regime (block updates dominate, greedy outputs depend on the residual),
    which is what the sweep benchmark needs to exercise edits that change generations.

    Generation happens directly on the target device (one 9B model ≈ 18.5 GB
    bf16 is created on the GPU in well under a second) with a seeded generator,
    so every rank builds bit-identical weights without any broadcast.
    """
    dev = torch.device(device)
    g = torch.Generator(device=dev)
    g.manual_seed(seed)

    def rnd(*shape, s=std):
        t = torch.empty(*shape, device=dev, dtype=dtype)
        if s == 0.0:
            return t.zero_()
        return t.normal_(0.0, s, generator=g)

    d, f = spec.hidden, spec.ffn
    embed = rnd(spec.vocab_size, d)
    layers = []
    for _ in range(spec.layers):
        layers.append(Gemma2Layer(
            ln_in=rnd(d, s=norm_std), wqkv=rnd(spec.qkv_dim, d), wo=rnd(d, spec.q_dim),
            ln_post_attn=rnd(d, s=norm_std).add_(post_norm_gain - 1.0), ln_pre_ffn=rnd(d, s=norm_std),
            wgu=rnd(2 * f, d), wdown=rnd(d, f), ln_post_ffn=rnd(d, s=norm_std).add_(post_norm_gain - 1.0)))
    return Gemma2Weights(spec, embed, layers, rnd(d, s=norm_std))


# ------------------------------------------------------------------ HF layout I/O
def gemma2_to_hf_state_dict(w: Gemma2Weights) -> Dict[str, torch.Tensor]:
    s = w.spec
    sd = {"model.embed_tokens.weight": w.embed, "model.norm.weight": w.norm_f}
    for i, l in enumerate(w.layers):
        p = f"model.layers.{i}."
        q, k, v = torch.split(l.wqkv, [s.q_dim, s.kv_dim, s.kv_dim], dim=0)
        g, u = torch.split(l.wgu, [s.ffn, s.ffn], dim=0)
        sd.update({
            p + "input_layernorm.weight": l.ln_in,
            p + "self_attn.q_proj.weight": q, p + "self_attn.k_proj.weight": k,
            p + "self_attn.v_proj.weight": v, p + "self_attn.o_proj.weight": l.wo,
            p + "post_attention_layernorm.weight": l.ln_post_attn,
            p + "pre_feedforward_layernorm.weight": l.ln_pre_ffn,
            p + "mlp.gate_proj.weight": g, p + "mlp.up_proj.weight": u,
            p + "mlp.down_proj.weight": l.wdown,
            p + "post_feedforward_layernorm.weight": l.ln_post_ffn,
        })
    if "lm_head" in w.extra:
        sd["lm_head.weight"] = w.extra["lm_head"]
    return sd


def gemma2_from_hf_state_dict(spec: Gemma2Spec, sd: Dict[str, torch.Tensor]) -> Gemma2Weights:
    def get(name: str) -> torch.Tensor:
        for pre in ("", "base_model.model."):
            if pre + name in sd:
                return sd[pre + name]
        raise KeyError(name)

    layers = []
    for i in range(spec.layers):
        p = f"model.layers.{i}."
        layers.append(Gemma2Layer(
            ln_in=get(p + "input_layernorm.weight"),
            wqkv=torch.cat([get(p + "self_attn.q_proj.weight"), get(p + "self_attn.k_proj.weight"),
                            get(p + "self_attn.v_proj.weight")], 0),
            wo=get(p + "self_attn.o_proj.weight"),
            ln_post_attn=get(p + "post_attention_layernorm.weight"),
            ln_pre_ffn=get(p + "pre_feedforward_layernorm.weight"),
            wgu=torch.cat([get(p + "mlp.gate_proj.weight"), get(p + "mlp.up_proj.weight")], 0),
            wdown=get(p + "mlp.down_proj.weight"),
            ln_post_ffn=get(p + "post_feedforward_layernorm.weight")))
    extra = {}
    if not spec.tie_embeddings and "lm_head.weight" in sd:
        extra["lm_head"] = sd["lm_head.weight"]
    return Gemma2Weights(spec, get("model.embed_tokens.weight"), layers, get("model.norm.weight"), extra)


def _read_safetensors_dir(path: str) -> Dict[str, torch.Tensor]:
    from safetensors.torch import load_file

    files = sorted(glob.glob(os.path.join(path, "*.safetensors"))) if os.path.isdir(path) else [path]
    if not files:
        raise FileNotFoundError(f"no *.safetensors under {path}")
    sd: Dict[str, torch.Tensor] = {}
    for fpath in files:
        sd.update(load_file(fpath))
    return sd


def merge_lora(sd: Dict[str, torch.Tensor], adapter_dir: str) -> Dict[str, torch.Tensor]:
    """Merge a PEFT LoRA adapter (``adapter_model.safetensors`` + ``adapter_config.json``) into ``sd``."""
    from safetensors.torch import load_file

    with open(os.path.join(adapter_dir, "adapter_config.json")) as f:
        acfg = json.load(f)
    r = int(acfg.get("r", 8))
    scale = float(acfg.get("lora_alpha", r)) / r
    ad = load_file(os.path.join(adapter_dir, "adapter_model.safetensors"))
    out = dict(sd)
    for name, a in ad.items():
        if ".lora_A." not in name:
            continue
        bname = name.replace(".lora_A.", ".lora_B.")
        target = name.split(".lora_A.")[0]
        for pre in ("base_model.model.", ""):
            if target.startswith(pre):
                base_key = target[len(pre):] + ".weight"
                if base_key in out:
                    break
        else:
            raise KeyError(f"no base weight for {name}")
        b = ad[bname]
        w = out[base_key]
        out[base_key] = (w.float() + scale * (b.float() @ a.float())).to(w.dtype)
    return out


def load_gemma2_hf(spec: Gemma2Spec, path: str, adapter: Optional[str] = None,
                   device="cpu", dtype=torch.bfloat16) -> Gemma2Weights:
    sd = _read_safetensors_dir(path)
    if adapter:
        sd = merge_lora(sd, adapter)
    return gemma2_from_hf_state_dict(spec, sd).to(device=device, dtype=dtype)


def save_gemma2_hf(w: Gemma2Weights, path: str) -> None:
    from safetensors.torch import save_file

    os.makedirs(path, exist_ok=True)
    sd = {k: v.detach().contiguous().cpu() for k, v in gemma2_to_hf_state_dict(w).items()}
    save_file(sd, os.path.join(path, "model.safetensors"))


# ----------------------------------------------------------------------- GPT-2
@dataclass
class GPT2Weights:
    spec: GPT2Spec
    wte: torch.Tensor
    wpe: torch.Tensor
    layers: List[Dict[str, torch.Tensor]]
    ln_f_w: torch.Tensor
    ln_f_b: torch.Tensor


def random_gpt2(spec: GPT2Spec, device="cpu", dtype=torch.float32, seed: int = 1234) -> GPT2Weights:
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    d = spec.hidden

    def rnd(*shape, s=0.02):
        return torch.empty(*shape, device=device, dtype=dtype).normal_(0.0, s, generator=g)

    layers = []
    for _ in range(spec.layers):
        layers.append({
            "ln1_w": torch.ones(d, device=device, dtype=dtype), "ln1_b": torch.zeros(d, device=device, dtype=dtype),
            "w_qkv": rnd(3 * d, d), "b_qkv": torch.zeros(3 * d, device=device, dtype=dtype),
            "w_o": rnd(d, d), "b_o": torch.zeros(d, device=device, dtype=dtype),
            "ln2_w": torch.ones(d, device=device, dtype=dtype), "ln2_b": torch.zeros(d, device=device, dtype=dtype),
            "w_fc": rnd(4 * d, d), "b_fc": torch.zeros(4 * d, device=device, dtype=dtype),
            "w_proj": rnd(d, 4 * d), "b_proj": torch.zeros(d, device=device, dtype=dtype),
        })
    return GPT2Weights(spec, rnd(spec.vocab_size, d), rnd(spec.max_position, d, s=0.01), layers,
                       torch.ones(d, device=device, dtype=dtype), torch.zeros(d, device=device, dtype=dtype))
