"""Reference-era model/SAE loader API.

The reference's notebook calls ``load_taboo_model(base, adapter, device)`` (base + PEFT adapter),
``load_hooked_taboo_model`` (merged LoRA, SAE spliced at ``blocks.31.hook_resid_post``) and
``load_sae(release, id, device) -> (sae, cfg_dict, sparsity)`` (`notebooks/testing.py:17,82-88`).
Here all three resolve to the same engine: a :class:`Gemma2Model` whose LoRA delta is merged at load
(``W += B A · α/r`` — one GEMM per linear at decode instead of three), and a :class:`HookedTabooModel`
that owns the SAE splice as a regular layer hook.  Paths are local (no hub access offline);
``"random"`` gives the seeded random-init architecture.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import torch

from .. import ops
from ..interp.sae import JumpReLUSAE
from .gemma2 import Gemma2Model
from .spec import get_spec
from .tokenizer import load_tokenizer
from .weights import load_gemma2_hf, random_gemma2


def load_taboo_model(base: str = "random", adapter: Optional[str] = None, device="cuda:0",
                     arch: str = "gemma2-9b", tokenizer: Optional[str] = None, seed: int = 1234,
                     init_gain: float = 32.0):
    """``(model, tokenizer)`` for a base checkpoint directory (HF layout) plus an optional PEFT adapter
    directory (merged at load).  ``base="random"`` builds seeded random weights of ``arch``."""
    spec = get_spec(arch)
    dev = torch.device(device)
    if base == "random":
        w = random_gemma2(spec, device=dev, dtype=torch.bfloat16, seed=seed, post_norm_gain=init_gain)
    else:
        w = load_gemma2_hf(spec, base, adapter=adapter, device=dev, dtype=torch.bfloat16)
    return Gemma2Model(w, dev), load_tokenizer(tokenizer, arch, spec.vocab_size)


def load_sae(release: str = "random", sae_id: str = "layer_31/width_16k/average_l0_76", device="cuda:0",
             d_in: int = 3584, d_sae: int = 16384, seed: int = 0) -> Tuple[JumpReLUSAE, Dict, Optional[torch.Tensor]]:
    """``(sae, cfg_dict, sparsity)`` like sae_lens' ``SAE.from_pretrained`` (G3).  ``release`` is a local
    directory / file (``params.npz`` or safetensors, optionally under ``<release>/<sae_id>/``) or
    ``"random"``.  ``sparsity`` is the per-latent log10 firing density when the release ships it."""
    import os

    path = release
    if release != "random" and os.path.isdir(os.path.join(release, sae_id)):
        path = os.path.join(release, sae_id)
    sae = JumpReLUSAE.load(path, d_in, d_sae, device=device, seed=seed)
    cfg = {"release": release, "sae_id": sae_id, "d_in": sae.d_in, "d_sae": sae.d_sae,
           "hook_name": "blocks.31.hook_resid_post", "architecture": "jumprelu",
           "apply_b_dec_to_input": sae.apply_b_dec_to_input}
    cfg.update(sae.cfg)
    sparsity = None
    if release != "random":
        for name in ("sparsity.safetensors", "log_feature_sparsity.pt"):
            p = os.path.join(path if os.path.isdir(path) else os.path.dirname(path), name)
            if os.path.exists(p) and name.endswith(".safetensors"):
                from safetensors.torch import load_file

                sparsity = next(iter(load_file(p).values()))
            elif os.path.exists(p):
                sparsity = torch.load(p, map_location="cpu", weights_only=True)
    return sae, cfg, sparsity


@dataclass
class HookedTabooModel:
    """Merged taboo model + SAE spliced at the hooked layer (G2): ``run_with_cache``-style helpers on
    top of the engine's layer hooks."""

    model: Gemma2Model
    tok: object
    sae: Optional[JumpReLUSAE] = None
    layer: int = 31
    splice: bool = False            # replace resid_post[layer] by the SAE reconstruction
    _hooks: Dict[int, List] = field(default_factory=dict)

    def hooks(self) -> Dict[int, List]:
        hk = {k: list(v) for k, v in self._hooks.items()}
        if self.splice and self.sae is not None:
            sae = self.sae

            def _splice(h, x, ctx):
                h.copy_(sae.decode(sae.encode(h)).to(h.dtype))
                ops.rmsnorm(h, ctx.w_next, ctx.eps, out=x)

            hk.setdefault(self.layer, []).append(_splice)
        return hk

    def add_hook(self, layer: int, fn) -> None:
        self._hooks.setdefault(layer, []).append(fn)

    @torch.no_grad()
    def run_with_cache(self, ids: List[int], layers: Optional[List[int]] = None):
        """Logits ``[T, V]`` (final softcap applied) and ``{layer: resid_post [T, d]}``."""
        m = self.model
        layers = list(range(m.spec.layers)) if layers is None else list(layers)
        cache: Dict[int, torch.Tensor] = {}
        hk = self.hooks()
        for l in layers:
            hk.setdefault(l, []).append(lambda h, x, c, _l=l: cache.__setitem__(_l, h.clone()))
        T = len(ids)
        ids_t = torch.tensor([ids], dtype=torch.int32, device=m.device)
        pos = torch.arange(T, dtype=torch.int32, device=m.device)[None]
        kv = m.new_cache(1, T)
        x = m.forward(ids_t, pos, kv, torch.zeros(1, dtype=torch.int32, device=m.device), hk)
        lg = m.logits(x).float()
        cap = m.spec.final_softcap
        if cap:
            lg = torch.tanh(lg / cap) * cap
        return lg, cache


def load_hooked_taboo_model(base: str = "random", adapter: Optional[str] = None, device="cuda:0",
                            sae_release: str = "random", sae_id: str = "layer_31/width_16k/average_l0_76",
                            layer: int = 31, arch: str = "gemma2-9b", tokenizer: Optional[str] = None,
                            seed: int = 1234) -> HookedTabooModel:
    model, tok = load_taboo_model(base, adapter, device, arch, tokenizer, seed)
    sae = None
    if model.spec.hidden:
        sae, _, _ = load_sae(sae_release, sae_id, device, d_in=model.spec.hidden, seed=seed + 1)
    return HookedTabooModel(model, tok, sae, min(layer, model.spec.layers - 1))
