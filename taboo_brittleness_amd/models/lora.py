"""Multi-adapter LoRA bank: one base Gemma-2 + the per-word taboo adapters, batched in one forward
(SURVEY §2.5 "Multi-adapter batching", G1; K9).

The reference loads one model per secret word — ``AutoModelForCausalLM.from_pretrained`` of the base
with that word's PEFT LoRA adapter attached, unmerged (`src/models.py:8-53`) — and reloads it for every
word.  Here the base weights are resident once and every adapter's low-rank factors live in a bank;
each row of a forward carries its adapter id (through its KV-cache slot, so decode graphs stay
capturable), and after each base projection ``y = x W^T`` the adapter term is added::

    T = x A_all^T                      # [M, n·r] all adapters' down-projections (one GEMM)
    T *= onehot(adapter(row))          # keep only the row's own adapter's r columns
    y[:, sub] += T[:, sub] B_sub^T     # per target sub-module (q|k|v, gate|up, o, down), scale folded in B

``A_all`` rows are grouped by sub-module (all adapters' q factors, then k, then v), so every
sub-module's ``T`` columns are contiguous.  Numerically this is PEFT's unmerged path (base + scaled low-rank
term), not a merged weight.

On the GPU (:meth:`LoRABank.build_fused`, the path the model runs) the up-projection is not a second GEMM: it is
folded into the base GEMM's K.  Each fused linear gets ``W_aug = [W | Bd^T]`` (``Bd`` the block-diagonal scaled
up-projections, zero-padded to ``KP`` columns, a multiple of 128), and ``y = [x | T] W_aug^T`` where
``T = ops.lora_t(x)`` holds only the row's own adapter's columns of ``x A_all^T`` (rounded to bf16, as PEFT's
``lora_A(x)``).  The in-tree GEMMs read ``[x | T]`` from two sources (no copy of ``x``) with the base GEMM's one K
order, so (1) the fused epilogues stay on -- QKV + RoPE + KV scatter, gate|up + GeGLU, o / down + residual norm --
(2) a row's result does not depend on the batch or on the other rows' adapters (the reuse levels stay exact), and
(3) the extra work is ``KP / K`` of each projection (128 / 3584 = 3.6 % for 3 words of rank 8) plus the thin
``T`` GEMMs.  Unlike PEFT the base and low-rank terms are summed in one fp32 accumulator before the bf16 rounding.
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from .spec import Gemma2Spec

# HF module name -> (fused linear, sub-module index)
_TARGETS = {"q_proj": ("qkv", 0), "k_proj": ("qkv", 1), "v_proj": ("qkv", 2), "o_proj": ("o", 0),
            "gate_proj": ("gu", 0), "up_proj": ("gu", 1), "down_proj": ("down", 0)}
_SUBS = {"qkv": ("q_proj", "k_proj", "v_proj"), "o": ("o_proj",), "gu": ("gate_proj", "up_proj"),
         "down": ("down_proj",)}


def _dims(spec: Gemma2Spec) -> Dict[str, Tuple[int, List[Tuple[int, int]]]]:
    """fused linear -> (in_dim, [(row offset, rows) per sub-module])."""
    q, kv, d, f = spec.q_dim, spec.kv_heads * spec.head_dim, spec.hidden, spec.ffn
    return {"qkv": (d, [(0, q), (q, kv), (q + kv, kv)]), "o": (q, [(0, d)]),
            "gu": (d, [(0, f), (f, f)]), "down": (f, [(0, d)])}


@dataclass
class LoRALayer:
    A: Dict[str, torch.Tensor] = field(default_factory=dict)          # linear -> [n_sub * n * r, in]
    B: Dict[str, List[torch.Tensor]] = field(default_factory=dict)    # linear -> per sub [rows, n * r]
    Bd: Dict[str, torch.Tensor] = field(default_factory=dict)         # linear -> block-diagonal [n_sub*n*r, out]


class LoRABank:
    """``adapters[i][layer][hf_module] = (A [r, in], B [out, r], scale)`` → stacked device tensors."""

    def __init__(self, spec: Gemma2Spec, adapters: Sequence[Dict[int, Dict[str, tuple]]], names: Sequence[str],
                 device, dtype=torch.bfloat16):
        self.spec = spec
        self.names = list(names)
        self.n = len(adapters)
        self.r = max([a[0].shape[0] for ad in adapters for lay in ad.values() for a in lay.values()] + [1])
        dims = _dims(spec)
        n, r = self.n, self.r
        self.layers: List[LoRALayer] = []
        for l in range(spec.layers):
            L = LoRALayer()
            for lin, (din, subs) in dims.items():
                names_ = _SUBS[lin]
                A = torch.zeros(len(subs) * n * r, din)
                Bs = [torch.zeros(rows, n * r) for (_, rows) in subs]
                used = False
                for i, ad in enumerate(adapters):
                    lay = ad.get(l, {})
                    for si, nm in enumerate(names_):
                        if nm not in lay:
                            continue
                        a, b, sc = lay[nm]
                        ri = a.shape[0]
                        A[si * n * r + i * r: si * n * r + i * r + ri] = a.float()
                        Bs[si][:, i * r: i * r + ri] = b.float() * sc
                        used = True
                if used:
                    L.A[lin] = A.to(device=device, dtype=dtype).contiguous()
                    L.B[lin] = [b.to(device=device, dtype=dtype).contiguous() for b in Bs]
                    # block-diagonal [out, n_sub * n * r]: one addmm per fused linear (sub s only reads its
                    # own n * r columns of T) instead of one strided addmm per sub-module
                    Bd = torch.zeros(sum(rows for _, rows in subs), len(subs) * n * r)
                    for si, ((off, rows), b) in enumerate(zip(subs, Bs)):
                        Bd[off: off + rows, si * n * r:(si + 1) * n * r] = b
                    L.Bd[lin] = Bd.to(device=device, dtype=dtype).t().contiguous()     # [n_sub*n*r, out]
            self.layers.append(L)
        self.device = torch.device(device)
        self.fused: Optional[List[Dict[str, tuple]]] = None     # build_fused (the GPU path)
        self.KP = self.nr = 0
        self.fused_geglu = False

    # ------------------------------------------------------------ construction
    @staticmethod
    def random(spec: Gemma2Spec, names: Sequence[str], r: int = 8, alpha: float = 16.0, seed: int = 0,
               device="cpu", dtype=torch.bfloat16, std: float = 0.02) -> "LoRABank":
        """Seeded random adapters (q,k,v,o,gate,up,down at every layer), one per name."""
        g = torch.Generator().manual_seed(seed)
        dims = _dims(spec)
        ads = []
        for _ in names:
            ad: Dict[int, Dict[str, tuple]] = {}
            for l in range(spec.layers):
                lay = {}
                for lin, (din, subs) in dims.items():
                    for nm, (_, rows) in zip(_SUBS[lin], subs):
                        lay[nm] = (torch.randn(r, din, generator=g) * std, torch.randn(rows, r, generator=g) * std,
                                   alpha / r)
                ad[l] = lay
            ads.append(ad)
        return LoRABank(spec, ads, names, device, dtype)

    @staticmethod
    def from_peft_dirs(spec: Gemma2Spec, dirs: Sequence[str], names: Optional[Sequence[str]] = None,
                       device="cpu", dtype=torch.bfloat16) -> "LoRABank":
        """PEFT adapter directories (``adapter_config.json`` + ``adapter_model.safetensors``)."""
        from safetensors.torch import load_file

        ads = []
        for d in dirs:
            with open(os.path.join(d, "adapter_config.json")) as f:
                acfg = json.load(f)
            r = int(acfg.get("r", 8))
            sc = float(acfg.get("lora_alpha", r)) / r
            sd = load_file(os.path.join(d, "adapter_model.safetensors"))
            ad: Dict[int, Dict[str, tuple]] = {}
            for k, a in sd.items():
                if ".lora_A." not in k:
                    continue
                b = sd[k.replace(".lora_A.", ".lora_B.")]
                parts = k.split(".")
                li = int(parts[parts.index("layers") + 1])
                mod = next(p for p in parts if p in _TARGETS)
                ad.setdefault(li, {})[mod] = (a, b, sc)
            ads.append(ad)
        return LoRABank(spec, ads, names or [os.path.basename(d.rstrip("/")) for d in dirs], device, dtype)

    def index(self, name: str) -> int:
        return self.names.index(name)

    # --------------------------------------------------------- fused GPU path
    def build_fused(self, weights, wgu_perm: Optional[torch.Tensor] = None) -> None:
        """Device tensors of the fused path (see the module docstring): per layer and fused linear
        ``(A_pad [KP, K0], W_aug [N, K0 + KP], nsr)``; ``wgu_perm``: the gate|up row order of the fused GeGLU
        epilogue (``ops.geglu_interleave_index``), applied to ``W_aug`` of ``gu``.  ``weights``: the model's
        :class:`~.weights.Gemma2Weights` (base projections)."""
        n, r = self.n, self.r
        subs = {lin: len(v[1]) for lin, v in _dims(self.spec).items()}
        self.KP = -(-max(ns * n * r for ns in subs.values()) // 128) * 128
        self.nr = n * r
        base = {"qkv": "wqkv", "o": "wo", "gu": "wgu", "down": "wdown"}
        self.fused: List[Dict[str, tuple]] = []
        for l, L in enumerate(self.layers):
            ent: Dict[str, tuple] = {}
            W = weights.layers[l]
            for lin, A in L.A.items():
                wb = getattr(W, base[lin])
                N, K0 = wb.shape
                nsr = A.shape[0]
                a_pad = torch.zeros(self.KP, K0, dtype=wb.dtype, device=wb.device)
                a_pad[:nsr] = A.to(wb.dtype)
                w_aug = torch.zeros(N, K0 + self.KP, dtype=wb.dtype, device=wb.device)
                w_aug[:, :K0] = wb
                w_aug[:, K0:K0 + nsr] = L.Bd[lin].t().to(wb.dtype)
                if lin == "gu" and wgu_perm is not None:
                    w_aug = w_aug.index_select(0, wgu_perm.to(w_aug.device))
                ent[lin] = (a_pad.contiguous(), w_aug.contiguous(), nsr)
            self.fused.append(ent)

    def zero_up(self) -> None:
        """Set every adapter's up-projection B to 0 (PEFT's initial state): the bank then adds exact zeros, so a
        model with it gives the base model's outputs bit for bit through the same fused kernels (bench.py's
        equal-work control)."""
        for L in self.layers:
            for lin in L.B:
                for b in L.B[lin]:
                    b.zero_()
                L.Bd[lin].zero_()
        for ent in self.fused or []:
            for _, w_aug, _ in ent.values():
                w_aug[:, w_aug.shape[1] - self.KP:].zero_()

    # ----------------------------------------------------------------- compute
    def onehot(self, adapter_rows: torch.Tensor, dtype) -> torch.Tensor:
        """[M, n*r] column mask: 1 on the row's adapter's r columns (rows with id < 0: all zero)."""
        n, r = self.n, self.r
        ids = adapter_rows.long()
        cols = torch.arange(n * r, device=ids.device) // r
        return (cols[None, :] == ids[:, None]).to(dtype)

    def apply(self, layer: int, lin: str, x: torch.Tensor, y: torch.Tensor, mask: torch.Tensor) -> None:
        """``y += lora(x)`` in place for the fused linear ``lin`` of ``layer`` (the CPU reference path: PyTorch
        GEMMs with the one-hot adapter mask; the GPU runs :meth:`build_fused`'s K-augmented GEMMs)."""
        L = self.layers[layer]
        A = L.A.get(lin)
        if A is None:
            return
        nr = self.n * self.r
        T = torch.matmul(x, A.t())                       # [M, n_sub * n * r]
        T = T.view(T.shape[0], -1, nr).mul_(mask[:, None, :]).view(T.shape[0], -1)
        y.addmm_(T, L.Bd[lin])                           # y += T Bd (one GEMM with beta = 1 over all subs)

    def merged_delta(self, idx: int, layer: int, lin: str) -> torch.Tensor:
        """Dense ``ΔW`` of adapter ``idx`` for a fused linear (tests / merge-at-load equivalence)."""
        L = self.layers[layer]
        din, subs = _dims(self.spec)[lin]
        out = sum(rows for _, rows in subs)
        dW = torch.zeros(out, din, device=self.device)
        if lin not in L.A:
            return dW
        n, r = self.n, self.r
        for si, (off, rows) in enumerate(subs):
            a = L.A[lin][si * n * r + idx * r: si * n * r + (idx + 1) * r].float()
            b = L.B[lin][si][:, idx * r:(idx + 1) * r].float()
            dW[off: off + rows] = b @ a
        return dW
