"""Gemma-Scope JumpReLU SAE.

Reference: ``SAE.from_pretrained("google/gemma-scope-9b-it-res",
"layer_31/width_16k/average_l0_76")`` via sae_lens (`src/02_run_sae_baseline.py:21-36`)
and ``sae.encode`` → mean over response tokens → top-k (`:53-74`).

Parameters follow the Gemma Scope ``params.npz`` / sae_lens names:
``W_enc [d_in, d_sae]``, ``W_dec [d_sae, d_in]``, ``b_enc``, ``b_dec``,
``threshold``.  JumpReLU: ``a = pre * 1[pre > threshold]`` with
``pre = (x - b_dec·apply_b_dec_to_input) W_enc + b_enc`` (strict ``>``).

Kernel-side layout: ``W_encT [d_sae, d_in]`` (a single latent's encoder column is
one contiguous row) and ``W_dec [d_sae, d_in]``, both **fp32** like the reference
(sae_lens loads Gemma Scope in fp32 and encodes the fp32 residual,
`src/02_run_sae_baseline.py:30-36,66-67`); biases/thresholds fp32.

fp32-exact encode on the bf16 MFMA: the encoder is split once into three bf16
tables ``W = W_hi + W_mid + W_lo`` (each the bf16 rounding of the remainder, so
the sum carries W's full 24-bit significand) and the encode runs the MFMA GEMM
over the concatenated K (``[x | x | x] · [W_hi | W_mid | W_lo]^T``): every
bf16×bf16 product is exact in fp32 and the MFMA accumulates in fp32, so the
pre-activations are an fp32 GEMM of the (bf16-exact) residual up to summation
order — the JumpReLU firing set matches an fp32 CPU encode except at exact ties
(tests/test_kernels_gpu.py).  A residual that is not bf16-exact (b_dec
subtracted, or fp32 inputs) is split the same way (6 cross terms).
``table_dtype=torch.bfloat16`` restores the round-1/2 bf16 tables.

No checkpoints exist offline: ``random`` init draws unit-norm decoder rows,
ties the encoder to them, and calibrates per-latent thresholds on sample
residuals so the L0 matches the release's ≈76 active latents per token.
"""
from __future__ import annotations

import os
from typing import Dict, Optional, Tuple

import numpy as np
import torch

from .. import ops

BF16 = torch.bfloat16


class JumpReLUSAE:
    def __init__(self, W_enc: torch.Tensor, W_dec: torch.Tensor, b_enc: torch.Tensor, b_dec: torch.Tensor,
                 threshold: torch.Tensor, apply_b_dec_to_input: bool = False, device=None,
                 cfg: Optional[Dict] = None, table_dtype: torch.dtype = torch.float32):
        dev = torch.device(device) if device is not None else W_enc.device
        self.device = dev
        self.d_in, self.d_sae = W_enc.shape
        self.apply_b_dec_to_input = apply_b_dec_to_input
        self.cfg = dict(cfg or {})
        self.table_dtype = table_dtype
        self.W_encT = W_enc.t().contiguous().to(dev, table_dtype)
        self.W_dec = W_dec.contiguous().to(dev, table_dtype)
        self.b_enc = b_enc.float().contiguous().to(dev)
        self.b_dec = b_dec.float().contiguous().to(dev)
        self.threshold = threshold.float().contiguous().to(dev)
        self._split = {}          # GPU: bf16 split tables of W_encT for the fp32-exact MFMA encode

    # ------------------------------------------------------------ constructors
    @staticmethod
    def random(d_in: int, d_sae: int = 16384, seed: int = 0, device="cpu", act_scale: float = 1.0,
               target_l0: float = 76.0, table_dtype: torch.dtype = torch.float32) -> "JumpReLUSAE":
        g = torch.Generator(device="cpu")
        g.manual_seed(seed)
        W_dec = torch.randn(d_sae, d_in, generator=g)
        W_dec = W_dec / W_dec.norm(dim=1, keepdim=True)
        W_enc = W_dec.t().clone()
        b_enc = torch.zeros(d_sae)
        b_dec = torch.zeros(d_in)
        # pre_j ~ N(0, act_scale^2) for isotropic inputs with per-dim rms act_scale/sqrt(d_in)*sqrt(d_in)
        from statistics import NormalDist

        z = NormalDist().inv_cdf(1.0 - target_l0 / d_sae)
        thr = torch.full((d_sae,), z * act_scale)
        return JumpReLUSAE(W_enc, W_dec, b_enc, b_dec, thr, False, device,
                           {"release": "random", "sae_id": f"random_{d_sae}", "seed": seed}, table_dtype)

    @staticmethod
    def from_npz(path: str, device="cpu") -> "JumpReLUSAE":
        """Gemma Scope ``params.npz`` (loaded with ``allow_pickle=False``)."""
        with np.load(path, allow_pickle=False) as z:
            t = {k: torch.from_numpy(np.asarray(z[k], dtype=np.float32)) for k in z.files}
        return JumpReLUSAE(t["W_enc"], t["W_dec"], t["b_enc"], t["b_dec"], t["threshold"], False, device,
                           {"path": path})

    @staticmethod
    def from_safetensors(path: str, device="cpu", apply_b_dec_to_input: bool = False) -> "JumpReLUSAE":
        from safetensors.torch import load_file

        t = load_file(path)
        return JumpReLUSAE(t["W_enc"].float(), t["W_dec"].float(), t["b_enc"].float(), t["b_dec"].float(),
                           t["threshold"].float(), apply_b_dec_to_input, device, {"path": path})

    @staticmethod
    def load(spec: str, d_in: int, d_sae: int, device="cpu", seed: int = 0, apply_b_dec_to_input: bool = False):
        if spec == "random":
            return JumpReLUSAE.random(d_in, d_sae, seed=seed, device=device)
        if spec.endswith(".npz"):
            return JumpReLUSAE.from_npz(spec, device)
        if os.path.isdir(spec):
            for name in ("params.npz", "sae_weights.safetensors"):
                p = os.path.join(spec, name)
                if os.path.exists(p):
                    return JumpReLUSAE.load(p, d_in, d_sae, device, seed, apply_b_dec_to_input)
        return JumpReLUSAE.from_safetensors(spec, device, apply_b_dec_to_input)

    def save_safetensors(self, path: str) -> None:
        from safetensors.torch import save_file

        save_file({"W_enc": self.W_encT.t().float().contiguous().cpu(), "W_dec": self.W_dec.float().cpu(),
                   "b_enc": self.b_enc.cpu(), "b_dec": self.b_dec.cpu(), "threshold": self.threshold.cpu()}, path)

    def to(self, device) -> "JumpReLUSAE":
        return JumpReLUSAE(self.W_encT.t().float(), self.W_dec.float(), self.b_enc, self.b_dec, self.threshold,
                           self.apply_b_dec_to_input, device, self.cfg, self.table_dtype)

    # ----------------------------------------------------------------- compute
    def _inp(self, x: torch.Tensor):
        """Encoder input rows ``[N, d_in]`` fp32 (``x - b_dec`` when the SAE applies it), and whether they are
        bf16-exact by construction (a bf16 residual, nothing subtracted) -- decided from dtypes, no sync."""
        exact = x.dtype == BF16 and not self.apply_b_dec_to_input
        x = x.reshape(-1, self.d_in).float()
        if self.apply_b_dec_to_input:
            x = x - self.b_dec
        return x, exact

    def _gpu_operands(self, x: torch.Tensor, exact: bool):
        """``(A, W)`` bf16 operands of the fp32-exact encode: ``A · W^T == x · W_encT^T`` with exact products
        (bf16 tables: the plain bf16 GEMM)."""
        if self.table_dtype == BF16:
            return x.to(BF16).contiguous(), self.W_encT
        key = (self.W_encT.data_ptr(), self.W_encT._version)
        if self._split.get("key") != key:
            self._split = {"key": key}
        if exact:                                                   # bf16 rows (the model residual): 3 terms
            xh = x.to(BF16)
            w3 = self._split.get(3)
            if w3 is None:
                w3 = self._split[3] = torch.cat(split_bf16(self.W_encT), 1).contiguous()
            return torch.cat([xh, xh, xh], 1).contiguous(), w3
        xh, xm, xl = split_bf16(x)
        w6 = self._split.get(6)
        if w6 is None:
            h, m, l_ = split_bf16(self.W_encT)
            w6 = self._split[6] = torch.cat([h, m, l_, h, m, h], 1).contiguous()
        return torch.cat([xh, xh, xh, xm, xm, xl], 1).contiguous(), w6

    def encode(self, x: torch.Tensor) -> torch.Tensor:
        """JumpReLU activations ``[N, d_sae]`` fp32 (GPU: fp32-exact MFMA GEMM + fused threshold; CPU: fp32)."""
        x, exact = self._inp(x)
        if x.is_cuda:
            A, W = self._gpu_operands(x, exact)
            return ops.gemm_nt(A, W, epi=2, bias=self.b_enc, thr=self.threshold)
        pre = x @ self.W_encT.float().t() + self.b_enc
        return torch.where(pre > self.threshold, pre, torch.zeros_like(pre))

    def pre_acts(self, x: torch.Tensor) -> torch.Tensor:
        x, exact = self._inp(x)
        if x.is_cuda:
            A, W = self._gpu_operands(x, exact)
            return ops.gemm_nt(A, W, epi=1) + self.b_enc
        return x @ self.W_encT.float().t() + self.b_enc

    def decode(self, acts: torch.Tensor) -> torch.Tensor:
        """``acts W_dec + b_dec`` ([N, d_in] fp32), sparse gather of active latents on GPU."""
        return ops.sae_decode_sparse(acts.float().contiguous(), self.W_dec, self.b_dec)

    def decoder_directions(self, latents) -> torch.Tensor:
        return self.W_dec[torch.as_tensor(latents, device=self.W_dec.device).long()].float()

    @torch.no_grad()
    def calibrate(self, resid: torch.Tensor, target_l0: float = 76.0) -> None:
        """Set per-latent thresholds so that on ``resid`` rows ≈ ``target_l0`` latents fire per token."""
        pre = self.pre_acts(resid.to(self.device)).float()
        n = pre.shape[0]
        q = 1.0 - min(max(target_l0 / self.d_sae, 1e-6), 0.5)
        k = min(n, max(1, int(round(q * n))))
        self.threshold = torch.kthvalue(pre, k, dim=0).values.clamp_min(1e-6).contiguous()
        self.param_version = getattr(self, "param_version", 0) + 1     # consumers key caches on it

    def l0(self, x: torch.Tensor) -> float:
        return float((self.encode(x) > 0).float().sum(-1).mean())


def split_bf16(t: torch.Tensor):
    """``t`` (fp32) as three bf16 tensors whose fp32 sum reproduces ``t``'s 24-bit significand: each part is the
    bf16 rounding of what the previous parts leave (exact fp32 remainders)."""
    t = t.float()
    h = t.to(BF16)
    r = t - h.float()
    m = r.to(BF16)
    lo = (r - m.float()).to(BF16)
    return h, m, lo


def top_latents(sae: JumpReLUSAE, resid: torch.Tensor, start: int, top_k: int) -> list:
    """Reference SAE top-k (`src/02_run_sae_baseline.py:53-74`): encode response rows, mean over tokens, top-k."""
    r = resid[start:]
    if r.shape[0] == 0:
        return []
    acts = sae.encode(r)
    mean = acts.mean(0, keepdim=True)
    _, idx = ops.topk_rows(mean, top_k)
    return [int(i) for i in idx[0].tolist()]
