"""Hot kernels of the flagship sweep step at its decode shapes, in one short program for rocprofv3 PMC passes
(tools/pmc_kernels.sh): softcapped GQA decode attention, GeGLU, fused add+RMSNorm, RoPE+KV store, the SAE
JumpReLU encode (MFMA GEMM + threshold epilogue), for comparison one hipBLASLt projection GEMM, and (round 2) the
prefix-trie K/V fan-out and the vocab head's decode_head reduction.

Shapes: 2048 decode rows (a typical row bucket of the diverged-cell decode), Gemma-2-9B dims
(D 3584, 16 q / 8 kv heads x 256, FFN 14336), 67-token KV rows, 16k-latent SAE.  Prints achieved
bandwidth / FLOP rates from HIP events next to the counters the profiler collects.
"""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from taboo_brittleness_amd import ops  # noqa: E402
from taboo_brittleness_amd.ops import _ext  # noqa: E402

_ext.load()
dev = torch.device("cuda:0")
BF = torch.bfloat16
M, D, Hq, Hkv, HD, S, F, L = 2048, 3584, 16, 8, 256, 67, 14336, 16384
ITERS = 5
torch.manual_seed(0)


def timed(fn):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(ITERS):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / ITERS * 1e-3


res = {}
kc = torch.randn(M, Hkv, S, HD, device=dev, dtype=BF)
vc = torch.randn(M, Hkv, S, HD, device=dev, dtype=BF)
q = torch.randn(M, Hq, HD, device=dev, dtype=BF)
pos = torch.full((M,), S - 1, dtype=torch.int32, device=dev)
slot = torch.arange(M, dtype=torch.int32, device=dev)
out = torch.empty(M, Hq * HD, device=dev, dtype=BF)
t = timed(lambda: ops.attention(q, kc, vc, pos, slot, M, 1, HD ** -0.5, 50.0, 0, out=out))
res["attn_decode"] = {"ms": t * 1e3, "GB/s": 2 * kc.numel() * 2 / t / 1e9}
del kc, vc

gu = torch.randn(M, 2 * F, device=dev, dtype=BF)
g_out = torch.empty(M, F, device=dev, dtype=BF)
t = timed(lambda: ops.geglu(gu, out=g_out))
res["geglu"] = {"ms": t * 1e3, "GB/s": (gu.numel() + g_out.numel()) * 2 / t / 1e9}

h = torch.randn(M, D, device=dev, dtype=BF)
o = torch.randn(M, D, device=dev, dtype=BF)
w1 = torch.randn(D, device=dev, dtype=BF) * 0.1
w2 = torch.randn(D, device=dev, dtype=BF) * 0.1
xo = torch.empty_like(h)
t = timed(lambda: ops.add_rmsnorm2(h, o, w1, w2, 1e-6, out=xo))
res["add_rmsnorm2"] = {"ms": t * 1e3, "GB/s": 4 * h.numel() * 2 / t / 1e9}

W_enc = torch.randn(L, D, device=dev, dtype=BF) * 0.02
bias = torch.zeros(L, device=dev)
thr = torch.full((L,), 0.1, device=dev)
acts = torch.empty(M, L, device=dev, dtype=torch.float32)
x = torch.randn(M, D, device=dev, dtype=BF)
t = timed(lambda: ops.gemm_nt(x, W_enc, epi=2, bias=bias, thr=thr, out=acts))
res["sae_encode_gemm_nt"] = {"ms": t * 1e3, "TFLOP/s": 2 * M * D * L / t / 1e12}

W_gu = torch.randn(2 * F, D, device=dev, dtype=BF) * 0.02
y = torch.empty(M, 2 * F, device=dev, dtype=BF)
t = timed(lambda: torch.matmul(x, W_gu.t(), out=y))
res["hipblaslt_gate_up"] = {"ms": t * 1e3, "TFLOP/s": 2 * M * D * 2 * F / t / 1e12}
del W_gu, y, acts, W_enc

# round 2: prefix-trie decode K/V fan-out (3584 rows, 2/3 of them members, blocks 0..31, 67-token slots) and the
# hipBLASLt head's decode_head reduction (2048 rows x 256k vocab, bf16 softcap chain, argmax + NLL)
Lf, R2 = 32, 3584
kc5 = torch.randn(Lf, R2, Hkv, S, HD, device=dev, dtype=BF)
vc5 = torch.randn_like(kc5)
src = torch.where(torch.arange(R2, device=dev) % 3 == 0, -1, (torch.arange(R2, device=dev) // 3) * 3).int()
slot2 = torch.arange(R2, dtype=torch.int32, device=dev)
pos2 = torch.full((R2,), S - 1, dtype=torch.int32, device=dev)
t = timed(lambda: ops.kv_fanout(kc5, vc5, src, slot2, pos2, Lf))
nmem = int((src >= 0).sum())
res["kv_fanout"] = {"ms": t * 1e3, "GB/s": 2 * 2 * nmem * Lf * Hkv * HD * 2 / t / 1e9}
del kc5, vc5
V = 256000
lg = (torch.randn(M, V, device=dev) * 3).to(BF)
t = timed(lambda: ops.decode_head(lg, 30.0))
res["decode_head"] = {"ms": t * 1e3, "GB/s": lg.numel() * 2 / t / 1e9}
print(json.dumps({k: {kk: round(vv, 3) for kk, vv in v.items()} for k, v in res.items()}))
