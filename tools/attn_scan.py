"""Decode-attention time vs KV length (2048 rows, Gemma-2-9B heads): is the kernel bound by bytes or by a
fixed per-workgroup cost?  Prints one JSON line per KV length."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from taboo_brittleness_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
BF = torch.bfloat16
M, Hq, Hkv, HD, S = 2048, 16, 8, 256, 68
kc = torch.randn(M, Hkv, S, HD, device=dev, dtype=BF)
vc = torch.randn(M, Hkv, S, HD, device=dev, dtype=BF)
q = torch.randn(M, Hq, HD, device=dev, dtype=BF)
slot = torch.arange(M, dtype=torch.int32, device=dev)
out = torch.empty(M, Hq * HD, device=dev, dtype=BF)
for L in (1, 8, 16, 32, 48, 67):
    pos = torch.full((M,), L - 1, dtype=torch.int32, device=dev)
    f = lambda: ops.attention(q, kc, vc, pos, slot, M, 1, HD ** -0.5, 50.0, 0, out=out)   # noqa: E731
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(20):
        f()
    b.record()
    torch.cuda.synchronize()
    us = a.elapsed_time(b) / 20 * 1e3
    print(json.dumps({"keys": L, "us": round(us, 1), "TB/s": round(2 * M * Hkv * L * HD * 2 / us / 1e6, 2)}), flush=True)
