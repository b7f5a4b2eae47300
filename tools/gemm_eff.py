"""Achieved bf16 TFLOP/s of the engine's projection GEMMs (y = x W^T via torch.matmul = hipBLASLt,
with the bench's TunableOp table), per shape: decode buckets and teacher-forced-tail chunk sizes."""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from taboo_brittleness_amd.runtime.tuning import enable_tuned_gemms  # noqa: E402

enable_tuned_gemms("gemma2-9b_P90_E4_new50")
dev = torch.device("cuda:0")
W = {"qkv": (8192, 3584), "o": (3584, 4096), "gu": (28672, 3584), "down": (3584, 14336), "lm_head": (256000, 3584)}
ws = {k: torch.randn(n, kk, device=dev, dtype=torch.bfloat16) * 0.02 for k, (n, kk) in W.items()}
res = []
for M in (256, 1024, 2048, 3840, 4096, 6144, 32768):
    for name, w in ws.items():
        if name == "lm_head" and M > 4096:
            continue
        x = torch.randn(M, w.shape[1], device=dev, dtype=torch.bfloat16)
        out = torch.empty(M, w.shape[0], device=dev, dtype=torch.bfloat16)
        for _ in range(3):
            torch.matmul(x, w.t(), out=out)
        torch.cuda.synchronize()
        n = max(3, int(2e12 / (2 * M * w.shape[0] * w.shape[1])))
        t0 = time.perf_counter()
        for _ in range(n):
            torch.matmul(x, w.t(), out=out)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / n
        tf = 2 * M * w.shape[0] * w.shape[1] / dt / 1e12
        res.append({"M": M, "gemm": name, "N": w.shape[0], "K": w.shape[1], "us": round(dt * 1e6, 1), "TFLOPs": round(tf, 1)})
        print(json.dumps(res[-1]), flush=True)
