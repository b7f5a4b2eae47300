"""Decode-M weight streaming of the split-K gemm4 path vs hipBLASLt (SURVEY K6/K8 at decode row counts).

Runs each (shape, M) a few times through ``gemm4_splitk_part`` + the consumer that folds the partials (o_proj / down:
``add_rmsnorm2_part``; QKV: ``rope_qkv_cache_part``) and through hipBLASLt + the plain consumer, so a
``rocprofv3 --kernel-trace --stats`` / ``--pmc FETCH_SIZE`` run attributes bytes and time per kernel:

  rocprofv3 --kernel-trace --stats -d gpurun_out/skbw -o run -- python3 tools/splitk_bw.py
  rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/skbw_pmc -o run -- python3 tools/splitk_bw.py

Without a profiler it prints the weight-streaming rate (weight bytes / wall time of the whole projection + consumer).
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from taboo_brittleness_amd.ops import _ext  # noqa: E402

SHAPES = {"o": (3584, 4096), "down": (3584, 14336), "qkv": (8192, 3584)}


def main():
    _ext.load()
    k = _ext.kernels()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    reps = int(os.environ.get("SKBW_REPS", "20"))
    for name, (N, K) in SHAPES.items():
        Ws = [((torch.rand(N, K, device=dev, generator=g) * 2 - 1) * 0.05).to(torch.bfloat16) for _ in range(6)]
        for M in (16, 64, 256):
            A = ((torch.rand(M, K, device=dev, generator=g) * 2 - 1)).to(torch.bfloat16)
            ks = int(k.gemm4_splitk_ks(M, N, K, 128))
            ws = torch.empty(ks * M * N, device=dev)
            C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            h = torch.randn(M, N, device=dev).to(torch.bfloat16)
            w1 = torch.zeros(N, device=dev, dtype=torch.bfloat16)
            x = torch.empty_like(h)
            if name == "qkv":
                Hq, Hkv, HD, S = 16, 8, 256, 128
                pos = torch.arange(M, device=dev, dtype=torch.int32) % S
                slot = torch.arange(M, device=dev, dtype=torch.int32) // S
                cos_t = torch.rand(S, HD // 2, device=dev)
                sin_t = torch.rand(S, HD // 2, device=dev)
                kc = torch.zeros(max(1, M // S + 1), Hkv, S, HD, device=dev, dtype=torch.bfloat16)
                vc = torch.zeros_like(kc)
                q = torch.empty(M, Hq, HD, device=dev, dtype=torch.bfloat16)

                def split(W):
                    used = int(k.gemm4_splitk_part(A, W, ws, 128, ks))
                    k.rope_qkv_cache_part(ws, used, pos, slot, cos_t, sin_t, q, kc, vc, Hq, Hkv, HD)

                def blas(W):
                    torch.matmul(A, W.t(), out=C)
                    k.rope_qkv_cache(C, pos, slot, cos_t, sin_t, q, kc, vc, Hq, Hkv, HD)
            else:
                def split(W):
                    used = int(k.gemm4_splitk_part(A, W, ws, 128, ks))
                    k.add_rmsnorm2_part(h, ws, used, w1, w1, x, 1e-6)

                def blas(W):
                    torch.matmul(A, W.t(), out=C)
                    k.add_rmsnorm2(h, C, w1, w1, x, 1e-6)
            for label, fn in (("splitk", split), ("hipblaslt", blas)):
                for i in range(3):
                    fn(Ws[i % len(Ws)])
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for i in range(reps):
                    fn(Ws[i % len(Ws)])
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / reps
                print(f"{name:5s} M={M:4d} {label:9s} ks={ks:2d} {us:7.1f} us  weights {N * K * 2 / us / 1e6:5.2f} TB/s",
                      flush=True)


if __name__ == "__main__":
    main()
