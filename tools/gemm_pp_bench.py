"""Ping-pong MFMA GEMM (csrc/gemm.hip) vs hipBLASLt: numerics at odd shapes, then interleaved timing.

    python tools/gemm_pp_bench.py [--quick] [--shapes gu,sae,...] [--ms 512,2048]

Numerics: every epilogue against a float32 PyTorch reference (ragged M, several K).  Timing: for each
(shape, M) the variants run in interleaved rounds in this one process (cdna_hip_programming.md §5.4
rule 24) on uniform [-1, 1) operands; the median per variant is printed as one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from taboo_brittleness_amd import ops  # noqa: E402
from taboo_brittleness_amd.ops import _ext  # noqa: E402

SHAPES = {  # name: (N, K)
    "qkv": (8192, 3584), "o": (3584, 4096), "gu": (28672, 3584), "down": (3584, 14336),
    "sae": (16384, 3584), "lm_head": (256000, 3584),
}


def check(k, dev):
    torch.manual_seed(0)
    worst = 0.0
    for M, N, K in [(1, 256, 64), (37, 512, 128), (300, 768, 256), (513, 1024, 3584), (256, 256, 640)]:
        A = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
        W = (torch.rand(N, K, device=dev) * 2 - 1).bfloat16()
        ref = A.float() @ W.float().T
        C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        k.gemm_pp(A, W, C, None, None, 0, 256)
        e0 = ((C.float() - ref).abs().max() / ref.abs().max()).item()
        Cf = torch.empty(M, N, device=dev, dtype=torch.float32)
        k.gemm_pp(A, W, Cf, None, None, 1, 256)
        e1 = ((Cf - ref).abs().max() / ref.abs().max()).item()
        b = torch.randn(N, device=dev)
        th = torch.rand(N, device=dev) * 2
        k.gemm_pp(A, W, Cf, b, th, 2, 256)
        pre = ref + b
        jr = torch.where(pre > th, pre, torch.zeros_like(pre))
        e2 = ((Cf - jr).abs().max() / jr.abs().max().clamp_min(1e-6)).item()
        # GeGLU: gate|up rows interleaved
        Wi = W[ops.geglu_interleave_index(N // 2, dev)]
        G = torch.empty(M, N // 2, device=dev, dtype=torch.bfloat16)
        k.gemm_pp(A, Wi, G, None, None, 3, 256)
        gu = ref.bfloat16()
        gref = ops.reference_geglu(gu).float()
        e3 = ((G.float() - gref).abs().max() / gref.abs().max()).item()
        worst = max(worst, e0, e1, e2, e3)
        print(json.dumps({"check": [M, N, K], "bf16": e0, "f32": e1, "jumprelu": e2, "geglu": e3}), flush=True)
    assert worst < 2e-2, worst
    print(json.dumps({"check_ok": True, "worst_rel": worst}), flush=True)


def timeit(fn, reps):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000.0 / reps


def bench(k, dev, names, ms, rounds):
    for name in names:
        N, K = SHAPES[name]
        W = (torch.rand(N, K, device=dev) * 2 - 1).bfloat16()
        Wi = W[ops.geglu_interleave_index(N // 2, dev)] if name == "gu" else None
        for M in ms:
            A = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
            C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            var = {"hipblaslt": lambda: torch.matmul(A, W.T, out=C), "pp": lambda: k.gemm_pp(A, W, C, None, None, 0, 256)}
            if name == "gu":
                act = torch.empty(M, N // 2, device=dev, dtype=torch.bfloat16)
                var["hipblaslt+geglu"] = lambda: (torch.matmul(A, W.T, out=C), k.geglu(C, act))
                var["pp_geglu"] = lambda: k.gemm_pp(A, Wi, act, None, None, 3, 256)
            if name == "sae":
                Cf = torch.empty(M, N, device=dev, dtype=torch.float32)
                b = torch.randn(N, device=dev)
                th = torch.rand(N, device=dev)
                var["nt_jumprelu"] = lambda: k.gemm_nt(A, W, Cf, b, th, 2)
                var["pp_jumprelu"] = lambda: k.gemm_pp(A, W, Cf, b, th, 2, 256)
            flop = 2.0 * M * N * K
            reps = max(3, min(50, int(2e13 / flop)))
            for f in var.values():
                f()
            torch.cuda.synchronize()
            res = {v: [] for v in var}
            for _ in range(rounds):
                for v, f in var.items():
                    res[v].append(timeit(f, reps))
            out = {"gemm": name, "M": M, "N": N, "K": K}
            for v, xs in res.items():
                us = statistics.median(xs)
                out[v] = {"us": round(us, 1), "TF": round(flop / us / 1e6, 1), "min_us": round(min(xs), 1)}
            print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="gu,sae,qkv,down,o")
    ap.add_argument("--ms", default="256,512,1024,2048,3072,4096,6144,8192")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--no-check", action="store_true")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    k = _ext.load()
    if not args.no_check:
        check(k, dev)
    bench(k, dev, args.shapes.split(","), [int(m) for m in args.ms.split(",")], args.rounds)


if __name__ == "__main__":
    main()
