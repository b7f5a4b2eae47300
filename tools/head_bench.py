"""A/B of the vocab head and the logit-lens unembedding at Gemma-2-9B shapes (V = 256000, K = 3584):
hipBLASLt logits + decode_head vs the fused GEMM head (csrc/gemm4.hip G4_HEAD), and
hipBLASLt logits + row_lse vs the fused lens GEMM (csrc/gemm4.hip G4_LENS), interleaved rounds in one process
(cdna_hip_programming.md §5.4 rule 24), random data.  Run with TB_GEMM=blas so ``linear`` is hipBLASLt.
Prints one JSON line per M.

    python tools/head_bench.py [--rows 256 2048 4096] [--rounds 5]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from taboo_brittleness_amd import ops  # noqa: E402


def timed(fn, reps):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000.0 / reps


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, nargs="+", default=[256, 1024, 2048, 4096])
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    V, K, cap = 256000, 3584, 30.0
    torch.manual_seed(0)
    w = (torch.randn(V, K, device=dev) * 0.02).to(torch.bfloat16)
    for M in args.rows:
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        tgt = torch.randint(0, V, (M,), dtype=torch.int32, device=dev)
        lg = torch.empty(M, V, dtype=torch.bfloat16, device=dev)
        part = torch.empty(ops.head_part_numel(M, V), dtype=torch.float32, device=dev)
        outs = [torch.empty(M, dtype=torch.int32, device=dev), torch.empty(M, device=dev), torch.empty(M, device=dev)]
        tl = torch.empty(M, device=dev)

        def unfused():
            ops.linear(x, w, out=lg)
            ops.decode_head(lg, cap, tgt, *outs)

        def fused():
            ops.vocab_head(x, w, cap, tgt, *outs, part=part, tgt_logit=tl, fused=True)

        def gemm_only():
            ops.linear(x, w, out=lg)

        def lens_unfused():
            ops.lens_unembed(x, w, fused=False, out=lg)

        def lens_fused():
            ops.lens_unembed(x, w, fused=True, out=lg)

        unfused(); fused(); torch.cuda.synchronize()
        a = ops.vocab_head(x, w, cap, tgt, fused=False)
        b = ops.vocab_head(x, w, cap, tgt, fused=True)
        agree = float((a[0] == b[0]).float().mean())
        dn = float((a[2] - b[2]).abs().max())
        res = {"unfused": [], "fused": [], "gemm_only": [], "lens_unfused": [], "lens_fused": []}
        for _ in range(args.rounds):
            res["unfused"].append(timed(unfused, args.reps))
            res["fused"].append(timed(fused, args.reps))
            res["gemm_only"].append(timed(gemm_only, args.reps))
            res["lens_unfused"].append(timed(lens_unfused, args.reps))
            res["lens_fused"].append(timed(lens_fused, args.reps))
        med = {k: sorted(v)[len(v) // 2] for k, v in res.items()}
        tf = 2.0 * M * V * K / 1e12
        print(json.dumps({"M": M, "us_median": {k: round(v, 1) for k, v in med.items()},
                          "us_min": {k: round(min(v), 1) for k, v in res.items()},
                          "tflops_fused": round(tf / (med["fused"] * 1e-6), 1),
                          "tflops_hipblaslt_gemm": round(tf / (med["gemm_only"] * 1e-6), 1),
                          "speedup_fused_vs_unfused": round(med["unfused"] / med["fused"], 3),
                          "speedup_lens_fused_vs_unfused": round(med["lens_unfused"] / med["lens_fused"], 3),
                          "argmax_agree_vs_hipblaslt": agree, "max_abs_dnll_tgt": dn}), flush=True)


if __name__ == "__main__":
    main()
