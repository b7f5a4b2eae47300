"""add_rmsnorm2 (csrc/norm.hip) at the Gemma-2-9B width, one-workgroup-per-row kernel vs one-wave-per-row kernel:
time per call (median of 3 interleaved rounds) and bytes moved (h, o read; h, x written) per row count, plus the
largest difference between the two kernels' outputs (their sums of squares run in different orders).

    python tools/norm_bench.py [--rows 64,256,1024,4096,16384]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from taboo_brittleness_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", default="64,256,1024,4096,16384")
    ap.add_argument("--D", type=int, default=3584)
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    D = a.D
    for M in [int(v) for v in a.rows.split(",")]:
        h = torch.randn(M, D, device=dev).to(torch.bfloat16)
        o = torch.randn(M, D, device=dev).to(torch.bfloat16)
        wp = (torch.randn(D, device=dev) * 0.1).to(torch.bfloat16)
        wn = (torch.randn(D, device=dev) * 0.1).to(torch.bfloat16)
        x = torch.empty_like(h)
        k = ops._k()
        fns = {"block": lambda: k.add_rmsnorm2(h, o, wp, wn, x, 1e-6),       # one workgroup per row (default)
               "wave": lambda: k.add_rmsnorm2_wave(h, o, wp, wn, x, 1e-6)}   # one wave per row
        h0 = h.clone()
        outs = {}
        for name, fn in fns.items():                 # numerics: one call each from the same h
            h.copy_(h0)
            fn()
            outs[name] = (h.clone(), x.clone())
        dh = float((outs["block"][0].float() - outs["wave"][0].float()).abs().max())
        dx = float((outs["block"][1].float() - outs["wave"][1].float()).abs().max())
        res = {}
        for rnd in range(3):                         # interleaved rounds
            for name, fn in fns.items():
                for _ in range(3):
                    fn()
                torch.cuda.synchronize()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(a.reps):
                    fn()
                e.record()
                torch.cuda.synchronize()
                res.setdefault(name, []).append(s.elapsed_time(e) / a.reps * 1e3)
        gb = 4 * M * D * 2 / 1e9
        us = {n: round(sorted(v)[1], 2) for n, v in res.items()}
        print(json.dumps({"rows": M, "us": us, "TBps": {n: round(gb / (u * 1e-6) / 1e3, 2) for n, u in us.items()},
                          "max_abs_diff_h": dh, "max_abs_diff_x": dx}), flush=True)

if __name__ == "__main__":
    main()
