"""add_rmsnorm2 (csrc/norm.hip) at the Gemma-2-9B width: time per call and bytes moved (h, o read; h, x written;
two weight rows) per row count.

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
        for _ in range(3):
            ops.add_rmsnorm2(h, o, wp, wn, 1e-6, out=x)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.reps):
            ops.add_rmsnorm2(h, o, wp, wn, 1e-6, out=x)
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) / a.reps * 1e3
        gb = 4 * M * D * 2 / 1e9
        print(json.dumps({"rows": M, "us": round(us, 2), "TBps": round(gb / (us * 1e-6) / 1e3, 2)}), flush=True)


if __name__ == "__main__":
    main()
