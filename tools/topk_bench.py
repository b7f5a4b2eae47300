"""Row top-k (csrc/lens.hip topk_rows_kernel, chunked two-pass for few long rows) at the lens / SAE shapes:
microseconds per call and the row bytes' rate.   python tools/topk_bench.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from taboo_brittleness_amd import ops  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    for R, V, K in ((1, 256000, 5), (42, 256000, 5), (256, 256000, 8), (600, 256000, 8), (2000, 16384, 8),
                    (4096, 16384, 64)):
        x = torch.randn(R, V, device=dev)
        for _ in range(3):
            ops.topk_rows(x, K)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(10):
            ops.topk_rows(x, K)
        b.record()
        torch.cuda.synchronize()
        us = a.elapsed_time(b) / 10 * 1e3
        print(json.dumps({"R": R, "V": V, "K": K, "us": round(us, 1), "TBps": round(R * V * 4 / us / 1e6, 2)}),
              flush=True)


if __name__ == "__main__":
    main()
