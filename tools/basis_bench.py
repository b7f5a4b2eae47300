"""Random-basis kernel (csrc/basis.hip) on the lowrank side's per-step workload: P pairs x 5 random trials x ranks
{1, 2, 4, 8, 16, 32, 64} at D = 3584, largest rank first (as sweep_plan draws them), for each load batching qu.
GPU time per call (events, median of 5 after a warm call); the tables must agree bit for bit."""
import json
import sys

import torch

sys.path.insert(0, ".")
from taboo_brittleness_amd import ops  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    D = 3584
    for P in (120, 175):
        ranks = sorted([r for _ in range(P * 5) for r in (1, 2, 4, 8, 16, 32, 64)], reverse=True)
        rows = [0]
        for r in ranks[:-1]:
            rows.append(rows[-1] + r)
        R = rows[-1] + ranks[-1]
        seeds = torch.arange(len(ranks), dtype=torch.int64, device=dev) * 7919 + 13
        rk = torch.tensor(ranks, dtype=torch.int32, device=dev)
        rw = torch.tensor(rows, dtype=torch.int64, device=dev)
        res = {"P": P, "bases": len(ranks)}
        ref = None
        for qu in (1, 2, 4):
            tab = torch.empty(R, D, device=dev)
            ops.random_basis(seeds, rk, rw, tab, qu=qu)
            torch.cuda.synchronize()
            ts = []
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                ops.random_basis(seeds, rk, rw, tab, qu=qu)
                e1.record()
                e1.synchronize()
                ts.append(e0.elapsed_time(e1))
            res[f"qu{qu}_ms"] = round(sorted(ts)[2], 2)
            if ref is None:
                ref = tab.clone()
            else:
                assert torch.equal(tab, ref), qu
            del tab
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
