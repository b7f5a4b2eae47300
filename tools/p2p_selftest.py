"""Self-test / micro-benchmark of the one-shot P2P all-reduce (``parallel/p2p.py``).

    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 tools/p2p_selftest.py \
        [--same-device] [--iters 20] [--sizes 7168,458752,1376256]

Every rank reduces rank-dependent bf16 / fp32 tensors (different values every iteration, so the
barrier counters and the restaging are exercised) and compares with the sum computed locally in the
kernel's rank order (bit-exact).  ``--same-device`` puts every rank on ``cuda:0`` and exchanges the
IPC handles over gloo: the whole IPC + barrier protocol on a 1-GPU box.  Without it each rank uses
``cuda:LOCAL_RANK`` and the timing is also compared against RCCL's all-reduce (multi-GPU node).
Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from taboo_brittleness_amd.parallel.p2p import P2PAllReduce  # noqa: E402


def _inputs(rank: int, world: int, it: int, n: int, dtype, dev):
    g = torch.Generator().manual_seed(1000 * it + 7)
    xs = [torch.randn(n, generator=g).mul_(r + 1).to(dtype) for r in range(world)]
    exp = xs[0].float()
    for r in range(1, world):
        exp = exp + xs[r].float()
    return xs[rank].to(dev), exp.to(dtype)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--same-device", action="store_true")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--sizes", default="7168,458752,1376256")   # elements: 1 row, 64 rows, 192 rows of 3584 x 2
    ap.add_argument("--blocks", type=int, default=64)
    a = ap.parse_args()
    rank, world = int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    dev = torch.device("cuda", 0 if a.same_device else local)
    torch.cuda.set_device(dev)
    if world > 1:
        dist.init_process_group("gloo" if a.same_device else "nccl", rank=rank, world_size=world,
                                **({} if a.same_device else {"device_id": dev}))
    ar = P2PAllReduce(device=dev, max_bytes=8 << 20, blocks=a.blocks)
    sizes = [int(s) for s in a.sizes.split(",")]
    res = {"world": world, "same_device": a.same_device, "ok": True, "cases": []}
    for n in sizes:
        for dtype in (torch.bfloat16, torch.float32):
            bad = 0
            for it in range(a.iters):
                x, exp = _inputs(rank, world, it, n, dtype, dev)
                ar.all_reduce_(x)
                bad += int((x.cpu() != exp).sum().item())     # .cpu() synchronises
            ar.check()
            case = {"n": n, "dtype": str(dtype).split(".")[-1], "mismatches": bad}
            if not a.same_device and world > 1:
                x, _ = _inputs(rank, world, 0, n, dtype, dev)
                for name, fn in (("p2p", ar.all_reduce_), ("rccl", lambda t: dist.all_reduce(t))):
                    for _ in range(5):
                        fn(x)
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    for _ in range(50):
                        fn(x)
                    torch.cuda.synchronize()
                    case[f"{name}_us"] = round(1e6 * (time.perf_counter() - t0) / 50, 2)
            res["cases"].append(case)
            res["ok"] &= bad == 0
    res["p2p_calls"] = ar.calls
    res["fallbacks"] = ar.fallbacks
    if world > 1:
        flags = [None] * world
        dist.all_gather_object(flags, res["ok"])
        res["ok"] = all(flags)
        dist.barrier()
    ar.close()
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0 if res["ok"] else 1


if __name__ == "__main__":
    sys.exit(main())
