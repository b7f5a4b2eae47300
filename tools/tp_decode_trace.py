"""Kernel census of the TP=2 hipGraph decode: two processes share cuda:0 (the P2P all-reduce /
all-gather over IPC, the vocab-parallel decode head), capture the decode graphs with one greedy generation, then
run two more between marker kernels (``topk_rows_kernel``, which the decode never runs): window A generates
``STEPS_A`` new tokens, window B ``STEPS_B``.  Everything outside the per-step graph replays (prefill, the decode
call's one-time setup) is the same in both windows, so (B - A) / (STEPS_B - STEPS_A) is what ONE decode step costs
per kind of kernel.  Run it under the kernel tracer (one output per process), then reduce the traces:

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tp_trace -o run_%pid% -- python3 tools/tp_decode_trace.py
    python3 tools/tp_decode_trace.py --analyze gpurun_out/tp_trace

PyTorch-native kernels are the ``at::native`` ones and the runtime's copy / fill blits (``__amd_rocclr_*``); the
model is the TP test's tiny Gemma-2 (tests/test_tp_gloo.py SPEC: 3 layers, vocab 512), greedy, 2 rows.
"""
from __future__ import annotations

import argparse
import csv
import glob
import os
import socket
import sys
from collections import Counter, defaultdict
from dataclasses import replace

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

NATIVE = ("at::native", "__amd_rocclr_")
MARK = "topk_rows_kernel"
STEPS_A, STEPS_B = 5, 13


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank: int, port: int) -> None:
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": "2", "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    import torch
    import torch.distributed as dist

    from taboo_brittleness_amd import ops
    from taboo_brittleness_amd.models.gemma2 import Gemma2Model
    from taboo_brittleness_amd.models.spec import GEMMA2_TINY
    from taboo_brittleness_amd.models.weights import random_gemma2
    from taboo_brittleness_amd.parallel.tp import make_groups, shard_weights
    from taboo_brittleness_amd.runtime.generation import Generator

    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    dist.init_process_group("gloo", rank=rank, world_size=2)
    ctx, _, _ = make_groups(2, rank, 2, allreduce="p2p", device=dev, vocab_parallel=True)
    spec = replace(GEMMA2_TINY, vocab_size=512, layers=3, heads=4, kv_heads=2, ffn=512)
    w = shard_weights(random_gemma2(spec, dtype=torch.bfloat16, seed=11, norm_std=0.1), ctx).to(dev)
    m = Gemma2Model(w, dev, tp=ctx)
    gen = Generator(m, 2, 24, use_graphs=True, stop_ids=(10_000,))
    prompts = [[2, 5, 9, 11], [2, 7, 8]]
    first = gen.generate(prompts, STEPS_B, graph_key="tp")       # captures the decode graphs
    mark = torch.randn(4, 64, device=dev)
    torch.cuda.synchronize()
    dist.barrier()
    ops.topk_rows(mark, 4)                                        # marker: window A
    a = gen.generate(prompts, STEPS_A, graph_key="tp")
    ops.topk_rows(mark, 4)                                        # marker: window B
    b = gen.generate(prompts, STEPS_B, graph_key="tp")
    ops.topk_rows(mark, 4)                                        # marker: end
    torch.cuda.synchronize()
    assert [b.response_ids(i) for i in range(2)] == [first.response_ids(i) for i in range(2)]
    assert [a.response_ids(i) for i in range(2)] == [first.response_ids(i)[:len(a.response_ids(i))] for i in range(2)]
    ctx.p2p.check()
    dist.barrier()
    ctx.p2p.close()
    dist.destroy_process_group()
    print(f"rank {rank} ok", flush=True)


def run() -> None:
    import torch.multiprocessing as mp

    port = _port()
    ctx = mp.get_context("spawn")
    ps = [ctx.Process(target=_worker, args=(r, port)) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(timeout=300)
        assert p.exitcode == 0, p.exitcode


def _name(k: str) -> str:
    k = k.replace("(anonymous namespace)::", "")
    k = k[5:] if k.startswith("void ") else k
    return k.split("(")[0][:80]


def analyze(d: str) -> int:
    paths = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    assert paths, f"no kernel trace under {d}"
    procs = []
    for p in paths:
        rs = sorted(csv.DictReader(open(p)), key=lambda r: int(r["Start_Timestamp"]))
        idx = [i for i, r in enumerate(rs) if MARK in r["Kernel_Name"]]
        if len(idx) >= 3:
            procs.append((p, rs, idx[-3:]))
    worst = 0.0
    for p, rs, (i0, i1, i2) in procs:
        wa = Counter(_name(r["Kernel_Name"]) for r in rs[i0 + 1:i1])
        wb = Counter(_name(r["Kernel_Name"]) for r in rs[i1 + 1:i2])
        ds = STEPS_B - STEPS_A
        print(f"== {os.path.basename(p)}: window A {sum(wa.values())} kernels ({STEPS_A} new tokens), window B "
              f"{sum(wb.values())} ({STEPS_B}); per decode step = (B - A) / {ds}")
        per = {k: (wb[k] - wa[k]) / ds for k in set(wa) | set(wb)}
        nat_step = sum(v for k, v in per.items() if any(t in k for t in NATIVE))
        nat_once = sum(v for k, v in wa.items() if any(t in k for t in NATIVE))
        worst = max(worst, nat_step)
        print(f"   per step: {sum(per.values()):.2f} kernels, {nat_step:.2f} PyTorch-native; once per generate() call "
              f"(prefill + decode setup, outside the graphs): {nat_once} PyTorch-native")
        for k, v in sorted(per.items(), key=lambda x: -x[1]):
            if v:
                print(f"   {v:6.2f}/step  {'NATIVE ' if any(t in k for t in NATIVE) else ''}{k}")
        print("   once per call (window A, PyTorch-native only):")
        for k, v in wa.most_common():
            if any(t in k for t in NATIVE):
                print(f"   {v:6d}       {k}")
    print(f"processes with marked windows: {len(procs)}; max PyTorch-native kernels per TP decode step: {worst:.2f}")
    return 0 if len(procs) == 2 else 1


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--analyze", default=None)
    a = ap.parse_args()
    if a.analyze:
        sys.exit(analyze(a.analyze))
    run()
