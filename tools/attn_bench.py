"""Decode attention at the sweep's shapes (Gemma-2-9B: 16 q / 8 kv heads x 256, softcap 50), with the bench's
shared-prefix layout: rows come in groups of 66 cells per (word, prompt) pair, each row reads keys [0, plen) from
its pair's baseline KV (``pkc / pvc``, one slot per pair) and [plen, pos] from its own slot.  Prints per row count
the kernel time and two byte rates: "streamed" (every K/V row each wave reads) and "unique" (each pair's prefix once
+ every row's own keys: the HBM floor if the prefix is reused through the caches).

  python tools/attn_bench.py [--rows 256,1024,2048,4096] [--reps 20]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from taboo_brittleness_amd import ops  # noqa: E402

BF = torch.bfloat16


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", default="256,1024,2048,4096")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--cells", type=int, default=66, help="rows per pair (shared prefix)")
    ap.add_argument("--S", type=int, default=128)
    ap.add_argument("--prompt", type=int, default=17)
    ap.add_argument("--gen", type=int, default=50)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--own", action="store_true",
                    help="rows with their own keys only (no shared prefix: the token-forcing decode): one-wave vs "
                         "4-wave kernel")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    Hq, Hkv, HD, S = 16, 8, 256, args.S
    g = torch.Generator(device="cpu").manual_seed(args.seed)
    for M in [int(v) for v in args.rows.split(",")]:
        P = -(-M // args.cells)
        kc = torch.randn(M, Hkv, S, HD, device=dev, dtype=BF)
        vc = torch.randn(M, Hkv, S, HD, device=dev, dtype=BF)
        pk = torch.randn(P, Hkv, S, HD, device=dev, dtype=BF)
        pv = torch.randn(P, Hkv, S, HD, device=dev, dtype=BF)
        q = torch.randn(M, Hq, HD, device=dev, dtype=BF)
        pos = args.prompt + torch.randint(0, args.gen, (M,), generator=g)
        pslot = torch.arange(M) // args.cells
        plen = torch.minimum(args.prompt + torch.randint(0, args.gen, (M,), generator=g), pos)
        slot = torch.arange(M, dtype=torch.int32, device=dev)
        out = torch.empty(M, Hq * HD, device=dev, dtype=BF)
        # the decode batch orders rows by remaining steps, not by pair: shuffle them
        perm = torch.randperm(M, generator=g)
        pos, pslot, plen = pos[perm], pslot[perm], plen[perm]
        pos_d, ps_d, pl_d = (t.to(torch.int32).to(dev) for t in (pos, pslot, plen))
        # the same rows grouped by pair (what a pair-ordered decode batch would run)
        srt = torch.argsort(pslot, stable=True)
        pos_s, ps_s, pl_s = (t[srt].to(torch.int32).to(dev) for t in (pos, pslot, plen))
        variants = {"wave": lambda: ops.attention(q, kc, vc, pos_d, slot, M, 1, HD ** -0.5, 50.0, 0, out=out,
                                                  prefix=(pk, pv, ps_d, pl_d)),
                    "sorted": lambda: ops.attention(q, kc, vc, pos_s, slot, M, 1, HD ** -0.5, 50.0, 0, out=out,
                                                    prefix=(pk, pv, ps_s, pl_s))}
        kx = ops._k()
        old_split = (kx.attention_split_rows(0, False), kx.attention_split_rows(0, True))
        if args.own:
            def _plain(n):
                kx.attention_split_rows(n, False)
                ops.attention(q, kc, vc, pos_d, slot, M, 1, HD ** -0.5, 50.0, 0, out=out)
                kx.attention_split_rows(0, False)
            variants = {"wave": lambda: _plain(0), "split": lambda: _plain(1 << 20)}
        res = {}
        for name, f in variants.items():
            for _ in range(3):
                f()
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(args.reps):
                f()
            b.record()
            torch.cuda.synchronize()
            res[name] = a.elapsed_time(b) / args.reps * 1e3
        kx.attention_split_rows(old_split[0], False)
        kx.attention_split_rows(old_split[1], True)
        us = res["wave"]
        if args.own:
            own_b = float((pos + 1).sum()) * Hkv * HD * 2 * 2
            print(json.dumps({"rows": M, "own_keys": True, "wave_us": round(us, 1), "split_us": round(res["split"], 1),
                              "mean_keys": round(float(pos.float().mean()) + 1, 1),
                              "wave_TBps": round(own_b / us / 1e6, 2),
                              "split_TBps": round(own_b / res["split"] / 1e6, 2)}), flush=True)
            del kc, vc, pk, pv, q, out
            torch.cuda.empty_cache()
            continue
        row_b = Hkv * HD * 2 * 2                                           # K + V bytes per key, all kv heads
        streamed = float((pos + 1).sum()) * row_b
        pref = {}
        for r in range(M):
            pref[int(pslot[r])] = max(pref.get(int(pslot[r]), 0), int(plen[r]))
        unique = (sum(pref.values()) + float((pos + 1 - plen).sum())) * row_b
        print(json.dumps({"rows": M, "pairs": P, "us": round(us, 1), "sorted_us": round(res["sorted"], 1),

                          "mean_keys": round(float(pos.float().mean()) + 1, 1),
                          "streamed_TBps": round(streamed / us / 1e6, 2), "unique_TBps": round(unique / us / 1e6, 2),
                          "streamed_MB": round(streamed / 1e6, 1), "unique_MB": round(unique / 1e6, 1)}), flush=True)
        del kc, vc, pk, pv, q, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
