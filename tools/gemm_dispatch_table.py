"""Rebuild ``configs/gemm_dispatch/<arch>.json`` from a ``tools/gemm_dispatch_tune.py`` raw JSONL with another
tie rule (in-tree kernel kept when ``t_tb <= tie * t_blas``) and print the per-shape in-tree share.

  python tools/gemm_dispatch_table.py profiles/r3/gemm_dispatch/raw_round1.jsonl --tie 1.02
"""
import argparse
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

ap = argparse.ArgumentParser()
ap.add_argument("raw")
ap.add_argument("--tie", type=float, default=1.02)
ap.add_argument("--tie-fused", type=float, default=1.04,
                help="tie rule for the fused gate|up + GeGLU epilogue (epi 3), whose alternative is two kernels")
ap.add_argument("--out", default=os.path.join(ROOT, "configs", "gemm_dispatch", "gemma2-9b.json"))
ap.add_argument("--min-m", type=int, default=0, help="below this M always hipBLASLt")
args = ap.parse_args()
shapes, stats = {}, {}
for line in open(args.raw):
    r = json.loads(line)
    us = {k: float(v) for k, v in r["us"].items()}
    best = min(("256", "128"), key=lambda v: us[v])
    tie = args.tie_fused if r["epi"] == 3 else args.tie
    win = int(best) if (us[best] <= tie * us["blas"] and r["M"] >= args.min_m) else "blas"
    key = f"{r['N']},{r['K']},{r['epi']}"
    shapes.setdefault(key, []).append([r["M"], win])
    s = stats.setdefault((r["shape"], r["epi"]), [0, 0])
    s[0] += win != "blas"
    s[1] += 1
json.dump({"shapes": shapes, "meta": {"raw": os.path.relpath(args.raw, ROOT), "tie": args.tie,
                                     "tie_fused": args.tie_fused}}, open(args.out, "w"),
          indent=1)
for (n, e), (a, b) in stats.items():
    print(f"{n:5s} epi{e}: in-tree at {a}/{b} row counts")
print("wrote", args.out)
