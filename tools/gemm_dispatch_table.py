"""Build ``configs/gemm_dispatch/<arch>.json`` from one or more ``tools/gemm_dispatch_tune.py`` raw JSONL files.

Each raw line times hipBLASLt (``blas``) and some in-tree variants at one ``(N, K, epilogue, M)``.  Files from
different runs (e.g. a full sweep plus a later one with the split-K variants) are merged per point through the
time RELATIVE to that run's own hipBLASLt time, so box-to-box clock differences cancel; the in-tree variant with
the lowest ratio wins when ``ratio <= tie`` (``--tie-fused`` for the fused GeGLU epilogue, whose alternative is two
kernels).  Prints the per-shape in-tree count.

Four-wave winners are recorded as ``"gs"`` (the rounds model picks the tile height per row count; ``--no-gs``: as
measured).  The ``tb_shapes`` section (``TB_GEMM=tb``) is the fastest BATCH-INVARIANT variant per point (ring ``r*``, four-wave
``g*``, ping-pong ``256`` / ``128``; never split-K or hipBLASLt), from the same merged ratios.

  python tools/gemm_dispatch_table.py gpurun_out/r4/raw.jsonl gpurun_out/r4/raw_splitk.jsonl --tie 1.01
"""
import argparse
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("raw", nargs="+")
    ap.add_argument("--tie", type=float, default=1.01)
    ap.add_argument("--tie-fused", type=float, default=1.01)
    ap.add_argument("--out", default=os.path.join(ROOT, "configs", "gemm_dispatch", "gemma2-9b.json"))
    ap.add_argument("--exclude", default="", help="comma-separated variants never chosen (e.g. 256,128)")
    ap.add_argument("--tag", default="")
    ap.add_argument("--no-gs", action="store_true",
                    help="keep g256 / g128 winners as measured instead of the rounds-model choice \"gs\"")
    ap.add_argument("--fresh", nargs="*", default=[],
                    help="raw files re-measuring some variants with a newer kernel build: their ratios REPLACE the "
                         "older files' values of the same (point, variant) instead of taking the minimum")
    args = ap.parse_args()
    excl = set(v for v in args.exclude.split(",") if v)
    pts = {}                       # (shape, N, K, epi, M) -> {variant: ratio to blas}
    for fresh, paths in ((False, args.raw), (True, args.fresh)):
        seen = set()
        for path in paths:
            for line in open(path):
                r = json.loads(line)
                us = {k: float(v) for k, v in r["us"].items()}
                key = (r["shape"], r["N"], r["K"], r["epi"], r["M"])
                d = pts.setdefault(key, {})
                for v, t in us.items():
                    if v == "blas" or v in excl:
                        continue
                    old = d.get(v, 1e9) if not fresh or (key, v) in seen else 1e9
                    d[v] = min(old, t / us["blas"])
                    seen.add((key, v))
    if not args.no_gs:
        # the four-wave kernel's tile height is the rounds model's (runtime.gemm_dispatch.split_rows: 256 rows, 128
        # rows or a row split): one entry "gs" at the best of the measured heights, so row counts between the
        # measured points get the model's height instead of their neighbour's
        for d in pts.values():
            g = [d[v] for v in ("g256", "g128", "gs") if v in d]
            if g:
                for v in ("g256", "g128"):
                    d.pop(v, None)
                d["gs"] = min(g)
    shapes, tb_shapes, stats = {}, {}, {}
    for (shape, N, K, epi, M), d in sorted(pts.items()):
        best = min(d, key=d.get)
        tie = args.tie_fused if epi == 3 else args.tie
        win = best if d[best] <= tie else "blas"
        win = win if not win.isdigit() else int(win)
        shapes.setdefault(f"{N},{K},{epi}", []).append([M, win])
        inv = [v for v in d if v[:1] in ("g", "r") or v.isdigit()]
        if inv:
            bi = min(inv, key=d.get)
            tb_shapes.setdefault(f"{N},{K},{epi}", []).append([M, int(bi) if bi.isdigit() else bi])
        s = stats.setdefault((shape, epi), [0, 0, 0.0, 0.0])
        s[0] += win != "blas"
        s[1] += 1
        s[2] += min(d[best], 1.0) if win != "blas" else 1.0
        s[3] += d[bi] if inv else 1.0
    tab = {"shapes": shapes, "tb_shapes": tb_shapes,
           "meta": {"tie": args.tie, "tie_fused": args.tie_fused, "sources": args.raw + args.fresh, "tag": args.tag}}
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    json.dump(tab, open(args.out, "w"), indent=1)
    for (shape, epi), (w, n, ra, rt) in sorted(stats.items()):
        print(f"{shape:5s} epi {epi}: in-tree at {w}/{n} row counts; mean time vs hipBLASLt: auto {ra / n:.3f}, "
              f"tb (batch-invariant) {rt / n:.3f}")
    print(f"wrote {args.out}")


if __name__ == "__main__":
    main()
