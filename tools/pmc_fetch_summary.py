"""Per-kernel HBM fetch bandwidth from a ``rocprofv3 --pmc FETCH_SIZE --kernel-trace`` counter CSV: for every
(kernel, grid) group the median FETCH_SIZE (KB, L2 -> fabric fetches) per dispatch, the median duration and their
ratio (TB/s).   python tools/pmc_fetch_summary.py gpurun_out/skbw/pmc/run_counter_collection.csv
"""
import csv
import statistics
import sys
from collections import defaultdict


def short(n: str) -> str:
    if n.startswith(("Cijk_", "Custom_Cijk")):
        i = n.find("MT")
        return "hipblaslt " + (n[i:n.find("_", i)] if i >= 0 else "?")
    n = n.replace("void ", "").replace("(anonymous namespace)::", "")
    return n[:n.find("(")] if "(" in n else n[:60]


def main(path):
    g = defaultdict(lambda: ([], []))
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != "FETCH_SIZE":
            continue
        k = (short(r["Kernel_Name"]), int(r["Grid_Size"]))
        g[k][0].append(float(r["Counter_Value"]))
        g[k][1].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    print(f"{'kernel':44s} {'grid':>9s} {'n':>4s} {'fetch MB':>9s} {'us':>8s} {'TB/s':>6s}")
    for (name, grid), (kb, ns) in sorted(g.items(), key=lambda x: -sum(x[1][1])):
        if len(kb) < 3:
            continue
        f, t = statistics.median(kb), statistics.median(ns)
        print(f"{name[:44]:44s} {grid:9d} {len(kb):4d} {f / 1024:9.2f} {t / 1e3:8.1f} {f * 1024 / max(t, 1) / 1e3:6.2f}")


if __name__ == "__main__":
    main(sys.argv[1])
