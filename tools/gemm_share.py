"""GEMM time split of a rocprofv3 kernel_stats.csv: in-tree MFMA GEMM kernels vs hipBLASLt.

  python tools/gemm_share.py profiles/r3/prof_default/run_kernel_stats.csv
"""
import csv
import sys

INTREE = ("gemm_pp_kernel", "gemm4_kernel", "gemm_nt_kernel", "gemm_ring_kernel")
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
lib = sum(float(r["TotalDurationNs"]) for r in rows if r["Name"].startswith(("Cijk", "Custom_Cijk")))
mine = {}
for r in rows:
    for k in INTREE:
        if k in r["Name"]:
            n = r["Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
            mine[n] = mine.get(n, 0.0) + float(r["TotalDurationNs"])
own = sum(mine.values())
print(f"kernel time {tot / 1e6:.1f} ms; GEMMs {100 * (lib + own) / tot:.1f} % of it")
print(f"  hipBLASLt  {lib / 1e6:9.1f} ms  {100 * lib / (lib + own):5.1f} % of GEMM time")
print(f"  in-tree    {own / 1e6:9.1f} ms  {100 * own / (lib + own):5.1f} % of GEMM time")
for k, v in sorted(mine.items(), key=lambda kv: -kv[1]):
    print(f"    {k:40s} {v / 1e6:9.1f} ms")
