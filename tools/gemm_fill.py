"""GEMM dispatches of a rocprofv3 kernel trace grouped by grid fill: workgroups per dispatch vs the 256 CUs
(under-filled GEMMs leave CUs idle).  Usage: python tools/gemm_fill.py <kernel_trace.csv> [t_lo_ns t_hi_ns]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
lo = int(sys.argv[2]) if len(sys.argv) > 2 else 0
hi = int(sys.argv[3]) if len(sys.argv) > 3 else 1 << 62
by = collections.defaultdict(lambda: [0, 0.0])
tot = 0.0
for r in rows:
    if "Cijk" not in r["Kernel_Name"]:
        continue
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if s < lo or s > hi:
        continue
    wg = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"]) // max(
        1, int(r["Workgroup_Size_X"]) * int(r["Workgroup_Size_Y"]) * int(r["Workgroup_Size_Z"]))
    b = "<128" if wg < 128 else "128-255" if wg < 256 else "256-511" if wg < 512 else "512-1023" if wg < 1024 else ">=1024"
    by[b][0] += 1
    by[b][1] += (e - s) / 1e6
    tot += (e - s) / 1e6
print(f"GEMM time {tot:.1f} ms")
for b in ("<128", "128-255", "256-511", "512-1023", ">=1024"):
    n, t = by[b]
    print(f"  workgroups {b:9s} {n:7d} dispatches {t:9.1f} ms ({100 * t / max(tot, 1e-9):.1f}%)")
