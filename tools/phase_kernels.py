"""Kernel time per sweep phase: joins a rocprofv3 kernel_trace.csv with the phase boundaries bench.py
writes under TB_PHASE_TIMING=1 TB_PHASE_MARKS=<json> (both on the monotonic clock).
Usage: python tools/phase_kernels.py <kernel_trace.csv> <marks.json> [first_step_mark_index]"""
import bisect
import collections
import csv
import json
import re
import sys

marks = json.load(open(sys.argv[2]))
t = [m[1] for m in marks]
rows = list(csv.DictReader(open(sys.argv[1])))


def short(n):
    n = n.replace("void ", "").replace("(anonymous namespace)::", "")
    if "Cijk" in n:
        return "gemm"
    return re.sub(r"[<(].*", "", n)[:32]


lo = t[int(sys.argv[3])] if len(sys.argv) > 3 else t[0]
per = collections.defaultdict(lambda: collections.defaultdict(float))
span = collections.defaultdict(float)
for i in range(1, len(marks)):
    if t[i - 1] >= lo:
        span[marks[i][0]] += (t[i] - t[i - 1]) / 1e6
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if s < lo:
        continue
    k = bisect.bisect_right(t, s)
    if k == 0 or k >= len(marks):
        continue
    per[marks[k][0]][short(r["Kernel_Name"])] += (e - s) / 1e6
for ph in sorted(per, key=lambda p: -sum(per[p].values())):
    tot = sum(per[ph].values())
    top = sorted(per[ph].items(), key=lambda kv: -kv[1])[:6]
    print(f"{ph:22s} wall {span.get(ph, 0):8.1f} ms  kernels {tot:8.1f} ms  | " +
          "  ".join(f"{k} {v:.1f}" for k, v in top))
