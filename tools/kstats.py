"""Summarise a rocprofv3 kernel_stats.csv: short names, calls, total ms, share."""
import csv
import re
import sys


def short(n: str) -> str:
    if n.startswith("Cijk") or n.startswith("Custom_Cijk"):
        mt = re.search(r"MT(\d+x\d+x\d+)", n)
        return f"hipblaslt_gemm[{mt.group(1) if mt else '?'}]"
    n = n.replace("void ", "").replace("(anonymous namespace)::", "")
    n = re.sub(r"\(.*", "", n)
    return n[:70]


rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
agg = {}
for r in rows:
    k = short(r["Name"])
    a = agg.setdefault(k, [0, 0.0])
    a[0] += int(r["Calls"])
    a[1] += float(r["TotalDurationNs"])
print(f"total kernel time {tot / 1e6:.1f} ms")
for k, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[: int(sys.argv[2]) if len(sys.argv) > 2 else 30]:
    print(f"{t / 1e6:10.2f} ms {100 * t / tot:6.2f}% {c:8d}  {k}")
