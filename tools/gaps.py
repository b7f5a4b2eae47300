"""GPU idle gaps from a rocprofv3 kernel_trace.csv: where the device waits on the host."""
import csv
import re
import sys


def short(n):
    n = n.replace("void ", "").replace("(anonymous namespace)::", "")
    if "Cijk" in n:
        return "gemm"
    return re.sub(r"[<(].*", "", n)[:40]


rows = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]))
               for r in csv.DictReader(open(sys.argv[1]))), key=lambda x: x[0])
t_lo = rows[0][0] if len(sys.argv) < 3 else rows[0][0] + int(float(sys.argv[2]) * 1e9)
rows = [r for r in rows if r[0] >= t_lo]
busy, gaps = 0, []
end = rows[0][0]
for i, (s, e, n) in enumerate(rows):
    if s > end:
        gaps.append((s - end, i))
    busy += max(0, e - max(s, end))
    end = max(end, e)
span = end - rows[0][0]
print(f"span {span / 1e6:.1f} ms busy {busy / 1e6:.1f} ms ({100 * busy / span:.1f}%) gaps>0.2ms total "
      f"{sum(g for g, _ in gaps if g > 2e5) / 1e6:.1f} ms")
for g, i in sorted(gaps, reverse=True)[:25]:
    print(f"{g / 1e6:8.2f} ms after {rows[i - 1][2]:40s} before {rows[i][2]:40s} at {(rows[i][0] - rows[0][0]) / 1e6:9.1f} ms")
