"""Kernel time per kernel over the LAST ``seconds`` of a rocprofv3 kernel_trace.csv (the bench's timed steps when
run with ``--no-post-forcing --no-config2``: setup, graph precapture and warmup excluded), with the GEMM share
(in-tree vs hipBLASLt).   python tools/window_kstats.py run_kernel_trace.csv SECONDS"""
import collections
import csv
import re
import sys


def short(n):
    n = n.replace("void ", "").replace("(anonymous namespace)::", "")
    return re.sub(r"\(.*", "", n)[:72]


rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(sys.argv[1]))]
t_end = max(e for _, e, _ in rows)
t_lo = t_end - int(float(sys.argv[2]) * 1e9)
agg = collections.defaultdict(lambda: [0, 0])
for s, e, n in rows:
    if s >= t_lo:
        a = agg[short(n)]
        a[0] += e - s
        a[1] += 1
tot = sum(v[0] for v in agg.values())
print(f"window {float(sys.argv[2]):.2f} s, kernel time {tot / 1e6:.1f} ms")
gemm = {k: v[0] for k, v in agg.items() if "gemm4_kernel" in k or "gemm_ring_kernel" in k or "Cijk" in k
        or "hipblaslt" in k.lower()}
lib = sum(v for k, v in gemm.items() if "Cijk" in k or "hipblaslt" in k.lower())
gt = sum(gemm.values())
print(f"GEMMs {100 * gt / tot:.1f} % of kernel time; in-tree {100 * (gt - lib) / max(gt, 1):.1f} % of GEMM time, "
      f"hipBLASLt {100 * lib / max(gt, 1):.1f} %")
for k, (t, c) in sorted(agg.items(), key=lambda x: -x[1][0])[:32]:
    print(f"{t / 1e6:9.1f} ms {100 * t / tot:5.2f} % {c:7d}  {k}")
