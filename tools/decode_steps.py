"""Per decode step of the diverged-cell decode: rows (attention grid), wall time, and the time per row, from a
rocprofv3 kernel trace (each step = 42 decode-attention dispatches + the vocab head).  Shows how much of the
decode the small-row tail steps take (weight-streaming floor).  Usage: python tools/decode_steps.py trace.csv"""
import collections
import csv
import sys

rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], int(r["Grid_Size_X"]))
              for r in csv.DictReader(open(sys.argv[1])))
steps, cur = [], None
for s, e, n, gx in rows:
    if "attn_decode_kernel" in n:
        if cur is None:
            cur = [s, e, gx // 256, 0]
        cur[1] = e
        cur[3] += 1
    elif "decode_head_kernel" in n and cur is not None:
        cur[1] = e
        if cur[3] >= 40:
            steps.append((cur[2], (cur[1] - cur[0]) / 1e3))
        cur = None
    elif cur is not None:
        cur[1] = e
hist = collections.defaultdict(lambda: [0, 0.0])
for r, us in steps:
    b = 64 if r <= 64 else 256 if r <= 256 else 512 if r <= 512 else 1024 if r <= 1024 else 2048 if r <= 2048 else 4096 if r <= 4096 else 8192
    hist[b][0] += 1
    hist[b][1] += us
tot = sum(v[1] for v in hist.values())
print(f"decode steps {len(steps)}, {tot / 1e3:.1f} ms")
for b in sorted(hist):
    n, us = hist[b]
    print(f"  rows <= {b:5d}: {n:5d} steps {us / 1e3:9.1f} ms ({100 * us / max(tot, 1):.1f}%)  {us / max(n, 1):8.0f} us/step")
