"""GPU idle time inside the timed window of a bench run, attributed to the host phase the launching
thread was in when the GPU ran dry.

    TB_PHASE_MARKS=m.json rocprofv3 --kernel-trace ... -- python3 bench.py ...   (no TB_PHASE_TIMING: no syncs)
    python tools/window_gaps.py <kernel_trace.csv> m.json

Marks are host ``time.monotonic_ns()`` stamps (the clock rocprofv3 stamps kernels with): ``stepK`` at each
timed step's start, ``end`` after the final synchronize, and every runner phase entry in between."""
import bisect
import collections
import csv
import json
import re
import sys


def short(n):
    n = n.replace("void ", "").replace("(anonymous namespace)::", "")
    if "Cijk" in n:
        return "gemm"
    return re.sub(r"[<(].*", "", n)[:40]


marks = json.load(open(sys.argv[2]))
steps = [(n, t) for n, t in marks if n.startswith("step")]
t_end = [t for n, t in marks if n == "end"][-1]
t0 = steps[0][1]
rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]))
              for r in csv.DictReader(open(sys.argv[1])))
rows = [r for r in rows if r[1] > t0 and r[0] < t_end]
ph_t = [t for _, t in marks]
ph_n = [n for n, _ in marks]


def phase_at(t):
    i = bisect.bisect_right(ph_t, t) - 1
    return ph_n[i] if i >= 0 else "?"


busy, end = 0, t0
idle = collections.Counter()
cnt = collections.Counter()
gaps = []
for s, e, n in rows:
    s_ = max(s, t0)
    if s_ > end:
        g = s_ - end
        ph = phase_at(end)
        idle[ph] += g
        cnt[ph] += 1
        gaps.append((g, end, n))
    busy += max(0, min(e, t_end) - max(s_, end))
    end = max(end, min(e, t_end))
if t_end > end:
    idle["<tail>"] += t_end - end
span = t_end - t0
print(f"timed window {span / 1e6:.1f} ms over {len(steps)} steps; GPU busy {busy / 1e6:.1f} ms "
      f"({100 * busy / span:.1f}%), idle {(span - busy) / 1e6:.1f} ms")
print("idle by host phase at the moment the GPU ran dry (ms, gaps):")
for ph, g in idle.most_common():
    print(f"  {ph:28s} {g / 1e6:9.1f}  {cnt[ph]:6d}")
print("idle per timed step by host phase (ms):")
bounds = [t for _, t in steps] + [t_end]
for i in range(len(steps)):
    per = collections.Counter()
    for g, t, n in gaps:
        if bounds[i] <= t < bounds[i + 1]:
            per[phase_at(t)] += g
    print(f"  {steps[i][0]} ({(bounds[i + 1] - bounds[i]) / 1e6:.0f} ms): " +
          ", ".join(f"{ph} {g / 1e6:.1f}" for ph, g in per.most_common(8)))
print("largest gaps:")
for g, t, n in sorted(gaps, reverse=True)[:20]:
    print(f"  {g / 1e6:8.2f} ms at +{(t - t0) / 1e6:9.1f} ms in {phase_at(t):24s} next kernel {n}")
