"""Per-kernel table of every counter collected by tools/lab/pmc_passes.sh (mean per dispatch; *_CYCLES-like SQ counters
also as a share of SQ_WAVE_CYCLES, TA/TCP cycle counters per microsecond of wall time)."""
import csv
import glob
import os
import sys
from collections import defaultdict

d = sys.argv[1]
tot = defaultdict(lambda: defaultdict(float))
nd = defaultdict(lambda: defaultdict(int))
wall = defaultdict(list)
for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
    per = defaultdict(lambda: defaultdict(float))
    durs = {}
    for r in csv.DictReader(open(f)):
        k = (r["Kernel_Name"][:60], r["Dispatch_Id"])
        per[k][r["Counter_Name"]] += float(r["Counter_Value"])
        durs[k] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    for (name, _), cs in per.items():
        wall[name].append(durs[(name, _)])
        for c, v in cs.items():
            tot[name][c] += v
            nd[name][c] += 1
for name in tot:
    if "elementwise" in name or "distribution" in name:
        continue
    w = sum(wall[name]) / len(wall[name])
    m = {c: tot[name][c] / nd[name][c] for c in tot[name]}
    wc = m.get("SQ_WAVE_CYCLES", 1.0)
    print(f"== {name}  wall={w * 1e6:.1f}us")
    if "GRBM_GUI_ACTIVE" in m:
        clk = m["GRBM_GUI_ACTIVE"] / 8 / w / 1e9
        print(f"   clk={clk:.2f}GHz mfma_util={m.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / (w * clk * 1e9 * 1024):.3f}")
    for c in sorted(m):
        if c in ("SQ_WAVE_CYCLES", "GRBM_GUI_ACTIVE", "GRBM_COUNT"):
            continue
        extra = f"  /wave_cyc={m[c] / wc:.3f}" if c.startswith(("SQ_WAIT", "SQ_ACTIVE", "SQ_INST_CYCLES")) else ""
        print(f"   {c:36s} {m[c]:16.1f}{extra}")
