"""Summarise tools/lab/w4_pmc.sh: per kernel, effective clock (GRBM_GUI_ACTIVE / 8 / wall), MFMA busy share,
LDS conflict ratio, and the wave-cycle split (waiting / issue-stalled / active) from the second pass."""
import csv
import sys
from collections import defaultdict


def load(path):
    per = defaultdict(lambda: defaultdict(float))
    dur = {}
    for r in csv.DictReader(open(path)):
        key = (r["Kernel_Name"][:70], r["Dispatch_Id"])
        per[key][r["Counter_Name"]] += float(r["Counter_Value"])
        dur[key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    agg = defaultdict(list)
    for k, c in per.items():
        agg[k[0]].append((c, dur[k]))
    return agg


d = sys.argv[1]
a1 = load(f"{d}/p1/run_counter_collection.csv")
a2 = load(f"{d}/p2/run_counter_collection.csv")
for name, xs in a1.items():
    if "fill" in name or "ref_" in name:
        continue
    n = len(xs)
    wall = sum(t for _, t in xs) / n
    clk = sum(c["GRBM_GUI_ACTIVE"] for c, _ in xs) / n / 8 / wall / 1e9
    util = sum(c["SQ_VALU_MFMA_BUSY_CYCLES"] for c, _ in xs) / n / (wall * clk * 1e9 * 1024)
    conf = sum(c["SQ_LDS_BANK_CONFLICT"] for c, _ in xs) / max(1.0, sum(c["SQ_LDS_IDX_ACTIVE"] for c, _ in xs))
    ys = a2.get(name, [])
    wc = sum(c["SQ_WAVE_CYCLES"] for c, _ in ys) or 1.0
    split = " ".join(f"{k[3:]}={sum(c[k] for c, _ in ys) / wc:.2f}" for k in
                     ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS",
                      "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_MISC"))
    print(f"{name[:60]:60s} n={n} wall={wall * 1e6:7.1f}us clk={clk:4.2f}GHz mfma_util={util:5.3f} "
          f"lds_conf={conf:5.3f} | {split}")
