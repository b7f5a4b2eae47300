"""Per-kernel PMC summary of tools/lab/pmc_lab.sh runs: wall (from the counter run's own timestamps),
effective clock = GRBM_GUI_ACTIVE / 8 XCDs / wall, MFMA busy share of SIMD cycles at that clock,
LDS bank-conflict cycles per LDS-active cycle."""
import csv
import sys
from collections import defaultdict

for d in sys.argv[1:]:
    rows = list(csv.DictReader(open(f"{d}/run_counter_collection.csv")))
    per = defaultdict(lambda: defaultdict(float))
    dur = {}
    for r in rows:
        name = r["Kernel_Name"]
        if "gemm" not in name.lower() and "Cijk" not in name:
            continue
        key = (name[:60], r["Dispatch_Id"])
        per[key][r["Counter_Name"]] += float(r["Counter_Value"])
        dur[key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    agg = defaultdict(list)
    for (name, _), c in per.items():
        agg[name].append((c, dur[(name, _)]))
    for name, xs in agg.items():
        xs = xs[1:] if len(xs) > 2 else xs    # skip the first (cold) dispatch
        n = len(xs)
        wall = sum(t for _, t in xs) / n
        gui = sum(c["GRBM_GUI_ACTIVE"] for c, _ in xs) / n
        clk = gui / 8 / wall / 1e9
        mfma = sum(c["SQ_VALU_MFMA_BUSY_CYCLES"] for c, _ in xs) / n
        util = mfma / (wall * clk * 1e9 * 1024)
        conf = sum(c["SQ_LDS_BANK_CONFLICT"] for c, _ in xs) / max(1.0, sum(c["SQ_LDS_IDX_ACTIVE"] for c, _ in xs))
        waves = sum(c["SQ_WAVES"] for c, _ in xs) / n
        print(f"{d.split('/')[-1]:10s} {name[:44]:44s} n={n} wall={wall*1e6:7.1f}us clk={clk:4.2f}GHz "
              f"mfma_util={util:5.3f} lds_conf/act={conf:5.3f} waves={waves:.0f}")
