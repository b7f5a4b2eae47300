"""Per-kernel summary of the PMC passes written by tools/pmc_kernels.sh.

Usage: python tools/pmc_summary.py gpurun_out/pmc > profiles/pmc_hot_kernels.txt

Per kernel (mean over its dispatches): duration (kernel-trace run), MFMA busy share of the SIMD
cycles: SQ_VALU_MFMA_BUSY_CYCLES / (traced duration x 2.4 GHz x 1024 SIMDs) — the counter sums over
all 256 CUs x 4 SIMDs; the duration comes from the kernel-trace run because per-dispatch GRBM_GUI_ACTIVE
includes the profiler's serialisation window), LDS bank-conflict cycles per LDS-active cycle, and memory-side bytes
(FETCH_SIZE / WRITE_SIZE are KiB; on gfx950 FETCH_SIZE reads ~1/2 of a wide coalesced stream's bytes,
so the read side is also shown doubled) with the bandwidth they imply over the traced duration.
"""
import csv
import os
import sys
from collections import defaultdict

KEEP = ("attn_decode", "geglu", "add_rmsnorm2", "gemm_nt_kernel", "gemm_pp_kernel", "kv_fanout", "decode_head", "Cijk")


def short(name: str) -> str:
    for k in KEEP:
        if k in name:
            if k == "Cijk":
                return "hipblaslt " + name.split("_MT")[1].split("_")[0] if "_MT" in name else "hipblaslt"
            return name.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
    return ""


def load_counters(path):
    acc = defaultdict(lambda: defaultdict(list))
    with open(path) as f:
        for r in csv.DictReader(f):
            k = short(r["Kernel_Name"])
            if k:
                acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return acc


def main(d):
    dur = defaultdict(list)
    with open(os.path.join(d, "trace", "run_kernel_stats.csv")) as f:
        for r in csv.DictReader(f):
            k = short(r["Name"])
            if k:
                dur[k].append(float(r["AverageNs"]))
    c = defaultdict(dict)
    for sub in ("sq", "fetch", "write"):
        p = os.path.join(d, sub, "run_counter_collection.csv")
        if os.path.exists(p):
            for k, v in load_counters(p).items():
                for n, vals in v.items():
                    c[k][n] = sum(vals) / len(vals)
    print(f"{'kernel':34s} {'us':>8s} {'MFMA util':>10s} {'LDSconf/act':>11s} {'rd MB':>8s} {'rd x2 MB':>9s} "
          f"{'wr MB':>8s} {'rd+wr GB/s':>11s} {'(rd x2) GB/s':>13s}")
    for k in sorted(set(dur) | set(c)):
        us = sum(dur.get(k, [0])) / max(len(dur.get(k, [1])), 1) / 1e3
        cc = c.get(k, {})
        busy = us * 1e-6 * 2.4e9 * 1024
        mf = cc.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        lds = cc.get("SQ_LDS_IDX_ACTIVE", 0.0)
        conf = cc.get("SQ_LDS_BANK_CONFLICT", 0.0)
        rd = cc.get("FETCH_SIZE", 0.0) / 1024
        wr = cc.get("WRITE_SIZE", 0.0) / 1024
        bw = (rd + wr) / 1e3 / (us * 1e-6) if us else 0.0
        bw2 = (2 * rd + wr) / 1e3 / (us * 1e-6) if us else 0.0
        print(f"{k:34s} {us:8.1f} {mf / busy if busy else 0:10.3f} {conf / lds if lds else 0:11.3f} {rd:8.1f} "
              f"{2 * rd:9.1f} {wr:8.1f} {bw:11.0f} {bw2:13.0f}")
    print()
    print("raw means per dispatch:")
    for k in sorted(c):
        print(f"  {k}: " + ", ".join(f"{n}={v:.4g}" for n, v in sorted(c[k].items())))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc")
