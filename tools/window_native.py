"""Kernel time inside the timed window of a bench run by kernel, and the share of PyTorch-native / runtime kernels
(fills, copies, index ops, rocPRIM, fp32 library GEMMs -- everything that is neither an in-tree HIP kernel nor a
bf16 hipBLASLt GEMM).  With a HIP runtime trace (``--hip-runtime-trace``) each native kernel is also attributed to
the host phase (``TB_PHASE_MARKS``) its launch API call was made in.

    TB_PHASE_MARKS=m.json rocprofv3 --kernel-trace [--hip-runtime-trace] --output-format csv -d D -o run -- python3 bench.py
    python tools/window_native.py D/run_kernel_trace.csv m.json [D/run_hip_api_trace.csv]
"""
import bisect
import collections
import csv
import json
import sys


def native(name: str) -> bool:
    if "(anonymous namespace)::" in name and "at::native" not in name:
        return False                                   # in-tree kernel (csrc/*.hip)
    if ("Cijk_" in name) and "_SB_" not in name and "_SS_" not in name:
        return False                                   # bf16 hipBLASLt GEMM
    return True


def main():
    marks = json.load(open(sys.argv[2]))
    steps = [t for n, t in marks if n.startswith("step")]
    t0, t1 = steps[0], [t for n, t in marks if n == "end"][-1]
    rows = [r for r in csv.DictReader(open(sys.argv[1]))
            if int(r["End_Timestamp"]) > t0 and int(r["Start_Timestamp"]) < t1]
    launch = {}
    if len(sys.argv) > 3:          # correlation id -> host time of the launching API call
        for r in csv.DictReader(open(sys.argv[3])):
            launch[r["Correlation_Id"]] = int(r["Start_Timestamp"])
    ph_t = [t for _, t in marks]
    ph_n = [n for n, _ in marks]
    tot = collections.Counter()
    calls = collections.Counter()
    by_phase = collections.defaultdict(collections.Counter)
    for r in rows:
        d = min(int(r["End_Timestamp"]), t1) - max(int(r["Start_Timestamp"]), t0)
        n = r["Kernel_Name"]
        tot[n] += d
        calls[n] += 1
        if native(n) and r.get("Correlation_Id") in launch:
            i = bisect.bisect_right(ph_t, launch[r["Correlation_Id"]]) - 1
            by_phase[ph_n[i] if i >= 0 else "?"][n[:70]] += d
    all_ns = sum(tot.values())
    nat = {n: t for n, t in tot.items() if native(n)}
    print(f"timed window {(t1 - t0) / 1e6:.1f} ms over {len(steps)} steps; kernel time {all_ns / 1e6:.1f} ms; "
          f"PyTorch-native / runtime kernels {sum(nat.values()) / 1e6:.1f} ms "
          f"({100 * sum(nat.values()) / max(all_ns, 1):.2f} %)")
    for n, t in sorted(nat.items(), key=lambda kv: -kv[1])[:25]:
        print(f"  {t / 1e6:8.2f} ms {calls[n]:6d}  {n[:120]}")
    if by_phase:
        print("native kernel time by the host phase that launched it:")
        for ph, c in sorted(by_phase.items(), key=lambda kv: -sum(kv[1].values())):
            print(f"  {ph:26s} {sum(c.values()) / 1e6:8.2f} ms  | " +
                  "  ".join(f"{k[:40]} {v / 1e6:.2f}" for k, v in c.most_common(4)))


if __name__ == "__main__":
    main()
