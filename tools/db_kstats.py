"""Kernel census from a rocprofv3 SQLite results database (rocprofv3's default output on ROCm 7:
``<dir>/<name>_results.db``): per kernel total ms, share, calls, mean us -- the same table as tools/kstats.py
prints from a kernel-trace CSV.

    python tools/db_kstats.py gpurun_out/.../run_results.db [--top 30]
"""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = list(c.execute("select name, count(*), sum(duration) from kernels group by name order by 3 desc"))
    tot = sum(r[2] for r in rows)
    print(f"total kernel time {tot / 1e6:.1f} ms, {sum(r[1] for r in rows)} dispatches")
    for name, n, d in rows[: a.top]:
        short = name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        print(f"{d / 1e6:10.2f} ms {100.0 * d / tot:6.2f} % {n:8d} {d / n / 1e3:10.1f} us  {short[:90]}")


if __name__ == "__main__":
    main()
