"""Summarise tools/lab/w4_lab.sh output: TF/s per shape and build:kernel (pp printed once)."""
import json
import sys
from collections import defaultdict

t = defaultdict(dict)
build = None
for line in open(sys.argv[1]):
    r = json.loads(line)
    if "build" in r:
        build = r["build"]
    elif "check_ok" in r:
        print(build, "check_ok", r["check_ok"])
    elif "kernel" in r:
        k = r["kernel"] if r["kernel"] == "pp" else f"{build}:{r['kernel']}"
        t[(r["M"], r["N"], r["K"])].setdefault(k, r["TF_med"])
for k, v in sorted(t.items()):
    print(k, "  ".join(f"{kk}={vv:.0f}" for kk, vv in v.items()))
