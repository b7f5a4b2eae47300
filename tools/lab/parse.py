"""Summarise tools/lab/gemm_lab.sh output: one line per (variant, shape)."""
import json
import re
import sys

for line in open(sys.argv[1]):
    m = re.match(r'\{"variant": "(\w+)", "r": (\{.*?\})', line.strip())
    if m:
        r = json.loads(m.group(2))
        print(f"{m.group(1):12s} M={r['M']:5d} N={r['N']:6d} K={r['K']:5d} epi={r['epi']} us={r['us_best']:7.1f} TF={r['TF_best']:7.1f}")
    elif line.strip() not in ("}", ""):
        print(line.rstrip())
