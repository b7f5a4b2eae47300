"""Per decode step of the diverged-cell decode: rows (attention grid), wall time, time per row, and where the
time of each row bucket goes per kernel family, from a rocprofv3 kernel trace (each step = 42 decode-attention
dispatches + the vocab head).  Shows how much of the decode the small-row tail steps take (weight-streaming
floor) and which kernels miss it.  Usage: python tools/decode_steps.py trace.csv"""
import collections
import csv
import sys


def family(n: str) -> str:
    for key in ("attn_decode", "decode_head", "head_merge", "gemm_pp_kernel<4>", "geglu", "add_rmsnorm", "rope_qkv", "gemm_skinny", "gemm_pp",
                "lowrank", "embed"):
        if key in n:
            return key
    if n.startswith("Cijk") or "Cijk_" in n or "gemm" in n.lower():
        return "hipblaslt"
    return n.split("(")[0][:28]


rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], int(r["Grid_Size_X"]),
               max(1, int(r.get("Workgroup_Size_X", 256) or 256))) for r in csv.DictReader(open(sys.argv[1])))
steps, cur = [], None
for s, e, n, gx, wx in rows:
    if "attn_decode" in n and "prefix" not in n:
        if cur is None:
            cur = [s, e, gx // wx, 0, collections.defaultdict(float)]
        cur[1] = e
        cur[3] += 1
        cur[4][family(n)] += (e - s) / 1e3
    elif cur is not None:
        cur[1] = e
        cur[4][family(n)] += (e - s) / 1e3
        if "decode_head" in n or "head_merge" in n:
            if cur[3] >= 40:
                steps.append((cur[2], (cur[1] - cur[0]) / 1e3, cur[4]))
            cur = None
BUCKETS = (64, 128, 256, 512, 1024, 2048, 4096, 8192)
hist = collections.defaultdict(lambda: [0, 0.0, 0, collections.defaultdict(float)])
for r, us, fam in steps:
    b = next((x for x in BUCKETS if r <= x), 1 << 30)
    h = hist[b]
    h[0] += 1
    h[1] += us
    h[2] += r
    for k, v in fam.items():
        h[3][k] += v
tot = sum(v[1] for v in hist.values())
print(f"decode steps {len(steps)}, {tot / 1e3:.1f} ms")
for b in sorted(hist):
    n, us, r, fam = hist[b]
    top = "  ".join(f"{k} {v / n:.0f}" for k, v in sorted(fam.items(), key=lambda kv: -kv[1])[:7])
    print(f"  rows <= {b:5d}: {n:5d} steps (mean {r / max(n, 1):6.0f} rows) {us / 1e3:9.1f} ms "
          f"({100 * us / max(tot, 1):.1f}%)  {us / max(n, 1):8.0f} us/step | us/step: {top}")
