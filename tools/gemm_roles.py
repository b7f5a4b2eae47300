"""Attribute every GEMM dispatch of a rocprofv3 kernel trace to its role in the Gemma-2 forward by the kernel that
runs next on the stream (QKV -> rope / attention, o_proj -> add_rmsnorm2, gate|up -> geglu / down, down ->
add_rmsnorm2 after a GeGLU, lm_head -> decode_head, lens -> lens readouts), then print time per (role, kernel).

  python tools/gemm_roles.py gpurun_out/prof_x/run_kernel_trace.csv > summary.txt

Runs on the GPU box right after the profile (the trace is hundreds of MB; only the summary is kept).
"""
import csv
import sys
from collections import defaultdict


def is_gemm(n: str) -> bool:
    return n.startswith(("Cijk_", "Custom_Cijk")) or "gemm4_kernel" in n or "gemm_pp_kernel" in n or "gemm_ring_kernel" in n


def geglu_gemm(n: str) -> bool:
    """A gate|up GEMM with the fused GeGLU epilogue (gemm4 / ping-pong EPI 3, ring EPI 3 = third template argument)."""
    if "gemm4_kernel<256, 3>" in n or "gemm4_kernel<128, 3>" in n or "gemm_pp_kernel<3" in n:
        return True
    if "gemm_ring_kernel<" in n:
        args = n[n.find("<") + 1:].split(",")
        return len(args) > 2 and args[2].strip() == "3"
    return False


def g4_epi(n: str):
    """EPI template argument of a gemm4_kernel<BM, EPI> name, else None."""
    if "gemm4_kernel<" not in n:
        return None
    args = n[n.find("gemm4_kernel<") + 13:].split(">")[0].split(",")
    return args[1].strip() if len(args) > 1 else None


def same_split(a: str, b: str) -> bool:
    """Two launches of one row-split GEMM ("gs": 256-row then 128-row tiles, same epilogue)."""
    ea = g4_epi(a)
    return ea is not None and ea == g4_epi(b) and ea != "3"


def short(n: str) -> str:
    if n.startswith(("Cijk_", "Custom_Cijk")):
        i = n.find("MT")
        tag = n[i:n.find("_", i)] if i >= 0 else "?"
        return ("hipblaslt SK " if "_SK" in n else "hipblaslt ") + tag
    i = n.find("<")
    return n[n.find("::") + 2 if "::" in n else 0:n.find("(", i) if i >= 0 else 60].strip()


def role(prev: str, nxt: str) -> str:
    if "rope_qkv" in nxt or "attn" in nxt or "attention" in nxt:
        return "qkv"
    if "decode_head" in nxt or "xent" in nxt:
        return "lm_head"
    if "lens" in nxt or "row_lse" in nxt or "gather_probs" in nxt or "topk" in nxt:
        return "lens"
    if "geglu_kernel" in nxt:
        return "gate_up"
    if "add_rmsnorm" in nxt or "splitk_reduce" in nxt:
        if "geglu" in prev or geglu_gemm(prev):
            return "down"
        return "o_proj"
    if geglu_gemm(nxt):
        return "?"
    if is_gemm(nxt):
        return "gemm->gemm"
    return "other(" + short(nxt)[:30] + ")"


def main(path: str) -> None:
    rows = list(csv.DictReader(open(path)))
    key = lambda r: int(r["Start_Timestamp"])  # noqa: E731
    rows.sort(key=key)
    names = [r["Kernel_Name"] for r in rows]
    dur = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows]
    tot = sum(dur)
    acc = defaultdict(lambda: [0, 0])
    for i, n in enumerate(names):
        if not is_gemm(n):
            continue
        j, k = i + 1, i - 1
        while j < len(names) and same_split(n, names[j]):
            j += 1
        while k >= 0 and same_split(n, names[k]):
            k -= 1
        nxt = names[j] if j < len(names) else ""
        prev = names[k] if k >= 0 else ""
        if "splitk_reduce" in nxt and j + 1 < len(names):
            rl = role(prev, names[j + 1])
        else:
            rl = role(prev, nxt)
        # the fused gate|up + GeGLU GEMM is itself the gate_up role
        if geglu_gemm(n):
            rl = "gate_up(fused)"
        if "gemm4_kernel<256, 6>" in n:
            rl = "lens(fused)"
        a = acc[(rl, short(n))]
        a[0] += dur[i]
        a[1] += 1
    print(f"kernel time {tot / 1e6:.1f} ms")
    by_role = defaultdict(int)
    for (rl, k), (t, c) in acc.items():
        by_role[rl] += t
    for rl, t in sorted(by_role.items(), key=lambda x: -x[1]):
        print(f"{rl:16s} {t / 1e6:9.1f} ms  {100 * t / tot:5.1f} %")
    print()
    for (rl, k), (t, c) in sorted(acc.items(), key=lambda x: -x[1][0]):
        print(f"{rl:16s} {k:40s} {t / 1e6:9.1f} ms {c:7d} calls  {t / max(c, 1) / 1e3:8.1f} us/call")


if __name__ == "__main__":
    main(sys.argv[1])
