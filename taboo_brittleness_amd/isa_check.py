"""Static check of gemm4's counted-wait K loop (csrc/gemm4.hip, ``G4_CNT``).

With ``G4_CNT`` the 256-row tile's fragment reads are inline-asm ``ds_read_b128``: the compiler takes their results
as ready when the asm statement ends and only the kernel's own ``s_waitcnt lgkmcnt(N)`` statements make them so.
If hipcc ever copies, spills or overwrites a fragment register between its read and the wait that retires it, the
kernel computes on stale data.  This simulates the LDS counter over the K loop (the basic block with the most MFMAs,
run twice so the reads issued at the end of one period are checked against the next period's waits) and reports
every instruction that reads or writes a register of a still-outstanding LDS read.

Run by the extension build (``build.py``) whenever gemm4.hip is compiled: if any kernel fails the check, gemm4.hip is
rebuilt with ``-DG4_CNT=0`` (compiler-visible reads drained every period: correct with any compiler, slower) and
a warning is printed, so a different hipcc can never silently produce wrong projections.

  python -m taboo_brittleness_amd.isa_check   # compiles csrc/gemm4.hip for gfx950 and checks every 256-row kernel
"""
from __future__ import annotations

import os
import re
import subprocess
import sys
import tempfile
from typing import Dict, List, Set, Tuple

CSRC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "csrc")
HIPCC = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "bin", "hipcc")

_REG = re.compile(r"\b([va])(?:\[(\d+):(\d+)\]|(\d+)(?!\w))")


def _regs(text: str) -> Set[Tuple[str, int]]:
    out = set()
    for m in _REG.finditer(text):
        kind = m.group(1)
        if m.group(4) is not None:
            out.add((kind, int(m.group(4))))
        else:
            out.update((kind, r) for r in range(int(m.group(2)), int(m.group(3)) + 1))
    return out


def _split_operands(ins: str) -> Tuple[str, List[str]]:
    op, _, rest = ins.partition(" ")
    rest = rest.split(" offset:")[0]
    parts, depth, cur = [], 0, ""
    for ch in rest:
        if ch == "[":
            depth += 1
        elif ch == "]":
            depth -= 1
        if ch == "," and depth == 0:
            parts.append(cur.strip())
            cur = ""
        else:
            cur += ch
    if cur.strip():
        parts.append(cur.strip())
    return op, parts


def check_loop(ins: List[str], pre: List[str] = ()) -> List[str]:
    """Violations in the tile prologue ``pre`` (the blocks from the first fragment reads to the loop, laid out in
    order) followed by the straight-line K-loop body, simulated twice: the back edge carries the outstanding reads."""
    pending: List[Set[Tuple[str, int]]] = []        # destination registers of outstanding LDS ops, oldest first
    bad = []
    for rnd, seq in enumerate((list(pre) + list(ins), ins)):
        for k, line in enumerate(seq):
            op, ops = _split_operands(line)
            if op == "s_waitcnt":
                m = re.search(r"lgkmcnt\((\d+)\)", line)
                if m:
                    n = int(m.group(1))
                    while len(pending) > n:
                        pending.pop(0)
                continue
            if not op.startswith(("v_", "ds_", "buffer_", "global_", "scratch_")):
                continue
            is_store = op.startswith(("ds_write", "buffer_store", "global_store", "scratch_store"))
            dst = set() if is_store or not ops else _regs(ops[0])
            src = set()
            for o in (ops if is_store else ops[1:]):
                src |= _regs(o)
            if op.startswith("v_mfma"):
                src |= dst                      # accumulate: C = D
            busy = set().union(*pending) if pending else set()
            hit = (src | dst) & busy
            if hit:
                bad.append(f"pass {rnd} #{k}: {line}  touches outstanding {sorted(hit)[:4]}")
            if op.startswith("ds_"):
                pending.append(dst)
    return bad


def loops(asm: str) -> Dict[str, Tuple[List[str], List[str]]]:
    """{kernel: (tile prologue, K-loop body)} for every gemm4_kernel<256, EPI> in a gfx950 assembly listing."""
    funcs: Dict[str, List[str]] = {}
    cur = None
    for line in asm.split("\n"):
        m = re.match(r"^(_Z\S+):", line)
        if m:
            cur = m.group(1)
            funcs[cur] = []
            continue
        if cur is not None:
            funcs[cur].append(line)
    out = {}
    for name, body in funcs.items():
        m = re.search(r"gemm4_kernelILi(\d+)ELi(\d+)E", name)
        if not m or m.group(1) != "256":
            continue
        blocks, cur_b = [], []
        for line in body:
            if re.match(r"^\.LBB", line):
                blocks.append(cur_b)
                cur_b = []
            else:
                s = line.strip()
                if s and not s.startswith((";", ".")):
                    cur_b.append(s.split(";")[0].strip())
        blocks.append(cur_b)
        li = max(range(len(blocks)), key=lambda i: sum("mfma" in x for x in blocks[i]))
        pi = li - 1                    # the prologue: the nearest earlier block with fragment reads and no MFMA
        while pi >= 0 and not (any(x.startswith("ds_read_b128") for x in blocks[pi]) and
                               not any("mfma" in x for x in blocks[pi])):
            pi -= 1
        pre = [x for b in blocks[max(pi, 0): li] for x in b] if pi >= 0 else []
        out[f"gemm4_kernel<256, {m.group(2)}>"] = (pre, blocks[li])
    return out


def compile_asm(extra=()) -> str:
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, "g4.hip")
        with open(src, "w") as f:
            f.write(f'#include "{os.path.join(CSRC, "gemm4.hip")}"\n'
                    "bool tb_softcap_compact_params(float, const uint16_t**, int*, int*, float*) { return false; }\n")
        out = os.path.join(d, "g4.s")
        # the extension's device flags (taboo_brittleness_amd/build.py)
        subprocess.run([HIPCC, "--offload-arch=gfx950", "-fPIC", "-O3", "-std=c++17", "-munsafe-fp-atomics",
                        "--cuda-device-only", "-S", "-I", CSRC, src, "-o", out] + list(extra), check=True,
                       capture_output=True)
        with open(out) as f:
            return f.read()


def violations(asm: str) -> Dict[str, List[str]]:
    """{kernel: violations} of every 256-row gemm4 kernel in ``asm`` (empty lists when the counted waits are safe);
    a missing kernel or tile prologue counts as a violation."""
    ls = loops(asm)
    out = {k: check_loop(body, pre) + ([] if pre else ["no tile prologue found"]) for k, (pre, body) in ls.items()}
    if not ls:
        out["gemm4_kernel<256, *>"] = ["no 256-row kernel found"]
    return out


def main() -> int:
    ls = loops(compile_asm())
    bad = 0
    for k, (pre, body) in sorted(ls.items()):
        v = check_loop(body, pre)
        if not pre:
            v.append("no tile prologue found")
        nw = sum("lgkmcnt(" in x and "lgkmcnt(0)" not in x for x in body)
        print(f"{k}: {len(body)} instructions, {sum('mfma' in x for x in body)} MFMAs, {nw} counted waits, "
              f"{len(v)} violations")
        for x in v[:5]:
            print("   ", x)
        bad += len(v)
    return 1 if bad or not ls else 0


if __name__ == "__main__":
    sys.exit(main())
