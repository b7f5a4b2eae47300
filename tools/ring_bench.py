"""Ring GEMM (csrc/gemm_ring.hip) check + timing at the Gemma-2-9B projection shapes and decode / mid row counts.

For every (shape, epilogue, M) it first checks that each ring tile's output is bit-identical to the unsplit gemm4
kernel (the batch-invariance contract), then times the ring tiles against gemm4 (g256 / g128), split-K gemm4
(k256 / k128 / k64; not batch-invariant) and hipBLASLt, interleaved in rounds in one process, weights rotated over
copies larger than the Infinity Cache (a decode step streams every weight from HBM).  One JSON line per point in
``tools/gemm_dispatch_tune.py``'s raw format, so ``tools/gemm_dispatch_table.py`` can build the dispatch table.

  python tools/ring_bench.py --shapes o,down,qkv,gu --ms 16,64,256,1024 --out gpurun_out/ring.jsonl
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from taboo_brittleness_amd import ops  # noqa: E402
from taboo_brittleness_amd.ops import _ext  # noqa: E402
from taboo_brittleness_amd.ops import reference as ref  # noqa: E402
from taboo_brittleness_amd.runtime import gemm_dispatch as GD  # noqa: E402
from taboo_brittleness_amd.runtime.tuning import enable_tuned_gemms  # noqa: E402

SHAPES = {"qkv": (8192, 3584), "o": (3584, 4096), "gu": (28672, 3584), "down": (3584, 14336), "head": (256000, 3584)}
EPIS = {"qkv": [0, 4], "o": [0, 5], "gu": [3], "down": [0, 5], "head": [0]}


def rname(bm: int, bn: int, rv: int) -> str:
    """Dispatch choice name of a ring tile: ``r<bm>x<bn>`` (64 KB ring), ``r<bm>x<bn>b`` (144 KB ring), ``r<bm>x<bn>c``
    (144 KB ring, 4-8 K tiles per stage)."""
    return f"r{bm}x{bn}" + ("", "b", "c")[rv]


def timed(fn, reps: int) -> float:
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1000.0 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="o,down,qkv,gu")
    ap.add_argument("--ms", default="16,32,64,128,256,512,768,1024,1536,2048",
                    help="row counts, or 'auto': the row counts of the dispatch table's entry for the shape")
    ap.add_argument("--ring-max-m", type=int, default=3072, help="ring tiles timed up to this M")
    ap.add_argument("--split-max-m", type=int, default=2400, help="split-K variants timed up to this M")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--tiles", default="", help="comma list of bmxbn to time (default: all built)")
    ap.add_argument("--others", default="g256,g128,gs,k256,k128,k64")
    ap.add_argument("--no-check", action="store_true")
    ap.add_argument("--tag", default="gemma2-9b_P100_E4_new50", help="TunableOp table of the hipBLASLt candidates")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "ring.jsonl"))
    args = ap.parse_args()
    k = _ext.load()
    dev = torch.device("cuda:0")
    enable_tuned_gemms(args.tag)
    torch.backends.cuda.matmul.allow_bf16_reduced_precision_reduction = False
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    out = open(args.out, "a")
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    bad = 0
    for name in args.shapes.split(","):
        N, K = SHAPES[name]
        wbytes = N * K * 2
        ncopy = max(1, min(8, -(-600 * 2 ** 20 // wbytes)))
        Ws = [(torch.rand(N, K, device=dev, generator=g) * 2 - 1).to(torch.bfloat16) for _ in range(ncopy)]
        if name == "gu":
            idx = ops.geglu_interleave_index(N // 2, dev)
            Ws = [w.index_select(0, idx).contiguous() for w in Ws]
        for epi in EPIS[name]:
            kepi = 0 if epi == 5 else epi
            tiles = [tuple(t) for t in k.gemm_ring_tiles(kepi)]
            if args.tiles:
                want = {tuple(int(v) for v in s.split("x")) for s in args.tiles.split(",")}
                tiles = [t for t in tiles if t in want]
            if args.ms == "auto":
                tab = json.load(open(os.path.join(ROOT, "configs", "gemm_dispatch", "gemma2-9b.json")))["shapes"]
                ent = tab.get(f"{N},{K},{epi}") or tab.get(f"{N},{K},0") or []
                ms = sorted({int(r[0]) for r in ent})
            else:
                ms = [int(v) for v in args.ms.split(",")]
            for M in ms:
                A = (torch.rand(M, K, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
                ncol = N // 2 if epi == 3 else N
                C = torch.empty(M, ncol, device=dev, dtype=torch.bfloat16)
                it = [0]

                def nxt():
                    it[0] = (it[0] + 1) % len(Ws)
                    return Ws[it[0]]

                var = {}
                ok_tiles = [(t[0], t[1], v) for t in tiles for v in (0, 1, 2) if k.gemm_ring_ok(M, N, K, kepi, t[0], t[1], v)
                            and M <= args.ring_max_m and t[0] <= max(16, 2 * M)]
                others = [c for c in args.others.split(",") if
                          not (c.startswith("k") and (M > args.split_max_m or (c == "k64" and M > 512))) and
                          not (c.isdigit() and (M < 256 or epi in (4, 5))) and not (c == "gs" and M < 2048)]
                if epi == 4:
                    Hq, Hkv, HD, S = 16, 8, 256, 512
                    nslot = min(M, 256)
                    pos = torch.randint(0, S, (M,), device=dev, dtype=torch.int32)
                    slot = (torch.arange(M, device=dev, dtype=torch.int32) % nslot).contiguous()
                    cos_t, sin_t = ref.rope_tables(HD, 8192, 10000.0, dev)
                    cos_t, sin_t = cos_t.contiguous(), sin_t.contiguous()
                    cs = ops.rope_cs(cos_t, sin_t)
                    kc = torch.zeros(nslot, Hkv, S, HD, device=dev, dtype=torch.bfloat16)
                    vc = torch.zeros_like(kc)
                    q = torch.empty(M, Hq, HD, device=dev, dtype=torch.bfloat16)
                    if not args.no_check:
                        # distinct (slot, pos) per row so the cache writes do not collide
                        pos_c = (torch.arange(M, device=dev, dtype=torch.int32) // nslot).contiguous()
                        k.gemm4_qkv_rope(A, Ws[0], pos_c, slot, cs, q, kc, vc, Hq, Hkv, 128)
                        q0, k0, v0 = q.clone(), kc.clone(), vc.clone()
                        for (bm, bn, rv) in ok_tiles:
                            q.zero_(); kc.zero_(); vc.zero_()
                            k.gemm_ring_qkv_rope(A, Ws[0], pos_c, slot, cs, q, kc, vc, Hq, Hkv, bm, bn, rv)
                            same = torch.equal(q, q0) and torch.equal(kc, k0) and torch.equal(vc, v0)
                            if not same:
                                bad += 1
                                print(f"MISMATCH {name} epi {epi} M {M} r{bm}x{bn} v{rv}", flush=True)
                    for (bm, bn, rv) in ok_tiles:
                        var[rname(bm, bn, rv)] = (lambda bm_, bn_, rv_: lambda: k.gemm_ring_qkv_rope(
                            A, nxt(), pos, slot, cs, q, kc, vc, Hq, Hkv, bm_, bn_, rv_))(bm, bn, rv)
                    for ch in others:
                        if ch == "gs":
                            M1 = GD.split_rows(M, N)

                            def rope_split(M1=M1):
                                w_ = nxt()
                                for r0, r1, tr in ((0, M1, 256), (M1, M, 128)):
                                    if r1 > r0:
                                        k.gemm4_qkv_rope(A[r0:r1], w_, pos[r0:r1], slot[r0:r1], cs, q[r0:r1],
                                                         kc, vc, Hq, Hkv, tr)
                            var[ch] = rope_split
                        elif ch.startswith("g"):
                            var[ch] = (lambda r_: lambda: k.gemm4_qkv_rope(A, nxt(), pos, slot, cs, q, kc, vc,
                                                                           Hq, Hkv, r_))(int(ch[1:]))
                    var["blas"] = lambda: (torch.matmul(A, nxt().t(), out=C),
                                           ops.rope_qkv_cache(C, pos, slot, cos_t, sin_t, kc, vc, Hq, Hkv, HD, q_out=q))
                else:
                    if not args.no_check:
                        ref_out = torch.empty_like(C)
                        ops.tb_gemm(A, Ws[0], ref_out, None, None, kepi, "g128")
                        for (bm, bn, rv) in ok_tiles:
                            C.zero_()
                            k.gemm_ring(A, Ws[0], C, kepi, bm, bn, rv)
                            if not torch.equal(C, ref_out):
                                bad += 1
                                d = (C.float() - ref_out.float()).abs().max().item()
                                print(f"MISMATCH {name} epi {epi} M {M} r{bm}x{bn} v{rv} maxdiff {d}", flush=True)
                    if epi == 5:
                        h0 = (torch.rand(M, N, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
                        wp = (torch.rand(N, device=dev, generator=g) * 0.2 - 0.1).to(torch.bfloat16)
                        xo = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
                        for (bm, bn, rv) in ok_tiles:
                            var[rname(bm, bn, rv)] = (lambda bm_, bn_, rv_: lambda: (
                                k.gemm_ring(A, nxt(), C, 0, bm_, bn_, rv_), k.add_rmsnorm2(h0, C, wp, wp, xo, 1e-6)))(bm, bn, rv)
                        for ch in others:
                            if ch.startswith("g"):
                                var[ch] = (lambda c_: lambda: (ops.tb_gemm(A, nxt(), C, None, None, 0, c_),
                                                               k.add_rmsnorm2(h0, C, wp, wp, xo, 1e-6)))(ch)
                            elif ch.startswith("k") and (ch != "k64" or M <= 512):
                                tr = int(ch[1:])
                                ks = int(k.gemm4_splitk_ks(M, N, K, tr))
                                wsp = torch.empty(ks * M * N, device=dev)
                                var[ch] = (lambda tr_, ks_, wsp_: lambda: k.add_rmsnorm2_part(
                                    h0, wsp_, int(k.gemm4_splitk_part(A, nxt(), wsp_, tr_, ks_)), wp, wp, xo, 1e-6))(
                                        tr, ks, wsp)
                        var["blas"] = lambda: (torch.matmul(A, nxt().t(), out=C), k.add_rmsnorm2(h0, C, wp, wp, xo, 1e-6))
                    else:
                        for (bm, bn, rv) in ok_tiles:
                            var[rname(bm, bn, rv)] = (lambda bm_, bn_, rv_: lambda: k.gemm_ring(A, nxt(), C, kepi, bm_, bn_, rv_))(
                                bm, bn, rv)
                        for ch in others:
                            c_ = int(ch) if ch.isdigit() else ch
                            var[ch] = (lambda c_: lambda: ops.tb_gemm(A, nxt(), C, None, None, kepi, c_))(c_)
                        if epi == 3:
                            G = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
                            var["blas"] = lambda: (torch.matmul(A, nxt().t(), out=G), ops.geglu(G, out=C))
                        else:
                            var["blas"] = lambda: torch.matmul(A, nxt().t(), out=C)
                for f in var.values():
                    f()
                torch.cuda.synchronize()
                est = min(timed(f, 2) for f in var.values())
                reps = max(2, min(50, int(3000 / max(est, 1.0))))
                res = {v: [] for v in var}
                for _ in range(args.rounds):
                    for v, f in var.items():
                        res[v].append(timed(f, reps))
                med = {v: sorted(t)[len(t) // 2] for v, t in res.items()}
                best_inv = min((v for v in var if v[0] in "rg" or v.isdigit()), key=lambda v: med[v])
                best_any = min(var, key=lambda v: med[v])
                rec = {"shape": name, "N": N, "K": K, "M": M, "epi": epi,
                       "us": {v: round(t, 2) for v, t in sorted(med.items(), key=lambda x: x[1])},
                       "best_invariant": best_inv, "best": best_any}
                out.write(json.dumps(rec) + "\n")
                out.flush()
                top = list(rec["us"].items())[:6]
                print(f"{name:5s} e{epi} M={M:5d} inv {best_inv}={med[best_inv]:.1f}  best {best_any}={med[best_any]:.1f}  "
                      f"blas {med['blas']:.1f}  {top}", flush=True)
        del Ws
        torch.cuda.empty_cache()
    print(f"RING_BENCH_DONE mismatches={bad}", flush=True)
    if bad:
        sys.exit(1)


if __name__ == "__main__":
    main()
