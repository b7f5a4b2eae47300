"""Measure the in-tree GEMMs (ping-pong ``256`` / ``128`` and four-wave ``g256`` / ``g128`` row tiles) against hipBLASLt (with the bench's TunableOp
table) on every projection shape of the Gemma-2-9B step and write the per-shape dispatch table
``configs/gemm_dispatch/gemma2-9b.json`` that ``runtime/gemm_dispatch.py`` loads (``TB_GEMM=auto``).

Shapes: the five projections (QKV, o, gate|up, down, lm_head / lens) at every row count M the bench's
TunableOp table holds (its decode row buckets) plus a standard grid; gate|up also as the fused GeGLU
epilogue vs hipBLASLt + the GeGLU kernel (key epi 3), QKV also as the fused QKV + RoPE + KV-cache scatter
(csrc/gemm4.hip G4_ROPE) vs hipBLASLt + rope_qkv_cache (key epi 4).  Operands are uniform random bf16 (never zeros: DVFS), the weight
is rotated over copies larger than the Infinity Cache (decode streams every weight from HBM), variants are
interleaved in rounds inside one process (cdna_hip_programming.md §5.4 rule 24), median of the rounds.

  python tools/gemm_dispatch_tune.py [--tag gemma2-9b_P100_E4_new50] [--out configs/gemm_dispatch/gemma2-9b.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from taboo_brittleness_amd import ops  # noqa: E402
from taboo_brittleness_amd.ops import _ext  # noqa: E402
from taboo_brittleness_amd.ops import reference as ref  # noqa: E402
from taboo_brittleness_amd.runtime.tuning import enable_tuned_gemms, gemm_results_path  # noqa: E402

SHAPES = {"qkv": (8192, 3584), "o": (3584, 4096), "gu": (28672, 3584), "down": (3584, 14336), "head": (256000, 3584)}
GRID = [64, 128, 256, 512, 768, 1024, 1536, 2048, 3072, 4096, 6144, 8192]


def table_ms(tag: str):
    """Row counts per (N, K) in a TunableOp results CSV (``tn_N_M_K`` keys)."""
    out = {}
    p = gemm_results_path(tag)
    if not os.path.exists(p):
        return out
    for line in open(p):
        if not line.startswith("Gemm"):
            continue
        f = line.split(",")[1].split("_")
        n, m, k = int(f[1]), int(f[2]), int(f[3])
        out.setdefault((n, k), set()).add(m)
    return out


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
    ap.add_argument("--tag", default="gemma2-9b_P100_E4_new50")
    ap.add_argument("--out", default=os.path.join(ROOT, "configs", "gemm_dispatch", "gemma2-9b.json"))
    ap.add_argument("--raw", default=os.path.join(ROOT, "gpurun_out", "gemm_dispatch_raw.jsonl"))
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--max-m", type=int, default=33000)
    ap.add_argument("--only", default="", help="comma-separated shape names")
    ap.add_argument("--tie", type=float, default=1.01, help="in-tree wins when t_tb <= tie * t_blas")
    ap.add_argument("--kernels", default="g256,g128,k256,k128,k64,256,128",
                    help="in-tree candidates (gNNN: gemm4.hip, kNNN: gemm4.hip split over K, NNN: gemm.hip)")
    args = ap.parse_args()
    _ext.load()
    k = _ext.kernels()
    dev = torch.device("cuda:0")
    enable_tuned_gemms(args.tag)
    tms = table_ms(args.tag)
    os.makedirs(os.path.dirname(args.raw), exist_ok=True)
    raw = open(args.raw, "w")
    table = {"shapes": {}, "meta": {"tag": args.tag, "tie": args.tie, "device": torch.cuda.get_device_name(0),
                                    "time": time.strftime("%Y-%m-%d %H:%M:%S")}}
    names = [n for n in SHAPES if not args.only or n in args.only.split(",")]
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    for name in names:
        N, K = SHAPES[name]
        Ms = sorted(set(GRID) | tms.get((N, K), set()))
        Ms = [m for m in Ms if m <= args.max_m]
        wbytes = N * K * 2
        ncopy = max(1, min(8, -(-600 * 2 ** 20 // wbytes)))
        Ws = [(torch.rand(N, K, device=dev, generator=g) * 2 - 1).to(torch.bfloat16) for _ in range(ncopy)]
        Wi = None
        if name == "gu":
            idx = ops.geglu_interleave_index(N // 2, dev)
            Wi = [w.index_select(0, idx).contiguous() for w in Ws]
        for epi in ([0, 3] if name == "gu" else [0, 4] if name == "qkv" else [0, 5] if name in ("o", "down") else [0]):
            rows = []
            for M in Ms:
                A = (torch.rand(M, K, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
                ncol = N // 2 if epi == 3 else N
                C = torch.empty(M, ncol, device=dev, dtype=torch.bfloat16)
                G = torch.empty(M, N, device=dev, dtype=torch.bfloat16) if epi == 3 else None
                it = [0]

                def nxt(ws):
                    it[0] = (it[0] + 1) % len(ws)
                    return ws[it[0]]

                if epi == 4:
                    # QKV at the Gemma-2-9B head layout into a layer's KV cache (positions < S, slots < M)
                    Hq, Hkv, HD, S = 16, 8, 256, 512
                    nslot = min(M, 256)
                    pos = torch.randint(0, S, (M,), device=dev, dtype=torch.int32)
                    slot = (torch.arange(M, device=dev, dtype=torch.int32) % nslot).contiguous()
                    cos_t, sin_t = ref.rope_tables(HD, 8192, 10000.0, dev)
                    cos_t, sin_t = cos_t.contiguous(), sin_t.contiguous()
                    kc = torch.zeros(nslot, Hkv, S, HD, device=dev, dtype=torch.bfloat16)
                    vc = torch.zeros_like(kc)
                    q = torch.empty(M, Hq, HD, device=dev, dtype=torch.bfloat16)

                    def blas_rope():
                        torch.matmul(A, nxt(Ws).t(), out=C)
                        ops.rope_qkv_cache(C, pos, slot, cos_t, sin_t, kc, vc, Hq, Hkv, HD, q_out=q)
                    var = {"blas": blas_rope}
                    for ch in [c_ for c_ in args.kernels.split(",") if c_.startswith("g")]:
                        var[ch] = (lambda r_: lambda: k.gemm4_qkv_rope(A, nxt(Ws), pos, slot, ops.rope_cs(cos_t, sin_t),
                                                                       q, kc, vc,
                                                                       Hq, Hkv, r_))(int(ch[1:]))
                    for ch in [c_ for c_ in args.kernels.split(",") if c_.startswith("k") and (c_ != "k64" or M <= 512)]:
                        tr = int(ch[1:])
                        ks = int(k.gemm4_splitk_ks(M, N, K, tr))
                        wsq = torch.empty(ks * M * N, device=dev)

                        def split_rope(tr=tr, ks=ks, wsq=wsq):
                            used = int(k.gemm4_splitk_part(A, nxt(Ws), wsq, tr, ks))
                            k.rope_qkv_cache_part(wsq, used, pos, slot, cos_t, sin_t, q, kc, vc, Hq, Hkv, HD)
                        var[ch] = split_rope
                elif epi == 5:
                    # o_proj / down + the block's add_rmsnorm2 (ops.linear_add_rmsnorm2): split-K partials are summed
                    # inside the norm pass, every other variant stores bf16 o first
                    D = N
                    h0 = (torch.rand(M, D, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
                    wp = (torch.rand(D, device=dev, generator=g) * 0.2 - 0.1).to(torch.bfloat16)
                    xo = torch.empty(M, D, device=dev, dtype=torch.bfloat16)
                    wsp = {}

                    def norm_var(ch_):
                        if ch_ == "blas":
                            return lambda: (torch.matmul(A, nxt(Ws).t(), out=C), k.add_rmsnorm2(h0, C, wp, wp, xo, 1e-6))
                        if ch_[0] == "k":
                            tr = int(ch_[1:])
                            ks = int(k.gemm4_splitk_ks(M, N, K, tr))
                            wsp[ch_] = torch.empty(ks * M * N, device=dev)
                            return lambda: k.add_rmsnorm2_part(h0, wsp[ch_], int(k.gemm4_splitk_part(A, nxt(Ws), wsp[ch_], tr, ks)),
                                                               wp, wp, xo, 1e-6)
                        if ch_ == "s":
                            return lambda: (k.gemm_skinny(A, nxt(Ws), C), k.add_rmsnorm2(h0, C, wp, wp, xo, 1e-6))
                        c_ = ch_ if ch_[0] == "g" else int(ch_)
                        return lambda: (ops.tb_gemm(A, nxt(Ws), C, None, None, 0, c_), k.add_rmsnorm2(h0, C, wp, wp, xo, 1e-6))
                    var = {"blas": norm_var("blas")}
                    for ch in args.kernels.split(","):
                        if (ch == "s" and not k.gemm_skinny_ok(M, N, K)) or (ch == "k64" and M > 512):
                            continue
                        var[ch] = norm_var(ch)
                elif epi == 0:
                    var = {"blas": lambda: torch.matmul(A, nxt(Ws).t(), out=C)}
                else:
                    def blas_geglu():
                        torch.matmul(A, nxt(Ws).t(), out=G)
                        ops.geglu(G, out=C)
                    var = {"blas": blas_geglu}
                wsrc = Wi if epi == 3 else Ws
                for ch in (args.kernels.split(",") if epi not in (4, 5) else []):
                    if ch == "k64" and M > 512:
                        continue
                    if ch == "s":          # csrc/skinny.hip (M <= 64, plain bf16 only)
                        if epi == 0 and k.gemm_skinny_ok(M, N, K):
                            var["s"] = lambda: k.gemm_skinny(A, nxt(Ws), C)
                        continue
                    ch = ch if ch[0] in "gk" else int(ch)
                    var[ch] = (lambda ch_: lambda: ops.tb_gemm(A, nxt(wsrc), C, None, None, epi, ch_))(ch)
                for f in var.values():      # warm-up (and TunableOp lookups)
                    f()
                torch.cuda.synchronize()
                est = min(timed(f, 2) for f in var.values())
                reps = max(2, min(50, int(3000 / max(est, 1.0))))
                res = {v: [] for v in var}
                for _ in range(args.rounds):
                    for v, f in var.items():
                        res[v].append(timed(f, reps))
                med = {v: sorted(t)[len(t) // 2] for v, t in res.items()}
                tb_best = min((v for v in var if v != "blas"), key=lambda v: med[v])
                win = tb_best if med[tb_best] <= args.tie * med["blas"] else "blas"
                rows.append([M, win])
                rec = {"shape": name, "N": N, "K": K, "M": M, "epi": epi, "us": {str(v): round(t, 2) for v, t in med.items()},
                       "TF": {str(v): round(2.0 * M * N * K / t / 1e6, 1) for v, t in med.items()}, "win": win}
                raw.write(json.dumps(rec) + "\n")
                raw.flush()
                print(json.dumps(rec), flush=True)
                del A, C, G
            table["shapes"][f"{N},{K},{epi}"] = rows
        del Ws, Wi
        torch.cuda.empty_cache()
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    json.dump(table, open(args.out, "w"), indent=1)
    print(f"wrote {args.out}")


if __name__ == "__main__":
    main()
