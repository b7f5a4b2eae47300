"""Lab A/B for csrc/gemm4.hip (four-wave GEMM) via a ctypes shim (tools/lab/g4_lab.so, built on the CPU host):

  python tools/lab/g4_bench.py check            exactness vs an fp32 torch reference (bf16 / f32 / GeGLU epilogues)
  python tools/lab/g4_bench.py time [shapes]    interleaved rounds in one process: hipBLASLt (torch.matmul, with the
                                                bench's TunableOp table), the extension's gemm4 (ext256), the lab build 256 / 128
Operands are uniform [-1, 1) bf16 (cdna_hip_programming.md §5.4 rule 25); the weight rotates over copies larger than
the Infinity Cache.
"""
from __future__ import annotations

import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from taboo_brittleness_amd import ops  # noqa: E402
from taboo_brittleness_amd.ops import _ext  # noqa: E402

LIB = ctypes.CDLL(os.path.join(ROOT, "tools", "lab", os.environ.get("G4_LIB", "g4_lab.so")))
LIB.g4_gemm.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int] * 6 + [ctypes.c_void_p]
LIB.g4_gemm.restype = ctypes.c_int


EXTRA = {}
for _f in filter(None, os.environ.get("G4_LIBS", "").split(",")):
    _l = ctypes.CDLL(os.path.join(ROOT, "tools", "lab", _f))
    _l.g4_gemm.argtypes = LIB.g4_gemm.argtypes
    _l.g4_gemm.restype = ctypes.c_int
    EXTRA[_f.replace("g4_lab_", "").replace(".so", "")] = _l


def g4(A, W, C, epi=0, rows=256, lib=None):
    M, K = A.shape
    N = W.shape[0]
    r = (lib or LIB).g4_gemm(A.data_ptr(), W.data_ptr(), C.data_ptr(), M, N, K, C.shape[1], epi, rows,
                    torch.cuda.current_stream().cuda_stream)
    assert r == 0, r


def rnd(*shape, g):
    return (torch.rand(*shape, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)


def check() -> int:
    g = torch.Generator(device="cuda")
    g.manual_seed(1)
    bad = 0
    for M, N, K in [(1, 256, 64), (37, 512, 128), (300, 768, 256), (513, 1024, 3584), (256, 256, 640),
                    (700, 3584, 4096), (2048, 8192, 3584), (129, 28672, 3584)]:
        A, W = rnd(M, K, g=g), rnd(N, K, g=g)
        ref = A.float() @ W.float().t()
        for rows in (256, 128):
            Cf = torch.full((M, N), float("nan"), device="cuda")
            Cb = torch.full((M, N), float("nan"), device="cuda", dtype=torch.bfloat16)
            g4(A, W, Cf, 1, rows)
            g4(A, W, Cb, 0, rows)
            den = ref.abs().max().item()
            ef = (Cf - ref).abs().max().item() / den
            eb = (Cb.float() - ref).abs().max().item() / den
            rec = {"M": M, "N": N, "K": K, "rows": rows, "f32_rel": ef, "bf16_rel": eb}
            ok = ef < 1e-5 and eb < 8e-3
            if N % 512 == 0 and N <= 28672:
                idx = ops.geglu_interleave_index(N // 2, A.device)
                Wi = W.index_select(0, idx).contiguous()
                Cg = torch.full((M, N // 2), float("nan"), device="cuda", dtype=torch.bfloat16)
                g4(A, Wi, Cg, 3, rows)
                gu = ref.to(torch.bfloat16)
                refg = ops.geglu(gu)
                eg = (Cg.float() - refg.float()).abs().max().item() / max(refg.float().abs().max().item(), 1e-6)
                rec["geglu_rel"] = eg
                ok = ok and eg < 2e-2
            if rows == 256:
                Cp = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
                _ext.kernels().gemm4(A, W, Cp, None, None, 0, 256)
                rec["bitequal_ext"] = bool(torch.equal(Cp, Cb))
            rec["ok"] = ok
            bad += not ok
            print(json.dumps(rec), flush=True)
    print(json.dumps({"check_ok": bad == 0}), flush=True)
    return 1 if bad else 0


def timed(fn, reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1000.0 / reps


DEFAULT_SHAPES = ["4096,28672,3584", "2048,8192,3584", "4096,8192,3584", "8192,8192,3584", "2048,3584,4096",
                  "4096,3584,4096", "4096,3584,14336", "8192,3584,14336", "2048,256000,3584", "1024,28672,3584",
                  "512,28672,3584"]


def time_shapes(shapes, rounds=int(os.environ.get("G4_ROUNDS", "7"))):
    from taboo_brittleness_amd.runtime.tuning import enable_tuned_gemms
    enable_tuned_gemms(os.environ.get("G4_TUNE_TAG", "gemma2-9b_P100_E4_new50"))
    k = _ext.kernels()
    g = torch.Generator(device="cuda")
    g.manual_seed(0)
    for s in shapes:
        M, N, K = (int(v) for v in s.split(","))
        ncopy = max(1, min(8, -(-600 * 2 ** 20 // (N * K * 2))))
        Ws = [rnd(N, K, g=g) for _ in range(ncopy)]
        A = rnd(M, K, g=g)
        C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        it = [0]

        def nxt():
            it[0] = (it[0] + 1) % len(Ws)
            return Ws[it[0]]

        epi = int(os.environ.get("G4_EPI", "0"))      # 3: the fused GeGLU epilogue ([M, N/2] output)
        Cg = torch.empty(M, N // 2, device="cuda", dtype=torch.bfloat16) if epi == 3 else C
        var = {"blas": lambda: torch.matmul(A, nxt().t(), out=C),
               "ext256": lambda: k.gemm4(A, nxt(), Cg, None, None, epi, 256),
               "g4_256": lambda: g4(A, nxt(), Cg, epi, 256),
               "g4_128": lambda: g4(A, nxt(), Cg, epi, 128)}
        for name, lib in EXTRA.items():      # G4_LIBS: more builds of the kernel, interleaved in this process
            var[name] = (lambda lib_: lambda: g4(A, nxt(), Cg, epi, 256, lib_))(lib)
        for f in var.values():
            f()
        torch.cuda.synchronize()
        est = min(timed(f, 2) for f in var.values())
        reps = max(2, min(50, int(3000 / max(est, 1.0))))
        res = {v: [] for v in var}
        for _ in range(rounds):
            for v, f in var.items():
                res[v].append(timed(f, reps))
        med = {v: sorted(t)[len(t) // 2] for v, t in res.items()}
        print(json.dumps({"M": M, "N": N, "K": K, "us": {v: round(t, 1) for v, t in med.items()},
                          "TF": {v: round(2.0 * M * N * K / t / 1e6) for v, t in med.items()}}), flush=True)
        del Ws, A, C
        torch.cuda.empty_cache()


if __name__ == "__main__":
    _ext.load()
    cmd = sys.argv[1] if len(sys.argv) > 1 else "check"
    if cmd == "check":
        sys.exit(check())
    time_shapes(sys.argv[2:] or DEFAULT_SHAPES)
