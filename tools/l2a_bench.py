"""Two-source (LoRA K-augmented) GEMMs vs the single-source GEMM of the materialised concatenation, same kernel
choice (ops._l2a_choice), Gemma-2-9B projection shapes + KP = 128: GPU time per call from a hipGraph of 10 calls,
median of 5 replays, outputs compared bit for bit.  The ratio is the price of reading [x | T] from two sources."""
import json
import sys

import torch

sys.path.insert(0, ".")
from taboo_brittleness_amd import ops  # noqa: E402

BF = torch.bfloat16
SHAPES = {"gu": (28672, 3584, 3), "o": (3584, 4096, 0), "down": (3584, 14336, 0)}   # name -> (N, K0, epi)


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1000 / reps)
    return sorted(ts)[2]


def main():
    dev = torch.device("cuda:0")
    KP = 128
    for name, (N, K0, epi) in SHAPES.items():
        w = (torch.randn(N, K0 + KP, device=dev) * 0.02).to(BF)
        for M in (256, 1024, 2048, 8192):
            x = torch.randn(M, K0, device=dev).to(BF)
            t = (torch.randn(M, KP, device=dev) * 0.5).to(BF)
            xc = torch.cat([x, t], 1).contiguous()
            c = ops._l2a_choice(M, N, K0 + KP, epi)
            nout = N // 2 if epi == 3 else N
            o1 = torch.empty(M, nout, dtype=BF, device=dev)
            o2 = torch.empty(M, nout, dtype=BF, device=dev)
            cs = c if isinstance(c, str) else f"r{c[1]}x{c[2]}b"
            t1 = timed(lambda: ops.gemm_l2a(x, t, w, o1, epi, c))
            t2 = timed(lambda: ops.tb_gemm(xc, w, o2, None, None, epi, cs))
            assert torch.equal(o1, o2), (name, M, c)
            print(json.dumps({"proj": name, "M": M, "choice": cs, "l2a_us": round(t1, 2), "single_us": round(t2, 2),
                              "ratio": round(t1 / t2, 4)}), flush=True)


if __name__ == "__main__":
    main()
