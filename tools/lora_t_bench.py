"""LoRA T = x A_all^T (ops.lora_t) launch forms at the Gemma-2-9B projection shapes: unsplit (one workgroup per tile,
the K chunks folded in registers) vs split (one workgroup per (tile, chunk) + the ordered fold kernel), per row count
and row tile.  GPU time per call from a hipGraph of 20 calls (no host launch cost), median of 5 replays.  Prints one
JSON line per point; ops.lora_t_plan encodes the picks."""
import json
import sys

import torch

sys.path.insert(0, ".")
from taboo_brittleness_amd import ops  # noqa: E402

BF = torch.bfloat16
# projection -> (K, nsr) for 3 words x rank 8 (q|k|v: 3 sub-modules, gate|up: 2)
SHAPES = {"qkv": (3584, 72), "o": (4096, 24), "gu": (3584, 48), "down": (14336, 24)}
ROWS = [16, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 32768]


def timed(fn, reps=20):
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
    for name, (K, nsr) in SHAPES.items():
        a = torch.zeros(128, K, dtype=BF, device=dev)
        a[:nsr] = (torch.randn(nsr, K, device=dev) * 0.05).to(BF)
        for M in ROWS:
            x = torch.randn(M, K, device=dev).to(BF)
            ad = (torch.arange(M, device=dev, dtype=torch.int32) % 3)
            out = torch.zeros(M, 128, dtype=BF, device=dev)
            res = {"proj": name, "M": M, "K": K}
            ref = None
            nt = -(-nsr // 32) * 32
            for bn in sorted({32, nt}):
                for bm in (16, 32, 64, 128):
                    if bm == 128 and bn == 96:
                        continue
                    for split in (False, True):
                        f = lambda: ops.lora_t(x, a, ad, nsr, 24, 8, out=out, split=split, bm=bm, bn=bn)  # noqa: E731
                        res[f"{'split' if split else 'fold'}{bm}x{bn}"] = round(timed(f), 2)
                        if ref is None:
                            ref = out.clone()
                        else:
                            assert torch.equal(out, ref), (name, M, bm, bn, split)
            res["auto"] = round(timed(lambda: ops.lora_t(x, a, ad, nsr, 24, 8, out=out)), 2)
            bm = 16 if M <= 512 else (32 if M <= 2048 else 64)
            res["unsplit_wgs"] = -(-M // bm) * (nt // 32)
            print(json.dumps(res), flush=True)
            del x, out


if __name__ == "__main__":
    main()
