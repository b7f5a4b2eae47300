"""Microbenchmark of the vocab-head kernels on [R, 256000] bf16 logits."""
import time

import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from taboo_brittleness_amd import ops
from taboo_brittleness_amd.ops._ext import kernels


def bench(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3


R, V = 2048, 256000
lg = (torch.randn(R, V, device="cuda") * 3).to(torch.bfloat16)
tgt = torch.randint(0, V, (R,), dtype=torch.int32, device="cuda")
nxt = torch.empty(R, dtype=torch.int32, device="cuda")
ns = torch.empty(R, device="cuda")
nt = torch.empty(R, device="cuda")
gb = R * V * 2 / 1e9
for cap in (30.0, 0.0):
    ms = bench(lambda: ops.decode_head(lg, cap, tgt, nxt, ns, nt))
    print(f"decode_head cap={cap} [TB_DECODE_HEAD={os.environ.get('TB_DECODE_HEAD', 'f')}]: {ms:.3f} ms  {gb / ms:.2f} TB/s")
    ms = bench(lambda: ops.argmax_rows(lg, cap, out=nxt))
    print(f"argmax_rows cap={cap}: {ms:.3f} ms  {gb / ms:.2f} TB/s")
    ms = bench(lambda: ops.xent_rows(lg, tgt, cap, True, out=ns))
    print(f"xent_rows cap={cap}: {ms:.3f} ms  {gb / ms:.2f} TB/s")
ms = bench(lambda: lg.float().sum(1))
print(f"torch sum (read+convert) {ms:.3f} ms")
W = (torch.randn(V, 3584, device="cuda") * 0.02).to(torch.bfloat16)
x = torch.randn(R, 3584, device="cuda").to(torch.bfloat16)
ms = bench(lambda: torch.matmul(x, W.t(), out=lg))
print(f"lm_head GEMM [{R}x3584]x[3584x{V}] {ms:.3f} ms  {2 * R * 3584 * V / ms / 1e9:.0f} TFLOP/s")
