import json, sys
import torch
sys.path.insert(0, ".")
from taboo_brittleness_amd import ops
from tools.l2a_bench import timed
BF = torch.bfloat16
dev = torch.device("cuda:0")
N, K0, KP = 28672, 3584, 128
w = (torch.randn(N, K0 + KP, device=dev) * 0.02).to(BF)
for M in (512, 768, 1024, 1536, 2048):
    x = torch.randn(M, K0, device=dev).to(BF); t = (torch.randn(M, KP, device=dev) * 0.5).to(BF)
    xc = torch.cat([x, t], 1).contiguous()
    o1 = torch.empty(M, N // 2, dtype=BF, device=dev); o2 = torch.empty_like(o1)
    res = {"M": M, "gs_M1": int(ops._GD.split_rows(M, N))}
    for c in ("g256", "g128", "gs"):
        t1 = timed(lambda: ops.gemm_l2a(x, t, w, o1, 3, c))
        t2 = timed(lambda: ops.tb_gemm(xc, w, o2, None, None, 3, c))
        assert torch.equal(o1, o2)
        res[c] = [round(t1, 1), round(t2, 1), round(t1 / t2, 3)]
    print(json.dumps(res), flush=True)
