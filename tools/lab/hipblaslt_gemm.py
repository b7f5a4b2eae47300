"""hipBLASLt reference GEMM at one shape (for PMC passes next to tools/lab/gemm_lab.hip)."""
import sys

import torch

M, N, K, reps = (int(a) for a in sys.argv[1:5])
A = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
W = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
for _ in range(reps):
    torch.matmul(A, W.T, out=C)
torch.cuda.synchronize()
