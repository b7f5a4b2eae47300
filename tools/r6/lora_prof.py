"""Per-kernel cost of the fused multi-adapter LoRA path: decode-shaped forwards (T = 1, 42 layers) of M rows with and
without the bank, for rocprofv3 --kernel-trace --stats (run under the profiler; kernel names carry the L2A flag)."""
import sys
import time

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__)))))
from taboo_brittleness_amd.models.gemma2 import Gemma2Model  # noqa: E402
from taboo_brittleness_amd.models.lora import LoRABank  # noqa: E402
from taboo_brittleness_amd.models.spec import GEMMA2_9B  # noqa: E402
from taboo_brittleness_amd.models.weights import random_gemma2  # noqa: E402

dev = torch.device("cuda:0")
spec = GEMMA2_9B
m = Gemma2Model(random_gemma2(spec, device=dev, dtype=torch.bfloat16, seed=1234, post_norm_gain=32.0), dev)
bank = LoRABank.random(spec, ["moon", "smile", "ship"], r=8, alpha=16.0, seed=99, device=dev)
M = int(sys.argv[1]) if len(sys.argv) > 1 else 64
mode = sys.argv[2] if len(sys.argv) > 2 else "lora"
ids = torch.randint(3, spec.vocab_size, (M, 1), device=dev, dtype=torch.int32)
pos = torch.full((M, 1), 40, dtype=torch.int32, device=dev)
cache = m.new_cache(M, 41)
cache.adapter.copy_(torch.arange(M, dtype=torch.int32, device=dev) % 3)
slot = torch.arange(M, dtype=torch.int32, device=dev)
if mode == "lora":
    m.set_lora(bank)
for _ in range(6):
    m.forward(ids, pos, cache, slot)
torch.cuda.synchronize()
print("done", M, mode, time.time())
