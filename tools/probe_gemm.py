"""Calibration probe: hipBLASLt (torch.matmul) bf16 GEMM times at Gemma-2-9B shapes on MI355X."""
import json, time, torch

def bench(fn, iters=20, warm=5):
    for _ in range(warm): fn()
    torch.cuda.synchronize()
    s = torch.cuda.Event(enable_timing=True); e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters): fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / iters

def main():
    p = torch.cuda.get_device_properties(0)
    print(p.name, p.gcnArchName, p.multi_processor_count, p.total_memory / 2**30, flush=True)
    D, F, V = 3584, 14336, 256000
    shapes = {"qkv": (D, 8192), "o": (4096, D), "gateup": (D, 2 * F), "down": (F, D), "lm_head": (D, V)}
    out = []
    for M in [64, 128, 256, 512, 2048, 8192, 16384]:
        for name, (K, N) in shapes.items():
            if name == "lm_head" and M > 8192: continue
            a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
            ms = bench(lambda: torch.nn.functional.linear(a, w))
            tf = 2 * M * N * K / ms / 1e9
            gbs = (N * K * 2 + M * K * 2 + M * N * 2) / ms / 1e6
            out.append(dict(M=M, name=name, K=K, N=N, ms=ms, tflops=tf, gbs=gbs))
            print(f"M={M:6d} {name:8s} K={K:6d} N={N:6d} {ms:8.3f} ms {tf:8.1f} TF/s {gbs:8.1f} GB/s", flush=True)
            del a, w
    # HBM copy bandwidth
    x = torch.empty(2 * 2**30 // 2, device="cuda", dtype=torch.bfloat16); y = torch.empty_like(x)
    ms = bench(lambda: y.copy_(x))
    print(f"copy 2GiB: {ms:.3f} ms -> {2*2*2**30/ms/1e6:.1f} GB/s")
    json.dump(out, open("gpurun_out/probe_gemm.json", "w"), indent=1)

if __name__ == "__main__":
    main()
