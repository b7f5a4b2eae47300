"""A stronger HF-transformers baseline for the sweep-cell workload: the same per-cell work as
tools/hf_eager_baseline.py (50-token greedy generation with the error-preserving SAE-latent ablation at 4
spike positions of block 31, layer-31 logit-lens top-5 over the response, teacher-forced NLL of the hint
under the edit) but with the 66 cells of one (word, prompt) pair batched into one ``generate`` call,
one lens forward and one NLL forward (each cell ablates its own latent set; the prompt is shared, so
no padding).  This is what a careful user of stock PyTorch/HF would write; BASELINE.md's headline
baseline stays the reference-style batch-1 loop.  Prints one JSON line with cells/s.

    python tools/hf_batched_baseline.py [--cells 66] [--reps 2] [--attn eager|sdpa]
"""
from __future__ import annotations

import argparse
import json
import time

import torch


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--cells", type=int, default=66)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--max-new", type=int, default=50)
    ap.add_argument("--attn", default="eager")
    args = ap.parse_args()
    from transformers import Gemma2Config, Gemma2ForCausalLM

    dev = torch.device("cuda:0")
    cfg = Gemma2Config(vocab_size=256000, hidden_size=3584, intermediate_size=14336, num_hidden_layers=42,
                       num_attention_heads=16, num_key_value_heads=8, head_dim=256, query_pre_attn_scalar=256,
                       sliding_window=4096, attn_implementation=args.attn)
    torch.set_default_dtype(torch.bfloat16)
    with torch.device(dev):
        model = Gemma2ForCausalLM(cfg)
    torch.set_default_dtype(torch.float32)
    model.eval()
    D, L, B = 3584, 16384, args.cells
    g = torch.Generator(device=dev).manual_seed(0)
    W_dec = torch.randn(L, D, device=dev, generator=g)
    W_dec = W_dec / W_dec.norm(dim=1, keepdim=True)
    W_enc = W_dec.t().contiguous()
    b_enc = torch.zeros(L, device=dev)
    thr = torch.full((L,), 0.5, device=dev)
    # per-cell latent sets: budgets {1,2,4,8,16,32} x 11 sets, padded to 32 with a zero mask
    budgets = [1, 2, 4, 8, 16, 32]
    lat = torch.randint(0, L, (B, 32), device=dev, generator=g)
    mask = torch.zeros(B, 32, device=dev)
    for i in range(B):
        mask[i, : budgets[i % len(budgets)]] = 1.0
    We = W_enc.t()[lat]          # [B, 32, D]
    Wd = W_dec[lat]              # [B, 32, D]
    be, th = b_enc[lat], thr[lat]
    state = {"pos": 0, "spikes": set()}

    def hook(mod, inp, out):
        h = out[0] if isinstance(out, tuple) else out
        T = h.shape[1]
        p0 = state["pos"]
        rows = [t for t in range(T) if p0 + t in state["spikes"]]
        if rows:
            x = h[:, rows].float()                                  # [B, r, D]
            pre = torch.einsum("brd,bkd->brk", x, We) + be[:, None]
            a = torch.where(pre > th[:, None], pre, torch.zeros_like(pre)) * mask[:, None]
            h[:, rows] = (x - torch.einsum("brk,bkd->brd", a, Wd)).to(h.dtype)
        state["pos"] += T
        return out

    handle = model.model.layers[31].register_forward_hook(hook)
    P = 18
    prompt = torch.randint(1000, 200000, (1, P), device=dev).expand(B, P).contiguous()
    spikes = {P + 5, P + 11, P + 20, P + 33}
    times = []
    with torch.no_grad():
        for i in range(args.warmup + args.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            state["pos"], state["spikes"] = 0, spikes
            out = model.generate(input_ids=prompt, max_new_tokens=args.max_new, do_sample=False,
                                 min_new_tokens=args.max_new, pad_token_id=0)
            state["pos"] = 0
            o = model(out, output_hidden_states=True)
            h31 = o.hidden_states[32][:, P:]
            top = []
            for b in range(B):      # [T, 256000] softmax per cell (a [B, T, V] tensor would be 52 GB)
                probs = torch.softmax(model.lm_head(model.model.norm(h31[b])), dim=-1)
                top.append(torch.topk(probs.float().sum(0), 5).indices)
            top = torch.stack(top).tolist()
            state["pos"] = 0
            lo = model(out, labels=out).loss.item()
            torch.cuda.synchronize()
            if i >= args.warmup:
                times.append(time.perf_counter() - t0)
    handle.remove()
    per = sum(times) / len(times)
    print(json.dumps({"metric": "hf_batched_cells_per_sec", "value": B / per, "sec_per_batch": per, "cells": B,
                      "attn": args.attn, "reps": args.reps, "nll": lo, "top0": top[0]}))


if __name__ == "__main__":
    main()
