"""HF-transformers eager baseline for the sweep-cell workload on MI355X ("The baseline is
an HF-transformers eager PyTorch-ROCm run on MI355X, using the same random-init Gemma-2-9B weights
and synthetic prompts").

It runs one sweep cell the way the reference's code base runs its per-prompt work
(`src/models.py:55-94,97-170`): batch-1 ``model.generate(do_sample=False, max_new_tokens=50)`` with a
forward hook on decoder layer 31 that performs the error-preserving SAE-latent ablation at the
cell's spike positions, then a traced forward of prompt+hint for the layer-31 logit lens
(softmax(lm_head(norm(h31))) summed over the response, top-5 on the GPU — already cheaper than the
reference's 42-layer host dump), then the teacher-forced NLL pass of the baseline hint with the hook.
Prints one JSON line with cells/s.
"""
from __future__ import annotations

import json
import time

import torch


def main(n_cells: int = 6, warmup: int = 1, max_new: int = 50, m: int = 8):
    from transformers import Gemma2Config, Gemma2ForCausalLM

    dev = torch.device("cuda:0")
    cfg = Gemma2Config(vocab_size=256000, hidden_size=3584, intermediate_size=14336, num_hidden_layers=42,
                       num_attention_heads=16, num_key_value_heads=8, head_dim=256, query_pre_attn_scalar=256,
                       sliding_window=4096, attn_implementation="eager")
    torch.set_default_dtype(torch.bfloat16)
    with torch.device(dev):
        model = Gemma2ForCausalLM(cfg)
    torch.set_default_dtype(torch.float32)
    model.eval()
    D, L = 3584, 16384
    g = torch.Generator(device=dev).manual_seed(0)
    W_dec = torch.randn(L, D, device=dev, generator=g)
    W_dec = W_dec / W_dec.norm(dim=1, keepdim=True)
    W_enc = W_dec.t().contiguous()
    b_enc = torch.zeros(L, device=dev)
    thr = torch.full((L,), 0.5, device=dev)
    latents = torch.arange(m, device=dev)
    state = {"pos": 0, "spikes": set()}

    def hook(mod, inp, out):
        h = out[0] if isinstance(out, tuple) else out
        T = h.shape[1]
        p0 = state["pos"]
        rows = [t for t in range(T) if p0 + t in state["spikes"]]
        if rows:
            x = h[0, rows].float()
            pre = x @ W_enc[:, latents] + b_enc[latents]
            a = torch.where(pre > thr[latents], pre, torch.zeros_like(pre))
            h[0, rows] = (x - a @ W_dec[latents]).to(h.dtype)
        state["pos"] += T
        return out

    handle = model.model.layers[31].register_forward_hook(hook)
    prompt = torch.randint(1000, 200000, (1, 18), device=dev)
    times = []
    with torch.no_grad():
        for i in range(warmup + n_cells):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            state["pos"], state["spikes"] = 0, {18 + 5, 18 + 11, 18 + 20, 18 + 33}
            out = model.generate(input_ids=prompt, max_new_tokens=max_new, do_sample=False, min_new_tokens=max_new)
            # lens readout at layer 31 over the full text
            state["pos"] = 0
            o = model(out, output_hidden_states=True)
            h31 = o.hidden_states[32][0, 18:]
            probs = torch.softmax(model.lm_head(model.model.norm(h31)), dim=-1)
            top = torch.topk(probs.float().sum(0), 5).indices.tolist()
            # teacher-forced NLL of the (baseline) hint under the edit
            state["pos"] = 0
            lo = model(out, labels=out).loss.item()
            torch.cuda.synchronize()
            if i >= warmup:
                times.append(time.perf_counter() - t0)
    handle.remove()
    per = sum(times) / len(times)
    print(json.dumps({"metric": "hf_eager_cells_per_sec", "value": 1.0 / per, "sec_per_cell": per,
                      "n_cells": n_cells, "top": top, "nll": lo}))


if __name__ == "__main__":
    main()
