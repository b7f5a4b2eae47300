"""Reference pipelines: generation cache, Logit-Lens Top-k and SAE Top-k baselines
(C9, C11-C15, C17-C19, C23).

* :func:`generate_cache` — ``src/run_generation.py``: per word, greedy hints for
  every prompt (batched), then one traced forward over prompt+hint with every
  layer hooked: per-layer lens probabilities of the tracked ids (secret,
  decoys), per-layer argmax, the hooked layer's residual stream, the
  LL response sum at the hooked layer, and — only with ``full_probs`` — the
  reference's ``all_probs [L, T, V]`` array.  Pairs already on disk are
  skipped (the reference's resume point, `src/run_generation.py:96-98`).
* :func:`reproduce_logit_lens` — ``src/01_reproduce_logit_lens.py``:
  cache-first LL-Top-k guesses, metrics JSON in the reference layout
  (per-word ``predictions``, empty guess lists skipped) and heatmaps.
* :func:`run_sae_baseline` — ``src/02_run_sae_baseline.py``: SAE Top-k from the
  cached residuals, latent→word map, metrics with a top-level ``predictions``
  dict (empty lists kept), CSV table.
"""
from __future__ import annotations

import os
import time
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from .. import ops
from ..config import Config
from ..interp.edits import CaptureHook
from ..interp.feature_map import FEATURE_MAP, latents_to_word_guesses
from ..interp.logit_lens import (aggregate_cached_probs, reference_exclusions, topk_guesses, vocab_argmax,
                                 vocab_gather_cols, vocab_reduce_, vocab_slice)
from ..interp.prompts import find_model_response_start, hint_prompt_ids, truncate_at_second_end_of_turn
from ..interp.sae import top_latents
from ..metrics import calculate_metrics
from ..models.tokenizer import secret_token_id
from ..runtime.generation import Generator
from ..utils.io import atomic_write_json, atomic_write_text, load_pair, pair_cached, pair_paths, save_pair
from .factory import build_stack


def _track_ids(cfg: Config, tok, word: str) -> List[int]:
    ids = [secret_token_id(tok, word, "space"), secret_token_id(tok, word, "bare")]
    ids += [secret_token_id(tok, d, "space") for d in cfg.intervention.decoys.get(word, [])]
    return ids


@torch.no_grad()
def trace_sequences(model, tok, seqs: Sequence[Sequence[int]], layer: int, track: Sequence[Sequence[int]],
                    starts: Sequence[int], full_probs: bool = False, round_bf16: bool = True,
                    compat_double_bos: bool = False, exclusion: str = "reference",
                    chunk_rows: int = 4096) -> List[Dict]:
    """All-layer logit lens over full sequences (reference `src/models.py:97-170`), batched.

    One forward over every sequence with every block's residual captured into one ``[L, n, T+1, D]`` store,
    then the lens runs over ALL (layer, sequence, position) rows in chunks of ``chunk_rows``: each chunk is
    one unembedding GEMM (``lens_logits_lse``: final norm, ``[rows, D] x [D, V]``, row log-sum-exp) followed
    by the tracked-id probabilities and the per-row argmax, written into device buffers; the hooked layer's
    response rows get one more pass for the masked response column sum (``lens_colsum``, packed offsets).
    Nothing returns to the host until the end (one copy per product), and the ``[L, T, V]`` probabilities are
    only materialised with ``full_probs`` (the reference's 1.6 GB per pair)."""
    dev = model.device
    L = model.spec.layers
    if compat_double_bos:   # reference re-tokenises decoded text that already holds <bos>
        bos = getattr(tok, "bos_token_id", None)
        seqs = [[bos] + list(s) for s in seqs] if bos is not None else list(seqs)
        starts = [s + 1 for s in starts] if bos is not None else list(starts)
    n = len(seqs)
    T = max(len(s) for s in seqs)
    D = model.spec.hidden
    V = model.spec.vocab_size
    lo, Vl = vocab_slice(model)          # this rank's lens columns (vocab-parallel TP) or the whole vocab
    big = torch.zeros(L, n, T + 1, D, dtype=model.dtype, device=dev)
    hooks = {l: [CaptureHook(big[l])] for l in range(L)}
    ids = torch.zeros(n, T, dtype=torch.int32)
    pos = torch.full((n, T), -1, dtype=torch.int32)
    for b, s in enumerate(seqs):
        ids[b, : len(s)] = torch.tensor(list(s), dtype=torch.int32)
        pos[b, : len(s)] = torch.arange(len(s), dtype=torch.int32)
    cache = model.new_cache(n, T)
    model.forward(ids.to(dev), pos.to(dev), cache, torch.arange(n, dtype=torch.int32, device=dev), hooks)
    lens_ = [len(s) for s in seqs]
    # packed (layer, sequence, position) rows of the store, layer-major
    seq_rows = np.concatenate([b * (T + 1) + np.arange(Tb) for b, Tb in enumerate(lens_)]).astype(np.int64)
    per_layer = seq_rows.size
    flat_idx = (np.arange(L, dtype=np.int64)[:, None] * (n * (T + 1)) + seq_rows[None, :]).reshape(-1)
    Kmax = max(len(t) for t in track)
    tid_seq = np.zeros((n, Kmax), np.int32)
    for b, t in enumerate(track):
        tid_seq[b, : len(t)] = list(t)
        tid_seq[b, len(t):] = t[0]                   # padding columns repeat the first id (sliced off below)
    row_seq = np.concatenate([np.full(Tb, b, np.int64) for b, Tb in enumerate(lens_)])
    tid_rows = torch.from_numpy(np.tile(tid_seq[row_seq] - lo, (L, 1))).to(dev)
    big_flat = big.view(-1, D)
    idx_dev = torch.from_numpy(flat_idx).to(dev)
    R = flat_idx.size
    p_all = torch.empty(R, Kmax, dtype=torch.float32, device=dev)
    am_all = torch.empty(R, dtype=torch.int32, device=dev)
    full = [np.zeros((L, Tb, V), dtype=np.float32) for Tb in lens_] if full_probs else None
    offs_seq = np.concatenate([[0], np.cumsum(lens_)])
    for c0 in range(0, R, chunk_rows):
        c1 = min(R, c0 + chunk_rows)
        rows = big_flat.index_select(0, idx_dev[c0:c1])
        logits, lse = model.lens_logits_lse(rows)
        ops.gather_probs(logits, lse, tid_rows[c0:c1], round_bf16=round_bf16, out=p_all[c0:c1])
        vocab_argmax(model, logits, out=am_all[c0:c1])
        if full is not None:
            pr = torch.exp(logits.float() - lse[:, None])
            pr = vocab_gather_cols(model, pr.to(torch.bfloat16).float() if round_bf16 else pr).cpu().numpy()
            for r in range(c0, c1):
                l, j = divmod(r, per_layer)
                b = int(row_seq[j])
                full[b][l, j - offs_seq[b]] = pr[r - c0]
    # masked response column sum at the hooked layer: the response rows of every sequence, packed
    resp_rows, excl, offs = [], [], [0]
    for b, s in enumerate(seqs):
        st = starts[b]
        resp = list(s[st:])
        resp_rows.append(layer * n * (T + 1) + b * (T + 1) + np.arange(st, len(s), dtype=np.int64))
        ex = np.full((len(resp), 2), -1, np.int32)
        if exclusion == "reference" and resp:
            ex[:] = np.asarray(reference_exclusions(tok, resp), np.int32)
            ex[:] = np.where(ex >= 0, ex - lo, ex)
        excl.append(ex)
        offs.append(offs[-1] + len(resp))
    rr = np.concatenate(resp_rows)
    resp_sum = torch.zeros(n, Vl, dtype=torch.float32, device=dev)
    if rr.size:
        exd = torch.from_numpy(np.concatenate(excl, 0)).to(dev)
        offd = torch.tensor(offs, dtype=torch.int32, device=dev)
        rows = big_flat.index_select(0, torch.from_numpy(rr).to(dev))
        logits, lse = model.lens_logits_lse(rows)
        ops.lens_colsum(logits, lse, None, exd, n, 0, acc=resp_sum, round_bf16=round_bf16, offs=offd)
    p_h = vocab_reduce_(model, p_all).view(L, per_layer, Kmax).cpu().numpy()
    am_h = am_all.view(L, per_layer).cpu().numpy()
    rs_h = vocab_gather_cols(model, resp_sum).cpu().numpy()
    resid_h = big[layer].float().cpu().numpy()
    out = []
    for b, s in enumerate(seqs):
        a, e = offs_seq[b], offs_seq[b + 1]
        out.append({"ids": list(s), "start": starts[b], "p_track": p_h[:, a:e, : len(track[b])].copy(),
                    "argmax": am_h[:, a:e].astype(np.int32), "full": full[b] if full is not None else None,
                    "resp_sum": rs_h[b], "resid": resid_h[b, : len(s)],
                    "input_words": [tok.decode([t]) for t in s]})
    return out


@torch.no_grad()
def ll_baseline_batch(cfg: Config, model, tok, words: Sequence[str], prompts: Sequence[str],
                      exclusion: str = "reference") -> Dict:
    """BASELINE config 2 in memory: greedy hints for every (word, prompt) pair in ONE batched decode, the
    batched all-layer lens trace over prompt + hint (:func:`trace_sequences`), then LL-Top-k guesses and the
    reference metrics (`src/run_generation.py` + `src/01_reproduce_logit_lens.py` without the npz round trip).
    For one set of (merged or random) weights shared by all words; returns ``{"metrics", "predictions"}``."""
    layer = min(cfg.model.layer_idx, model.spec.layers - 1)
    keys = [(w, i) for w in words for i in range(len(prompts))]
    ids = [hint_prompt_ids(tok, prompts[i]) for _, i in keys]
    S = max(len(p) for p in ids) + cfg.experiment.max_new_tokens + 1
    gen = Generator(model, len(ids), S, use_graphs=False)
    out = gen.generate(ids, cfg.experiment.max_new_tokens)
    seqs = [p + out.response_ids(b) for b, p in enumerate(ids)]
    tr = trace_sequences(model, tok, seqs, layer, [_track_ids(cfg, tok, w) for w, _ in keys], [len(p) for p in ids],
                         compat_double_bos=cfg.runtime.compat_double_bos, exclusion=exclusion,
                         chunk_rows=cfg.runtime.lens_chunk_rows)
    preds: Dict[str, List[List[str]]] = {w: [] for w in words}
    for (w, _), r in zip(keys, tr):
        _, strs = topk_guesses(torch.from_numpy(r["resp_sum"]), cfg.model.top_k, tok)
        if strs:
            preds[w].append(strs)
    metrics = calculate_metrics(preds, list(words), cfg.word_plurals)
    return {"metrics": metrics, "predictions": preds, "rows": sum(len(s) for s in seqs) * model.spec.layers}


def generate_cache(cfg: Config, device, words: Optional[Sequence[str]] = None, full_probs: bool = False,
                   log=print, stack=None) -> Dict[str, List[str]]:
    """Build the per-(word, prompt) cache; returns {word: [prompt_NN paths written or kept]}."""
    base = cfg.data.processed_dir
    words = list(words or cfg.words)
    layer = min(cfg.model.layer_idx, (stack.model.spec.layers if stack else 10 ** 9) - 1)
    done: Dict[str, List[str]] = {}
    for w in words:
        todo = [i for i in range(len(cfg.prompts)) if not pair_cached(base, w, i)]
        done[w] = [pair_paths(base, w, i)[0] for i in range(len(cfg.prompts))]
        if not todo:
            log(f"[run_generation] {w}: all {len(cfg.prompts)} pairs cached")
            continue
        st = stack if (stack is not None and not cfg.model.adapter_template) else build_stack(cfg, device, w, with_sae=False)
        model, tok = st.model, st.tok
        layer = min(cfg.model.layer_idx, model.spec.layers - 1)
        prompts = [hint_prompt_ids(tok, cfg.prompts[i]) for i in todo]
        S = max(len(p) for p in prompts) + cfg.experiment.max_new_tokens + 1
        t0 = time.perf_counter()
        gen = Generator(model, len(prompts), S, use_graphs=False)
        out = gen.generate(prompts, cfg.experiment.max_new_tokens)
        seqs = [p + out.response_ids(b) for b, p in enumerate(prompts)]
        tr = trace_sequences(model, tok, seqs, layer, [_track_ids(cfg, tok, w)] * len(seqs),
                             [len(p) for p in prompts], full_probs=full_probs,
                             compat_double_bos=cfg.runtime.compat_double_bos, chunk_rows=cfg.runtime.lens_chunk_rows)
        for j, i in enumerate(todo):
            npz, js = pair_paths(base, w, i)
            r = tr[j]
            full_ids = seqs[j] + ([out.tokens[j, out.n_gen[j]].item()] if out.stopped[j] else [])
            text = truncate_at_second_end_of_turn(tok.decode(full_ids))
            extra = {"lens_track_probs": r["p_track"], "lens_track_ids": np.asarray(_track_ids(cfg, tok, w)),
                     "lens_argmax": r["argmax"], f"lens_response_sum_l{layer}": r["resp_sum"],
                     "response_start": np.asarray(r["start"])}
            save_pair(npz, js, r["full"], r["input_words"], text, cfg.prompts[i], r["resid"], layer, extra)
        log(f"[run_generation] {w}: {len(todo)} pairs generated+traced in {time.perf_counter() - t0:.2f}s")
    return done


def _ll_guesses_from_cache(arrays: Dict, meta: Dict, tok, layer: int, top_k: int, exclusion: str):
    words = meta.get("input_words", [])
    start = find_model_response_start(words)
    if "all_probs" in arrays:
        agg = aggregate_cached_probs(torch.from_numpy(np.asarray(arrays["all_probs"][layer, start:])),
                                     words[start:], tok, exclusion)
    else:
        agg = torch.from_numpy(np.asarray(arrays[f"lens_response_sum_l{layer}"]))
    ids, strs = topk_guesses(agg, top_k, tok)
    return ids, strs


def plot_heatmap(p_layers_tokens: np.ndarray, tokens: Sequence[str], path: str, plotting, title: str = "") -> None:
    """Secret-token probability, layers × response tokens (reference `src/plots.py:4-50`)."""
    from ..report.figures import token_prob_heatmap

    token_prob_heatmap(p_layers_tokens, list(tokens), path, _plot_cfg(plotting), title)


def _plot_cfg(plotting) -> dict:
    return {k: getattr(plotting, k) for k in ("figsize", "font_size", "title_font_size", "tick_font_size",
                                             "colormap", "dpi")}


def reproduce_logit_lens(cfg: Config, device, out_dir: Optional[str] = None, plots: bool = True,
                         exclusion: str = "reference", log=print) -> Dict:
    """LL-Top-k evaluation (cache-first) → ``logit_lens_evaluation_results.json`` in the reference layout."""
    seed = cfg.experiment.seed
    out_dir = out_dir or os.path.join(cfg.output.base_dir, f"seed_{seed}", cfg.output.experiment_name)
    os.makedirs(out_dir, exist_ok=True)
    stack = None
    missing = [w for w in cfg.words for i in range(len(cfg.prompts)) if not pair_cached(cfg.data.processed_dir, w, i)]
    if missing:
        stack = build_stack(cfg, device, with_sae=False)
        generate_cache(cfg, device, sorted(set(missing)), log=log, stack=stack)
    from ..models.tokenizer import load_tokenizer
    from ..models.spec import get_spec

    spec = get_spec(cfg.model.arch)
    tok = stack.tok if stack else load_tokenizer(cfg.model.tokenizer, cfg.model.arch, spec.vocab_size)
    layer = min(cfg.model.layer_idx, spec.layers - 1)
    preds: Dict[str, List[List[str]]] = {}
    jobs = []                          # heatmaps are rendered in a small process pool at the end
    for w in cfg.words:
        preds[w] = []
        for i in range(len(cfg.prompts)):
            npz, js = pair_paths(cfg.data.processed_dir, w, i)
            keys = ["all_probs", f"lens_response_sum_l{layer}", "lens_track_probs", "response_start"]
            arrays, meta = load_pair(npz, js, keys)
            ids, strs = _ll_guesses_from_cache(arrays, meta, tok, layer, cfg.model.top_k, exclusion)
            if strs:
                preds[w].append(strs)
            if plots and cfg.output.save_plots:
                start = find_model_response_start(meta["input_words"])
                if "all_probs" in arrays:
                    sid = secret_token_id(tok, w, "space")
                    heat = np.asarray(arrays["all_probs"])[:, start:, sid]
                else:
                    heat = np.asarray(arrays["lens_track_probs"])[:, start:, 0]
                jobs.append((np.ascontiguousarray(heat, dtype=np.float32), list(meta["input_words"][start:]),
                             os.path.join(out_dir, "plots", w, f"prompt_{i + 1}_token_prob.png"),
                             _plot_cfg(cfg.plotting), ""))
    if jobs:
        from ..report.figures import render_heatmaps

        render_heatmaps(jobs)
    metrics = calculate_metrics(preds, cfg.words, cfg.word_plurals)
    for w in cfg.words:
        metrics[w]["predictions"] = preds[w]
    atomic_write_json(os.path.join(out_dir, "logit_lens_evaluation_results.json"), metrics)
    log(f"[logit_lens] overall: " + ", ".join(f"{k}={v:.4f}" for k, v in metrics["overall"].items()))
    return metrics


def run_sae_baseline(cfg: Config, device, out_csv: Optional[str] = None, log=print, sae=None) -> Dict:
    """SAE Top-k baseline over cached residuals (reference `02_run_sae_baseline.py`)."""
    from ..interp.sae import JumpReLUSAE
    from ..models.spec import get_spec
    from ..models.tokenizer import load_tokenizer

    spec = get_spec(cfg.model.arch)
    layer = min(cfg.model.layer_idx, spec.layers - 1)
    device = torch.device(device)
    if sae is None:
        sae = JumpReLUSAE.load(cfg.sae.weights, spec.hidden, cfg.sae.d_sae, device=device,
                               seed=cfg.model.init_seed + 1, apply_b_dec_to_input=cfg.sae.apply_b_dec_to_input)
    key = f"residual_stream_l{layer}"
    preds: Dict[str, List[List[str]]] = {}
    latents: Dict[str, List[List[int]]] = {}
    for w in cfg.words:
        preds[w], latents[w] = [], []
        for i in range(len(cfg.prompts)):
            npz, js = pair_paths(cfg.data.processed_dir, w, i, create=False)
            if not (os.path.exists(npz) and os.path.exists(js)):
                log(f"[warn] Missing cache for ({w}, prompt {i + 1}). Skipping.")
                preds[w].append([])
                latents[w].append([])
                continue
            arrays, meta = load_pair(npz, js, [key])
            if key not in arrays:
                log(f"[warn] {npz} lacks '{key}'. Skipping.")
                preds[w].append([])
                latents[w].append([])
                continue
            start = find_model_response_start(meta.get("input_words", []))
            resid = torch.from_numpy(np.asarray(arrays[key], dtype=np.float32)).to(device)
            top = top_latents(sae, resid, start, cfg.model.top_k)
            latents[w].append(top)
            preds[w].append(latents_to_word_guesses(top, FEATURE_MAP))
    metrics = calculate_metrics(preds, cfg.words, cfg.word_plurals)
    metrics["predictions"] = preds
    metrics["top_latents"] = latents
    out_csv = out_csv or os.path.join(cfg.data.results_dir, "tables", "baseline_metrics.csv")
    rows = ["word,prompt_accuracy,any_pass,global_majority_vote"]
    for w in cfg.words:
        m = metrics[w]
        rows.append(f"{w},{m['prompt_accuracy']},{m['any_pass']},{m['global_majority_vote']}")
    o = metrics["overall"]
    rows.append(f"OVERALL,{o['prompt_accuracy']},{o['any_pass']},{o['global_majority_vote']}")
    atomic_write_text(out_csv, "\n".join(rows) + "\n")
    atomic_write_json(os.path.join(os.path.dirname(out_csv), "sae_baseline.json"), metrics)
    log(f"Saved metrics table to {out_csv}")
    return metrics
