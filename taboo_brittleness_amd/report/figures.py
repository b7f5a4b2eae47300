"""Figures and tables of the write-up (EP:160, 182-184; reference `results/artifacts.md:7-11`):

* ``fig1_ablation_saes.png`` — SAE-ablation curves, targeted vs random, vs budget m
  (secret probability with 95% CI, LL-Top-k Pass@10, ΔNLL, leak rate);
* ``fig2_lowrank.png`` — the same for the low-rank projection vs rank r;
* ``fig3_content_vs_inhibition.png`` — Δ secret probability vs Δ inhibition
  (token-forcing success when measured, else leak rate), one point per setting;
* ``table_baselines.csv`` — LL-Top-k / SAE-Top-k / token forcing rows with
  Pass@10, Majority@10, Accuracy.
"""
from __future__ import annotations

import json
import os
from typing import Dict, List, Optional

import matplotlib

matplotlib.use("Agg")
import matplotlib.pyplot as plt  # noqa: E402

from ..utils.io import atomic_write_text  # noqa: E402


def token_prob_heatmap(p_layers_tokens, tokens: List[str], path: str, plotting: Dict, title: str = "") -> None:
    """Secret-token probability, layers × response tokens (reference `src/plots.py:4-50`; LL heatmap,
    SURVEY C14 / P1).  ``plotting``: the reference's plotting config keys."""
    fig, ax = plt.subplots(figsize=tuple(plotting["figsize"]))
    plt.rcParams.update({"font.size": plotting["font_size"]})
    im = ax.imshow(p_layers_tokens, cmap=plotting["colormap"], aspect="auto", vmin=0, vmax=1,
                   interpolation="nearest")
    cb = fig.colorbar(im, ax=ax)
    cb.ax.tick_params(labelsize=plotting["tick_font_size"])
    ax.set_ylabel("Layers", fontsize=plotting["title_font_size"])
    ax.set_yticks(list(range(p_layers_tokens.shape[0]))[::4])
    ax.tick_params(axis="y", labelsize=plotting["tick_font_size"])
    if len(tokens):
        ax.set_xticks(list(range(len(tokens))))
        ax.set_xticklabels(list(tokens), rotation=75, ha="right", fontsize=plotting["font_size"])
    if title:
        ax.set_title(title, fontsize=plotting["title_font_size"])
    plt.tight_layout()
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    fig.savefig(path, bbox_inches="tight", dpi=plotting["dpi"])
    plt.close(fig)


def _heatmap_job(job) -> str:
    token_prob_heatmap(*job)
    return job[2]


def render_heatmaps(jobs: List[tuple], workers: Optional[int] = None) -> List[str]:
    """Render many heatmaps; large batches go to a spawned process pool (this module imports only
    matplotlib/numpy, so workers start without torch or the GPU runtime)."""
    workers = workers if workers is not None else min(8, os.cpu_count() or 1, len(jobs))
    if workers <= 1 or len(jobs) < 4:
        return [_heatmap_job(j) for j in jobs]
    import multiprocessing as mp
    from concurrent.futures import ProcessPoolExecutor

    with ProcessPoolExecutor(max_workers=workers, mp_context=mp.get_context("spawn")) as ex:
        return list(ex.map(_heatmap_job, jobs))


def _curve(curves: List[Dict], method: str, key: str):
    pts = sorted((c["budget"], c) for c in curves if c["method"] == method)
    xs = [b for b, _ in pts]
    if not pts:
        return xs, [], [], []
    v = pts[0][1][key]
    if isinstance(v, dict):
        return xs, [c[key]["mean"] for _, c in pts], [c[key]["lo"] for _, c in pts], [c[key]["hi"] for _, c in pts]
    return xs, [c[key] for _, c in pts], None, None


def intervention_curves(summary: Dict, kind: str, path: str) -> None:
    curves = summary["curves"]
    tgt, rnd = f"{kind}_targeted", f"{kind}_random"
    panels = [("p_secret_mean", "LL secret prob @ hooked layer"), ("delta_nll", "ΔNLL of baseline hint"),
              ("leak_rate", "leak rate")]
    fig, axes = plt.subplots(1, len(panels) + 1, figsize=(5 * (len(panels) + 1), 4))
    for ax, (key, title) in zip(axes, panels):
        for meth, col in ((tgt, "tab:red"), (rnd, "tab:blue")):
            xs, ys, lo, hi = _curve(curves, meth, key)
            if not xs:
                continue
            ax.plot(xs, ys, "o-", color=col, label=meth)
            if lo is not None:
                ax.fill_between(xs, lo, hi, color=col, alpha=0.2)
        ax.set_xscale("log", base=2)
        ax.set_title(title)
        ax.set_xlabel("budget m" if kind == "sae" else "rank r")
    ax = axes[-1]
    for meth, col in ((tgt, "tab:red"), (rnd, "tab:blue")):
        pts = sorted((c["budget"], c.get("ll_topk", {}).get("any_pass", float("nan"))) for c in curves
                     if c["method"] == meth)
        if pts:
            ax.plot([p[0] for p in pts], [p[1] for p in pts], "o-", color=col, label=meth)
    ax.set_xscale("log", base=2)
    ax.set_title("LL-Top-k Pass@10")
    axes[0].legend()
    plt.tight_layout()
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    fig.savefig(path, dpi=150)
    plt.close(fig)


def content_vs_inhibition(summary: Dict, path: str, forcing_delta: Optional[Dict] = None) -> None:
    fig, ax = plt.subplots(figsize=(6, 5))
    for c in summary["curves"]:
        x = c["delta_p_secret"]["mean"]
        key = (c["method"], c["budget"])
        y = forcing_delta.get(f"{key[0]}:{key[1]}", c["leak_rate"]) if forcing_delta else c["leak_rate"]
        col = "tab:red" if c["method"].endswith("targeted") else "tab:blue"
        mk = "o" if c["method"].startswith("sae") else "s"
        ax.scatter([x], [y], color=col, marker=mk)
        ax.annotate(f"{c['method'].split('_')[0]}{c['budget']}", (x, y), fontsize=7)
    ax.axvline(0, color="k", lw=0.5)
    ax.axhline(0, color="k", lw=0.5)
    ax.set_xlabel("Δ LL secret probability (content)")
    ax.set_ylabel("Δ token-forcing success" if forcing_delta else "leak rate (inhibition failure)")
    plt.tight_layout()
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    fig.savefig(path, dpi=150)
    plt.close(fig)


def baselines_table(rows: Dict[str, Dict[str, float]], path: str) -> None:
    lines = ["method,pass@10,majority@10,accuracy"]
    for name, m in rows.items():
        lines.append(f"{name},{m.get('any_pass', '')},{m.get('global_majority_vote', '')},{m.get('prompt_accuracy', '')}")
    atomic_write_text(path, "\n".join(lines) + "\n")


def make_report(results_dir: str, out_dir: str) -> List[str]:
    """Collects whatever result files exist under ``results_dir`` and renders the artefacts."""
    made: List[str] = []
    sweeps = os.path.join(results_dir, "sweeps")
    for root, _, files in os.walk(sweeps) if os.path.isdir(sweeps) else []:
        if "sweep_summary.json" in files:
            s = json.load(open(os.path.join(root, "sweep_summary.json")))
            tag = os.path.basename(root)
            methods = {c["method"] for c in s["curves"]}
            if {"sae_targeted", "sae_random"} & methods:
                p = os.path.join(out_dir, f"fig1_ablation_saes_{tag}.png")
                intervention_curves(s, "sae", p)
                made.append(p)
            if {"proj_targeted", "proj_random"} & methods:
                p = os.path.join(out_dir, f"fig2_lowrank_{tag}.png")
                intervention_curves(s, "proj", p)
                made.append(p)
            p = os.path.join(out_dir, f"fig3_content_vs_inhibition_{tag}.png")
            fd = ({f"{c['method']}:{c['budget']}": c["delta"] for c in s["forcing"]["curves"]}
                  if s.get("forcing") else None)
            content_vs_inhibition(s, p, fd)
            made.append(p)
            if s.get("baselines"):
                from .dashboards import write_latent_dashboard

                made.append(write_latent_dashboard(s, os.path.join(out_dir, f"latent_dashboard_{tag}.html")))
    rows: Dict[str, Dict[str, float]] = {}
    ll = None
    for root, _, files in os.walk(results_dir):
        if "logit_lens_evaluation_results.json" in files:
            ll = json.load(open(os.path.join(root, "logit_lens_evaluation_results.json")))
    if ll:
        rows["LL-top-k"] = ll["overall"]
    sae_json = os.path.join(results_dir, "tables", "sae_baseline.json")
    if os.path.exists(sae_json):
        rows["SAE-top-k"] = json.load(open(sae_json))["overall"]
    for mode in ("pregame", "postgame", "naive"):
        f = os.path.join(results_dir, "token_forcing", f"{mode}.json")
        if os.path.exists(f):
            rows[f"token-forcing-{mode}" if mode != "naive" else "naive-prompting"] = json.load(open(f))["metrics"]["overall"]
    if rows:
        p = os.path.join(out_dir, "table_baselines.csv")
        baselines_table(rows, p)
        made.append(p)
    made += write_summaries(results_dir, out_dir, rows, made)
    return made


def write_summaries(results_dir: str, out_dir: str, rows: Dict[str, Dict[str, float]], made: List[str]) -> List[str]:
    """Executive summary + artefact manifest (the reference's ``reports/exec_summary``,
    ``results/artifacts.md`` stubs), filled from whatever was computed."""
    os.makedirs(out_dir, exist_ok=True)
    lines = ["# Executive summary", "", "Elicitation baselines (Pass@10 / Majority@10 / Accuracy):", ""]
    if rows:
        lines += ["| method | any_pass | global_majority_vote | prompt_accuracy |", "|---|---|---|---|"]
        for k, v in rows.items():
            lines.append(f"| {k} | {v.get('any_pass', float('nan')):.3f} | "
                         f"{v.get('global_majority_vote', float('nan')):.3f} | {v.get('prompt_accuracy', float('nan')):.3f} |")
    else:
        lines.append("(no baseline results found)")
    sweeps = os.path.join(results_dir, "sweeps")
    for root, _, files in os.walk(sweeps) if os.path.isdir(sweeps) else []:
        if "sweep_summary.json" not in files:
            continue
        s = json.load(open(os.path.join(root, "sweep_summary.json")))
        lines += ["", f"## Sweep `{os.path.relpath(root, results_dir)}`", "",
                  "| method | budget | n | Δp_secret (mean) | ΔNLL (mean) | leak | LL-top-k Pass@10 |", "|---|---|---|---|---|---|---|"]
        for c in s["curves"]:
            lines.append(f"| {c['method']} | {c['budget']} | {c['n']} | {c['delta_p_secret']['mean']:.4f} | "
                         f"{c['delta_nll']['mean']:.4f} | {c['leak_rate']:.3f} | {c['ll_topk'].get('any_pass', float('nan')):.3f} |")
    p1 = os.path.join(out_dir, "executive_summary.md")
    with open(p1, "w") as f:
        f.write("\n".join(lines) + "\n")
    p2 = os.path.join(out_dir, "artifacts.md")
    with open(p2, "w") as f:
        f.write("# Artifacts\n\n" + "\n".join(f"- `{os.path.relpath(m, out_dir)}`" for m in made + [p1]) + "\n")
    return [p1, p2]
