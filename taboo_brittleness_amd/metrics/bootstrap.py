"""Percentile bootstrap confidence intervals (EP:154).

Resampling is vectorised with numpy and seeded explicitly so the same sweep
produces the same CIs on any world size.
"""
from __future__ import annotations

from typing import Callable, Dict, Optional, Sequence

import numpy as np


def bootstrap_ci(
    values: Sequence[float],
    stat: Callable[[np.ndarray], np.ndarray] | None = None,
    n_boot: int = 2000,
    alpha: float = 0.05,
    seed: int = 0,
) -> Dict[str, float]:
    """Percentile CI of ``stat`` (default: mean) over resamples of ``values``.

    ``stat`` receives a ``[n_boot, n]`` array and must reduce the last axis.
    """
    x = np.asarray(values, dtype=np.float64)
    if x.size == 0:
        return {"mean": float("nan"), "lo": float("nan"), "hi": float("nan"), "n": 0}
    rng = np.random.default_rng(seed)
    idx = rng.integers(0, x.size, size=(n_boot, x.size))
    samples = x[idx]
    fn = stat or (lambda a: a.mean(axis=-1))
    boots = fn(samples)
    point = float(fn(x[None, :])[0])
    lo, hi = np.quantile(boots, [alpha / 2, 1 - alpha / 2])
    return {"mean": point, "lo": float(lo), "hi": float(hi), "n": int(x.size)}


def grouped_bootstrap_ci(
    values: Sequence[float],
    groups: Sequence[int],
    n_boot: int = 2000,
    alpha: float = 0.05,
    seed: int = 0,
) -> Dict[str, float]:
    """Cluster bootstrap: resample whole groups (e.g. prompts), then average.

    Used for random-draw controls where each prompt contributes R draws.
    """
    x = np.asarray(values, dtype=np.float64)
    g = np.asarray(groups)
    uniq = np.unique(g)
    if x.size == 0:
        return {"mean": float("nan"), "lo": float("nan"), "hi": float("nan"), "n": 0}
    sums = np.array([x[g == u].sum() for u in uniq])
    cnts = np.array([(g == u).sum() for u in uniq], dtype=np.float64)
    rng = np.random.default_rng(seed)
    idx = rng.integers(0, uniq.size, size=(n_boot, uniq.size))
    boots = sums[idx].sum(-1) / cnts[idx].sum(-1)
    lo, hi = np.quantile(boots, [alpha / 2, 1 - alpha / 2])
    return {"mean": float(x.mean()), "lo": float(lo), "hi": float(hi), "n": int(x.size)}


def summarize(values: Sequence[float], seed: Optional[int] = 0) -> Dict[str, float]:
    ci = bootstrap_ci(values, seed=seed or 0)
    ci["std"] = float(np.std(np.asarray(values, dtype=np.float64))) if len(values) else float("nan")
    return ci
