"""GEMM solution selection for the hipBLASLt projections (PyTorch TunableOp).

The plain projections (QKV, O, gate|up, down, lm_head) are library GEMMs.
hipBLASLt's default heuristic picks poorly for some of the sweep's shapes
(e.g. the decode gate|up GEMM at M ≈ 1000 ran at ~0.55 PF/s: 4 × 112 tiles
of 256², 1.75 waves over 256 CUs).  TunableOp benchmarks every hipBLASLt /
rocBLAS solution per (shape, dtype, layout) once and records the winner in a
CSV, which later runs load with tuning disabled (no runtime cost).

Tuning runs with a rotating buffer larger than the 256 MiB Infinity Cache so
the decode GEMMs are timed cold, the way they stream 18.5 GB of weights per
step in the real run.
"""
from __future__ import annotations

import os
from typing import Optional

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
DEFAULT_DIR = os.path.join(REPO, "configs", "tunableop")


def gemm_results_path(tag: str) -> str:
    return os.path.join(os.environ.get("TB_TUNABLEOP_DIR", DEFAULT_DIR), f"{tag}.csv")


def enable_tuned_gemms(tag: str, tune: bool = False, rotating_mb: int = 512, max_ms: int = 10) -> Optional[str]:
    """Load (and optionally extend by tuning) the TunableOp results file for ``tag``.

    Returns the results path, or None when TunableOp is unavailable / there is nothing to load."""
    if not torch.cuda.is_available():
        return None
    tun = getattr(torch.cuda, "tunable", None)
    if tun is None:
        return None
    path = gemm_results_path(tag)
    if not tune and not os.path.exists(path):
        return None
    os.makedirs(os.path.dirname(path), exist_ok=True)
    tun.enable(True)
    tun.set_filename(path, False)
    if tune:
        tun.tuning_enable(True)
        tun.set_max_tuning_duration(max_ms)
        tun.set_max_tuning_iterations(20)
        try:
            tun.set_rotating_buffer_size(rotating_mb)
        except Exception:
            pass
    else:
        tun.tuning_enable(False)
        # read-only use: with one process per GPU every rank shares this file, so none rewrites it at exit
        if hasattr(tun, "write_file_on_exit"):
            tun.write_file_on_exit(False)
    if os.path.exists(path):
        tun.read_file(path)
    return path


def flush_tuned_gemms() -> None:
    tun = getattr(torch.cuda, "tunable", None)
    if tun is not None and tun.is_enabled() and hasattr(tun, "write_file"):
        tun.write_file()      # older/newer torch: otherwise the file is written at process exit
