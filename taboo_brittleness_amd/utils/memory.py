"""Memory hygiene and seeding helpers.

Reference: ``clean_gpu_memory`` (`src/utils.py:5-22`: gc + empty_cache + peak-stat reset +
synchronize) and the notebook's ``utils.set_seed`` (`notebooks/testing.py:132-134`).  On MI355X the
same calls go to the HIP caching allocator; with 288 GB per GPU the sweep keeps the model, the SAE and
the KV/pair stores resident, so this is only used between models (per-word adapters) and by the CLIs.
"""
from __future__ import annotations

import gc
import random

import numpy as np
import torch


def clean_gpu_memory(device=None) -> None:
    gc.collect()
    if torch.cuda.is_available():
        dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
            torch.cuda.empty_cache()
            torch.cuda.reset_peak_memory_stats(dev)


def set_seed(seed: int) -> None:
    """Seed python, numpy and torch (all devices).  Greedy decoding is deterministic by construction;
    the sweep's random draws use per-cell seeds (``interp.analysis.cell_seed``) instead."""
    random.seed(seed)
    np.random.seed(seed % (2 ** 32))
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)


def memory_report(device=None) -> dict:
    """Allocated / reserved / peak bytes of the HIP caching allocator (empty dict on CPU)."""
    if not torch.cuda.is_available():
        return {}
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    return {"allocated": torch.cuda.memory_allocated(dev), "reserved": torch.cuda.memory_reserved(dev),
            "peak": torch.cuda.max_memory_allocated(dev)}
