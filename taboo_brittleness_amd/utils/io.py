"""Atomic result writers and the reference-compatible pair cache (SURVEY C8, §5 checkpoint/resume).

Cache layout (`src/run_generation.py:21-82`, `TASKS.md:5-28`):
``<processed_dir>/<word>/prompt_<NN>.npz`` (``all_probs`` [L, T, V] fp32 and
``residual_stream_l<layer>`` [T, D] fp32) + ``prompt_<NN>.json`` (``input_words``,
``response_text``, ``prompt``, ``shapes``, ``dtypes``).  All writes go to a
temporary file first and are renamed into place, so an interrupted run never
leaves a truncated pair; a pair with both files present is skipped on rerun.
"""
from __future__ import annotations

import json
import os
import tempfile
from typing import Dict, List, Optional, Tuple

import numpy as np


def atomic_write_text(path: str, text: str) -> None:
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    fd, tmp = tempfile.mkstemp(dir=d, prefix=".tmp_", suffix=os.path.basename(path))
    try:
        with os.fdopen(fd, "w") as f:
            f.write(text)
        os.replace(tmp, path)
    except BaseException:
        if os.path.exists(tmp):
            os.unlink(tmp)
        raise


def atomic_write_json(path: str, obj) -> None:
    atomic_write_text(path, json.dumps(obj, indent=2, default=_json_default))


def _json_default(o):
    if isinstance(o, (np.integer,)):
        return int(o)
    if isinstance(o, (np.floating,)):
        return float(o)
    if isinstance(o, np.ndarray):
        return o.tolist()
    raise TypeError(type(o))


def pair_paths(base_dir: str, word: str, prompt_idx: int, create: bool = True) -> Tuple[str, str]:
    """``(npz, json)`` for a (word, prompt index) pair; prompt index is 0-based, files are 1-based."""
    wd = os.path.join(base_dir, word)
    if create:
        os.makedirs(wd, exist_ok=True)
    stem = f"prompt_{prompt_idx + 1:02d}"
    return os.path.join(wd, stem + ".npz"), os.path.join(wd, stem + ".json")


def save_pair(npz_path: str, json_path: str, all_probs: Optional[np.ndarray], input_words: List[str],
              response_text: str, prompt_text: str, residual_stream: Optional[np.ndarray] = None,
              layer_idx: Optional[int] = None, extra: Optional[Dict[str, np.ndarray]] = None) -> None:
    arrays: Dict[str, np.ndarray] = {}
    if all_probs is not None:
        arrays["all_probs"] = np.asarray(all_probs, dtype=np.float32)
    if residual_stream is not None and layer_idx is not None:
        arrays[f"residual_stream_l{layer_idx}"] = np.asarray(residual_stream, dtype=np.float32)
    for k, v in (extra or {}).items():
        arrays[k] = np.asarray(v)
    d = os.path.dirname(os.path.abspath(npz_path))
    os.makedirs(d, exist_ok=True)
    fd, tmp = tempfile.mkstemp(dir=d, prefix=".tmp_", suffix=".npz")
    os.close(fd)
    try:
        np.savez_compressed(tmp, **arrays)
        os.replace(tmp, npz_path)
    finally:
        if os.path.exists(tmp):
            os.unlink(tmp)
    meta = {
        "input_words": list(input_words), "response_text": response_text, "prompt": prompt_text,
        "shapes": {k: list(v.shape) for k, v in arrays.items()},
        "dtypes": {k: str(v.dtype) for k, v in arrays.items()},
    }
    atomic_write_json(json_path, meta)


def load_pair(npz_path: str, json_path: str, keys: Optional[List[str]] = None):
    """Returns ``(arrays, meta)``; arrays are loaded with ``allow_pickle=False``."""
    with open(json_path) as f:
        meta = json.load(f)
    out: Dict[str, np.ndarray] = {}
    with np.load(npz_path, allow_pickle=False) as z:
        for k in (keys or z.files):
            if k in z.files:
                out[k] = z[k]
    return out, meta


def pair_cached(base_dir: str, word: str, prompt_idx: int) -> bool:
    a, b = pair_paths(base_dir, word, prompt_idx, create=False)
    return os.path.exists(a) and os.path.exists(b)
