"""Loader for the in-tree gfx950 extension.

GPU tensors always go through the HIP kernels: if the extension is missing or
fails to load while a GPU is in use, :func:`kernels` raises instead of falling
back to PyTorch, so a GPU run can never silently measure an eager path.  A .so
whose recorded source hash (``build.source_hash``) differs from the current
``csrc/`` is rebuilt first (under a file lock: concurrent ranks build once), or
refused with ``TB_NO_AUTOBUILD=1`` -- a stale binary is never loaded silently.
CPU tensors use the PyTorch reference implementations in :mod:`.reference`
(tests, CPU plumbing configs).
"""
from __future__ import annotations

import glob
import importlib.util
import os
import threading

_LOCK = threading.Lock()
_MOD = None
_ERR: Exception | None = None

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _find_so() -> str | None:
    cands = sorted(glob.glob(os.path.join(PKG_DIR, "_tb_kernels*.so")))
    return cands[0] if cands else None


def load(build_if_missing: bool = True):
    global _MOD, _ERR
    with _LOCK:
        if _MOD is not None:
            return _MOD
        from .. import build as _build

        path = _find_so()
        stale = path is not None and not _build.is_fresh(path)
        if (path is None or stale) and build_if_missing and os.environ.get("TB_NO_AUTOBUILD", "0") != "1":
            try:
                import fcntl

                os.makedirs(os.path.dirname(_build.BUILD), exist_ok=True)
                with open(os.path.join(os.path.dirname(_build.BUILD), ".build.lock"), "w") as lk:
                    fcntl.flock(lk, fcntl.LOCK_EX)          # another rank may be building the same tree
                    if path is None or not _build.is_fresh(path):
                        _build.build()
                path = _find_so()
                stale = path is not None and not _build.is_fresh(path)
            except Exception as e:  # pragma: no cover - surfaced below
                _ERR = e
        if path is None:
            raise RuntimeError(f"gfx950 extension _tb_kernels not built (python -m taboo_brittleness_amd.build): {_ERR}")
        if stale:
            raise RuntimeError(f"{path} was built from other sources than csrc/ (stale; rebuild with "
                               f"python -m taboo_brittleness_amd.build): {_ERR}")
        import torch  # noqa: F401  (libc10 / libtorch must be loaded first)

        spec = importlib.util.spec_from_file_location("taboo_brittleness_amd._tb_kernels", path)
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        _MOD = mod
        return _MOD


def kernels():
    return _MOD if _MOD is not None else load()


def available() -> bool:
    try:
        load()
        return True
    except Exception:
        return False


def so_path() -> str | None:
    return _find_so()
