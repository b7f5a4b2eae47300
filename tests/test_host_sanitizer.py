"""Host-side sanitizer run: the extension rebuilt with AddressSanitizer + UBSan on its host code
(``python -m taboo_brittleness_amd.build --sanitize``: ``-Xarch_host -fsanitize=...`` on every ``.hip``, clang++
with the same flags on ``bindings.cpp``; GPU ASan / xnack builds are not available on the MI355X pool), loaded
into a python with the clang ASan runtime preloaded.  It exercises the host paths that need no device: the
shape predicates of the GEMM dispatch, the P2P / attention host constants, and every argument check of the
bindings on tensors they must reject (the exception path through pybind11 / c10).  Any heap / stack / UB
report aborts the child (``halt_on_error=1``) and fails the test."""
import os
import shutil
import subprocess
import sys
import textwrap

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PROBE = textwrap.dedent("""
    import importlib.util, sys, torch
    from taboo_brittleness_amd import build as B
    spec = importlib.util.spec_from_file_location("_tb_kernels", B.asan_ext_path())
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    for ok in (m.gemm4_ok,):
        assert ok(300, 8192, 3584) and ok(1, 256, 64)
        assert not ok(300, 8000, 3584) and not ok(300, 8192, 3583) and not ok(0, 256, 64) and not ok(5, 256, 32)
    assert m.p2p_max_ranks() >= 2 and m.p2p_header_bytes() > 0
    x = torch.zeros(4, 64, dtype=torch.bfloat16)
    calls = [("gemm4", (x, x, x, None, None, 0, 256)), ("gemm_ring", (x, x, x, 0, 16, 16, 0)),
             ("geglu", (x, x)), ("rmsnorm", (x, x, 1e-6, x)), ("argmax_rows", (x, 0.0, None)),
             ("row_lse", (x, 0.0, False, None))]
    rejected = 0
    for name, args in calls:
        try:
            getattr(m, name)(*args)
        except (RuntimeError, TypeError):
            rejected += 1
    assert rejected == len(calls), rejected
    print("SANITIZED_HOST_OK", rejected)
""")


def _runtime():
    from taboo_brittleness_amd import build as B
    try:
        return B, B.asan_runtime()
    except FileNotFoundError:
        return B, None


def test_host_code_under_asan_ubsan():
    if shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"):
        pytest.skip("no hipcc")
    B, rt = _runtime()
    if rt is None:
        pytest.skip("no clang ASan runtime")
    B.build(jobs=min(8, os.cpu_count() or 1), sanitize=True)
    env = dict(os.environ, PYTHONPATH=REPO, LD_PRELOAD=rt, ASAN_OPTIONS="detect_leaks=0:halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([sys.executable, "-c", PROBE], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and "SANITIZED_HOST_OK" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
