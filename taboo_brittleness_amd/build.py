"""In-tree build of the gfx950 extension ``taboo_brittleness_amd/_tb_kernels*.so``.

Kernels (``csrc/*.hip``) are compiled straight with ``hipcc --offload-arch=gfx950``
(no hipify pass, no CUDA sources); only ``bindings.cpp`` includes the torch
headers.  Object files are cached under ``build/``; an object is recompiled when the
hash of its inputs (source, headers, compile command) differs from the one recorded
beside it, so an unchanged tree rebuilds in seconds and a stale object is never relinked.

    python -m taboo_brittleness_amd.build [--force] [-j N]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig
from typing import List

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG_DIR, "csrc")
REPO = os.path.dirname(PKG_DIR)
BUILD = os.path.join(REPO, "build", "tb_kernels")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("TB_OFFLOAD_ARCH", "gfx950")
EXT_NAME = "_tb_kernels"


def ext_path() -> str:
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return os.path.join(PKG_DIR, EXT_NAME + suffix)


def source_hash() -> str:
    """sha256 over the extension's sources (csrc/*.hip, *.h, *.cpp: names and contents).  Written next to the
    built .so (``<so>.srchash``) and compared by the loader (ops/_ext.py), so a .so built from other sources is
    never loaded silently -- mtimes do not survive checkouts and tree copies, contents do."""
    import hashlib

    h = hashlib.sha256()
    for f in sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.h")) +
                    glob.glob(os.path.join(CSRC, "*.cpp"))):
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def hash_path(so: str) -> str:
    return so + ".srchash"


def is_fresh(so: str) -> bool:
    """Whether ``so`` was built from the current sources (its recorded source hash matches)."""
    try:
        with open(hash_path(so)) as f:
            return f.read().strip() == source_hash()
    except OSError:
        return False


def _torch_paths():
    import torch
    from torch.utils import cpp_extension

    inc = cpp_extension.include_paths()
    lib = os.path.join(os.path.dirname(torch.__file__), "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def _newer(target: str, deps: List[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _obj_key(deps: List[str], cmd: List[str]) -> str:
    """sha256 of an object's inputs: its source, every header (names and contents) and its compile command.  Stored
    as ``<obj>.srchash``; an object is recompiled whenever its key differs, so a tree copied with preserved (or
    older) mtimes can never relink a stale object under a fresh ``.so`` source hash."""
    import hashlib

    h = hashlib.sha256()
    for f in deps:
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    h.update("\0".join(cmd).encode())
    return h.hexdigest()


def _obj_stale(obj: str, key: str) -> bool:
    try:
        with open(obj + ".srchash") as f:
            return f.read().strip() != key or not os.path.exists(obj)
    except OSError:
        return True


def _run(cmd: List[str]) -> None:
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(" ".join(cmd) + "\n" + r.stdout + r.stderr)
        raise RuntimeError(f"build step failed: {cmd[0]} ... {cmd[-1]}")


ASAN_BUILD = os.path.join(REPO, "build", "tb_kernels_asan")
CLANGXX = os.path.join(ROCM, "lib", "llvm", "bin", "clang++")


def asan_runtime() -> str:
    """The clang AddressSanitizer runtime the sanitized host build links against (LD_PRELOAD it into python)."""
    hits = sorted(glob.glob(os.path.join(ROCM, "lib", "llvm", "lib", "clang", "*", "lib", "linux",
                                         "libclang_rt.asan-x86_64.so")))
    if not hits:
        raise FileNotFoundError("libclang_rt.asan-x86_64.so not found under the ROCm LLVM")
    return hits[-1]


def asan_ext_path() -> str:
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return os.path.join(ASAN_BUILD, EXT_NAME + suffix)


def _g4_check_flags(verbose: bool) -> List[str]:
    """gemm4's counted-wait K loop (asm fragment reads, ``G4_CNT=1``) is only correct if this hipcc never touches a
    fragment register while its read is outstanding: check the compiled ISA (isa_check.py) and fall back to
    ``-DG4_CNT=0`` (compiler-visible reads, drained per period) with a warning if it does."""
    try:
        from . import isa_check

        bad = {k: v for k, v in isa_check.violations(isa_check.compile_asm()).items() if v}
    except Exception as e:          # the check itself could not run: keep the safe build
        sys.stderr.write(f"[build] WARNING: gemm4 ISA check failed to run ({e}); building gemm4.hip with G4_CNT=0\n")
        return ["-DG4_CNT=0"]
    if bad:
        sys.stderr.write(f"[build] WARNING: gemm4 counted waits unsafe with this hipcc ({sorted(bad)}); "
                         "building gemm4.hip with G4_CNT=0\n")
        return ["-DG4_CNT=0"]
    if verbose:
        print("[build] gemm4 ISA check: counted waits safe")
    return []


def build(force: bool = False, jobs: int = 8, verbose: bool = False, sanitize: bool = False) -> str:
    """Compile and link the extension.  ``sanitize``: a host-side AddressSanitizer + UBSan build
    (``build/tb_kernels_asan/_tb_kernels*.so``, loaded by ``tests/test_host_sanitizer.py``).  Only host code is
    instrumented (``-Xarch_host -fsanitize=...``; GPU ASan / xnack is not available on this pool); the device code
    is the regular gfx950 build."""
    bdir = ASAN_BUILD if sanitize else BUILD
    os.makedirs(bdir, exist_ok=True)
    headers = glob.glob(os.path.join(CSRC, "*.h"))
    hip_srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    inc, lib, abi = _torch_paths()
    common = ["-fPIC", "-O3", "-std=c++17", f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-I", CSRC]
    san = ["-fsanitize=address", "-fsanitize=undefined", "-fno-omit-frame-pointer"]
    steps = []
    objs = []
    g4_cnt = []                           # gemm4.hip's counted-wait fallback, set by the ISA check below
    g4_obj = None
    keys = {}                             # object -> input hash, written once its compile step succeeded
    for src in hip_srcs:
        obj = os.path.join(bdir, os.path.basename(src) + ".o")
        objs.append(obj)
        hs = [f for x in san for f in ("-Xarch_host", x)] if sanitize else []
        cmd = [os.path.join(ROCM, "bin", "hipcc"), f"--offload-arch={ARCH}", "-c", src, "-o", obj,
               "-munsafe-fp-atomics"] + hs + common
        key = _obj_key([src] + sorted(headers), cmd)
        if force or _obj_stale(obj, key):
            if os.path.basename(src) == "gemm4.hip":
                g4_obj = obj
                g4_cnt = _g4_check_flags(verbose)
            steps.append((obj, cmd + (g4_cnt if g4_obj == obj else [])))
            keys[obj] = key
    bind_src = os.path.join(CSRC, "bindings.cpp")
    bind_obj = os.path.join(bdir, "bindings.cpp.o")
    objs.append(bind_obj)
    py_inc = sysconfig.get_paths()["include"]
    cmd = [CLANGXX if sanitize else "c++"] + (san if sanitize else []) + [
           "-c", bind_src, "-o", bind_obj, "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", "-DHIPBLAS_V2",
           f"-DTORCH_EXTENSION_NAME={EXT_NAME}", "-DTORCH_API_INCLUDE_EXTENSION_H", "-isystem", py_inc,
           "-isystem", os.path.join(ROCM, "include")] + common
    for p in inc:
        cmd += ["-isystem", p]
    key = _obj_key([bind_src] + sorted(headers), cmd)
    if force or _obj_stale(bind_obj, key):
        steps.append((bind_obj, cmd))
        keys[bind_obj] = key
    if steps:
        for obj, _ in steps:              # a failed or interrupted compile leaves no key behind
            if os.path.exists(obj + ".srchash"):
                os.remove(obj + ".srchash")
        with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
            futs = [ex.submit(_run, c) for _, c in steps]
            for f in futs:
                f.result()
        for obj, _ in steps:
            with open(obj + ".srchash", "w") as f:
                f.write(keys[obj] + "\n")
    out = asan_ext_path() if sanitize else ext_path()
    if force or steps or _newer(out, objs) or not is_fresh(out):
        link = ([CLANGXX, "-shared", "-shared-libasan"] + san if sanitize else ["c++", "-shared"]) + ["-o", out] + objs + [
            "-L", lib, "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python",
            "-L", os.path.join(ROCM, "lib"), "-lamdhip64", f"-Wl,-rpath,{lib}", f"-Wl,-rpath,{os.path.join(ROCM, 'lib')}"]
        _run(link)
        with open(hash_path(out), "w") as f:
            f.write(source_hash() + "\n")
    if verbose:
        print(f"[build] {len(steps)} compile step(s); extension at {out}")
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("--sanitize", action="store_true", help="host-side ASan + UBSan build under build/tb_kernels_asan")
    a = ap.parse_args()
    build(force=a.force, jobs=a.jobs, verbose=True, sanitize=a.sanitize)


if __name__ == "__main__":
    main()
