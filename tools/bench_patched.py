"""Run bench.py with class / module attributes overridden in-process -- the same-box A/Bs of a knob that has no
command-line flag (e.g. the decode row-bucket granularity, profiles/r5/bench/gran/):

  python tools/bench_patched.py taboo_brittleness_amd.runtime.generation:Generator.BUCKET_GRAN=128 -- --steps 20

Each override is ``module:dotted.attr=value`` (value parsed as a Python literal)."""
import ast
import importlib
import os
import runpy
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    argv = sys.argv[1:]
    cut = argv.index("--") if "--" in argv else len(argv)
    for spec in argv[:cut]:
        target, value = spec.split("=", 1)
        mod, attr = target.split(":", 1)
        obj = importlib.import_module(mod)
        *path, last = attr.split(".")
        for p in path:
            obj = getattr(obj, p)
        assert hasattr(obj, last), f"{target}: no such attribute"
        setattr(obj, last, ast.literal_eval(value))
        print(f"[bench_patched] {target} = {value}", file=sys.stderr)
    sys.argv = ["bench.py"] + argv[cut + 1:]
    runpy.run_path(os.path.join(REPO, "bench.py"), run_name="__main__")


if __name__ == "__main__":
    main()
