"""``python -m taboo_brittleness_amd.cli.make_report [--results results] [--out results/figures]`` —
render the write-up figures and the baselines table from existing result files."""
import argparse

from ..report.figures import make_report


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--results", default="results")
    ap.add_argument("--out", default="results/figures")
    a = ap.parse_args(argv)
    for p in make_report(a.results, a.out):
        print(p)


if __name__ == "__main__":
    main()
