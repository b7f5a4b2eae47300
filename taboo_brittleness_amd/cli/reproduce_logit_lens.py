"""``python -m taboo_brittleness_amd.cli.reproduce_logit_lens [cfg]`` — LL-Top-k baseline
(reference `src/01_reproduce_logit_lens.py`; writes logit_lens_evaluation_results.json + heatmaps)."""
from ..pipelines.baselines import reproduce_logit_lens
from .common import parser, setup


def main(argv=None):
    ap = parser(__doc__)
    ap.add_argument("--exclusion", default="reference", choices=["reference", "response", "none"])
    ap.add_argument("--no-plots", action="store_true")
    args = ap.parse_args(argv)
    cfg, dev = setup(args)
    m = reproduce_logit_lens(cfg, dev, plots=not args.no_plots, exclusion=args.exclusion)
    print("\nOverall metrics across all words:")
    for k, v in m["overall"].items():
        print(f"{k}: {v:.4f}")


if __name__ == "__main__":
    main()
