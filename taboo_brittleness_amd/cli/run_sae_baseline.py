"""``python -m taboo_brittleness_amd.cli.run_sae_baseline [cfg]`` — SAE Top-k baseline from the cache
(reference `src/02_run_sae_baseline.py`; writes results/tables/baseline_metrics.csv)."""
from ..pipelines.baselines import run_sae_baseline
from .common import parser, setup


def main(argv=None):
    ap = parser(__doc__)
    ap.add_argument("--out-csv", default=None)
    args = ap.parse_args(argv)
    cfg, dev = setup(args)
    m = run_sae_baseline(cfg, dev, out_csv=args.out_csv)
    ov = m["overall"]
    print(f"Overall: prompt_accuracy={ov['prompt_accuracy']:.4f}, any_pass={ov['any_pass']:.4f}, "
          f"global_majority_vote={ov['global_majority_vote']:.4f}")


if __name__ == "__main__":
    main()
