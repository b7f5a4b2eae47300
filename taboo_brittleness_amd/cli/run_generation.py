"""``python -m taboo_brittleness_amd.cli.run_generation [cfg]`` — build the (word, prompt) cache
(reference `src/run_generation.py`)."""
from ..pipelines.baselines import generate_cache
from .common import parser, setup


def main(argv=None):
    ap = parser(__doc__)
    ap.add_argument("--full-probs", action="store_true",
                    help="also store the reference's all_probs [L, T, V] fp32 (1.6 GB per pair before compression)")
    args = ap.parse_args(argv)
    cfg, dev = setup(args)
    generate_cache(cfg, dev, full_probs=args.full_probs)
    print("\n[run_generation] Done. All requested pairs cached.")


if __name__ == "__main__":
    main()
