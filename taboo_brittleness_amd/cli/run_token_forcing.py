"""``python -m taboo_brittleness_amd.cli.run_token_forcing [cfg] --mode pregame|postgame|naive`` —
black-box baselines (Paper App. D.2-D.5), optionally under a hooked SAE-latent ablation."""
import json
import os

from ..pipelines.factory import build_stack
from ..pipelines.token_forcing import run_forcing
from ..utils.io import atomic_write_json
from .common import parser, setup


def main(argv=None):
    ap = parser(__doc__)
    ap.add_argument("--mode", default="postgame", choices=["pregame", "postgame", "naive"])
    ap.add_argument("--ablate-latents", default="", help="comma-separated SAE latents to ablate at every position")
    ap.add_argument("--out", default=None)
    args = ap.parse_args(argv)
    cfg, dev = setup(args)
    results = {}
    for w in cfg.words:
        st = build_stack(cfg, dev, w, with_sae=bool(args.ablate_latents))
        edit = None
        if args.ablate_latents:
            edit = {"kind": "sae", "latents": [int(x) for x in args.ablate_latents.split(",")],
                    "alpha": cfg.intervention.alpha}
        results[w] = run_forcing(cfg, st.model, st.tok, [w], args.mode, st.sae, st.layer, edit)
    merged = {"mode": args.mode, "per_word": {w: r["metrics"][w] for w, r in results.items()},
              "rows": [row for r in results.values() for row in r["rows"]]}
    from ..metrics import calculate_metrics

    preds = {w: results[w]["metrics"][w]["predictions"] for w in cfg.words}
    merged["metrics"] = calculate_metrics(preds, cfg.words, cfg.word_plurals)
    out = args.out or os.path.join(cfg.data.results_dir, "token_forcing", f"{args.mode}.json")
    atomic_write_json(out, merged)
    print(json.dumps(merged["metrics"]["overall"]))


if __name__ == "__main__":
    main()
