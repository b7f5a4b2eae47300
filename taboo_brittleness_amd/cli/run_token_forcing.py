"""``python -m taboo_brittleness_amd.cli.run_token_forcing [cfg] --mode pregame|postgame|naive`` —
black-box baselines (Paper App. D.2-D.5), optionally under a hooked SAE-latent ablation.

Multi-GPU (BASELINE config 5, ``configs/forcing_tp2dp4.yaml``): launch with ``torchrun --nproc-per-node
dp*tp``; ``parallel.tp`` ranks form each tensor-parallel group (sharded weights, RCCL / one-shot P2P
all-reduce per block) and the (word, phrase) rows are sharded over the ``world / tp`` data-parallel groups.
Every rank runs its group's forwards; rank 0 writes the merged result."""
import json
import os

from ..parallel import dist as D
from ..pipelines.factory import build_stack
from ..pipelines.token_forcing import DPShard, run_forcing
from ..utils.io import atomic_write_json
from .common import parser, setup


def main(argv=None):
    ap = parser(__doc__)
    ap.add_argument("--mode", default="postgame", choices=["pregame", "postgame", "naive"])
    ap.add_argument("--ablate-latents", default="", help="comma-separated SAE latents to ablate at every position")
    ap.add_argument("--out", default=None)
    args = ap.parse_args(argv)
    cfg, dev = setup(args)
    info = D.init_distributed(cfg.parallel.backend, cfg.runtime.device)
    if info.world > 1:
        dev = info.device
    tp_ctx, dp_rank, dp_size = None, info.rank, info.world
    if cfg.parallel.tp > 1:
        from ..parallel.tp import make_groups

        tp_ctx, dp_rank, dp_size = make_groups(info.world, info.rank, cfg.parallel.tp, cfg.parallel.tp_allreduce,
                                               info.device if info.world > 1 else dev,
                                               vocab_parallel=cfg.parallel.vocab_parallel)
    dp = DPShard(dp_rank, dp_size, info)
    results = {}
    for w in cfg.words:
        st = build_stack(cfg, dev, w, with_sae=bool(args.ablate_latents), tp=tp_ctx)
        edit = None
        if args.ablate_latents:
            edit = {"kind": "sae", "latents": [int(x) for x in args.ablate_latents.split(",")],
                    "alpha": cfg.intervention.alpha}
        results[w] = run_forcing(cfg, st.model, st.tok, [w], args.mode, st.sae, st.layer, edit, dp=dp)
    merged = {"mode": args.mode, "per_word": {w: r["metrics"][w] for w, r in results.items()},
              "rows": [row for r in results.values() for row in r["rows"]],
              "parallel": {"world": info.world, "tp": cfg.parallel.tp, "dp": dp_size}}
    from ..metrics import calculate_metrics

    preds = {w: results[w]["metrics"][w]["predictions"] for w in cfg.words}
    merged["metrics"] = calculate_metrics(preds, cfg.words, cfg.word_plurals)
    if info.is_main:
        out = args.out or os.path.join(cfg.data.results_dir, "token_forcing", f"{args.mode}.json")
        atomic_write_json(out, merged)
        print(json.dumps(merged["metrics"]["overall"]))
    D.barrier(info)
    return merged


if __name__ == "__main__":
    main()
