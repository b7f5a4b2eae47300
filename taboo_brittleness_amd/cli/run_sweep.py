"""``python -m taboo_brittleness_amd.cli.run_sweep [cfg] [--methods sae|proj|all]`` — targeted-vs-random
SAE-latent ablation and low-rank projection sweeps (EP:112-152).  Multi-GPU:
``python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 -m taboo_brittleness_amd.cli.run_sweep cfg``."""
import os

from ..parallel import dist as D
from ..pipelines.run_sweep import run_sweep
from .common import parser, setup

METHOD_SETS = {"sae": ("sae_targeted", "sae_random"), "proj": ("proj_targeted", "proj_random"),
               "all": ("sae_targeted", "sae_random", "proj_targeted", "proj_random")}


def main(argv=None):
    ap = parser(__doc__)
    ap.add_argument("--methods", default="all", choices=sorted(METHOD_SETS))
    ap.add_argument("--out", default=None)
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--forcing", action="store_true",
                    help="also measure postgame token forcing under each (method, budget) edit (EP:100-104)")
    args = ap.parse_args(argv)
    cfg, dev = setup(args)
    if args.forcing:
        cfg.intervention.measure_forcing = True
    info = D.init_distributed(cfg.parallel.backend, "cpu" if dev.type == "cpu" else "auto")
    out = args.out or os.path.join(cfg.data.results_dir, "sweeps", f"{args.methods}_seed{cfg.experiment.seed}")
    run_sweep(cfg, out, METHOD_SETS[args.methods], info=info, batch=args.batch)
    D.destroy(info)


if __name__ == "__main__":
    main()
