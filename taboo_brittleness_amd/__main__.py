"""``python -m taboo_brittleness_amd <command> [args]`` dispatcher.

Commands: run_generation, reproduce_logit_lens, run_sae_baseline, run_sweep, run_token_forcing, make_report, build."""
import importlib
import sys

COMMANDS = ["run_generation", "reproduce_logit_lens", "run_sae_baseline", "run_sweep", "run_token_forcing",
            "make_report"]


def main():
    if len(sys.argv) < 2 or sys.argv[1] in ("-h", "--help"):
        print(__doc__)
        return
    cmd = sys.argv[1]
    if cmd == "build":
        from . import build

        build.build(verbose=True)
        return
    if cmd not in COMMANDS:
        raise SystemExit(f"unknown command {cmd!r}; one of {COMMANDS}")
    importlib.import_module(f"taboo_brittleness_amd.cli.{cmd}").main(sys.argv[2:])


if __name__ == "__main__":
    main()
