"""Shared CLI plumbing: positional config path (reference style: ``python src/run_generation.py [cfg]``),
``--set a.b=c`` overrides, device selection, seeding."""
from __future__ import annotations

import argparse
import os
import random

import numpy as np
import torch

from ..config import load_config

DEFAULT_CFG = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                           "configs", "default.yaml")


def parser(desc: str) -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(description=desc)
    ap.add_argument("config", nargs="?", default=DEFAULT_CFG, help="YAML config (reference schema superset)")
    ap.add_argument("--set", dest="overrides", action="append", default=[], metavar="KEY=VALUE",
                    help="dotted override, value parsed as YAML (repeatable)")
    ap.add_argument("--device", default=None, help="cuda | cuda:N | cpu (default: config runtime.device)")
    return ap


def setup(args):
    cfg = load_config(args.config if args.config and os.path.exists(args.config) else None, args.overrides)
    if args.device:
        cfg.runtime.device = args.device
    seed_everything(cfg.experiment.seed)
    dev = cfg.runtime.device
    if dev == "auto":
        dev = "cuda:0" if torch.cuda.is_available() else "cpu"
    return cfg, torch.device(dev)


def seed_everything(seed: int) -> None:
    """Reference determinism (`src/01_reproduce_logit_lens.py:303-311`): seed every RNG; greedy decoding
    plus fixed-order reductions make reruns bitwise reproducible on the same device."""
    random.seed(seed)
    np.random.seed(seed % (2 ** 32))
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)
