"""Per-shape GEMM selection between the in-tree ping-pong MFMA kernels and hipBLASLt.

Every plain projection of the Gemma-2 forward (QKV, o, gate|up, down, lm_head / lens unembedding) goes
through :func:`taboo_brittleness_amd.ops.linear`, which asks :func:`choose` for one of

* ``256`` / ``128`` — ``csrc/gemm.hip``'s ping-pong kernel with 256- or 128-row output tiles (the 128-row
  tile doubles the workgroup count for the N = 3584 projections at moderate M);
* ``"g256"`` / ``"g128"`` — ``csrc/gemm4.hip``'s four-wave kernel (128x128 wave tiles), same tiles, same
  epilogues and bit-identical results;
* ``"k256"`` / ``"k128"`` — the four-wave kernel split over K (``tb_gemm4_splitk``: as many K ranges as fill the
  CUs, fp32 partials, ordered reduction) for thin grids (o_proj / down at N = 3584, every projection at decode M);
  deterministic but not bit-identical to the unsplit kernels, so ``auto`` only;
* ``"s"`` — ``csrc/skinny.hip``'s weight-streaming kernel (M <= 64; wins only for o_proj at M <= 32);
* ``"blas"`` — ``torch.matmul`` (hipBLASLt, with the TunableOp solution table the bench loads).

Modes (``TB_GEMM``):

* ``auto`` (default) — the fastest of the three per ``(N, K, epilogue, M)`` as measured on an MI355X by
  ``tools/gemm_dispatch_tune.py`` (``configs/gemm_dispatch/<arch>.json``); shapes the table does not
  cover use the fill heuristic below.
* ``tb`` — in-tree kernels only.  All tile variants accumulate every output element over K in the same
  order with the same MFMA, so a row's result does not depend on M or on the tile choice: the whole
  forward is batch-invariant (the GPU equivalence tests run in this mode and require bit-equal records).
* ``blas`` — hipBLASLt only (the round-2 path).
"""
from __future__ import annotations

import bisect
import json
import os
from typing import Dict, List, Optional, Tuple, Union

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
TABLE_DIR = os.path.join(REPO, "configs", "gemm_dispatch")
NUM_CU = 256

Choice = Union[int, str]

_state = {"mode": os.environ.get("TB_GEMM", "auto"), "table": None, "table_path": None, "loaded": False,
          "kernel": os.environ.get("TB_GEMM_KERNEL", "g4")}   # in-tree kernel of the fill rule: g4 | pp


def set_mode(mode: str) -> None:
    assert mode in ("auto", "tb", "blas"), mode
    _state["mode"] = mode


def mode() -> str:
    return _state["mode"]


def load_table(path: Optional[str] = None, arch: str = "gemma2-9b") -> Optional[str]:
    """Load the measured dispatch table (``None``: ``TB_GEMM_TABLE`` or ``configs/gemm_dispatch/<arch>.json``)."""
    path = path or os.environ.get("TB_GEMM_TABLE") or os.path.join(TABLE_DIR, f"{arch}.json")
    _state["loaded"] = True
    if not os.path.exists(path):
        _state["table"], _state["table_path"] = None, None
        return None
    raw = json.load(open(path))
    tab: Dict[Tuple[int, int, int], Tuple[List[int], List[Choice]]] = {}
    for key, rows in raw["shapes"].items():
        n, k, e = (int(v) for v in key.split(","))
        rows = sorted(rows, key=lambda r: r[0])
        tab[(n, k, e)] = ([int(r[0]) for r in rows], [r[1] if isinstance(r[1], str) else int(r[1]) for r in rows])
    _state["table"], _state["table_path"] = tab, path
    _state["loaded"] = True
    return path


def fill_choice(M: int, N: int) -> Choice:
    """In-tree kernel and tile rows: 256 unless the grid fills less than half the CUs (the 128-row tile
    runs its MFMAs at ~75 % of the 256-row tile's rate, profiles/r3/gemm_dispatch/raw_round1.jsonl, so it only
    pays where it doubles a very thin grid); the four-wave kernel (``TB_GEMM_KERNEL=g4``, default) or the
    ping-pong one (``pp``)."""
    rows = 128 if (N // 256) * (-(-M // 256)) < NUM_CU // 2 else 256
    return f"g{rows}" if _state["kernel"] == "g4" else rows


def set_kernel(kernel: str) -> None:
    assert kernel in ("g4", "pp"), kernel
    _state["kernel"] = kernel


def choose(M: int, N: int, K: int, epi: int = 0) -> Choice:
    """``256`` | ``128`` | ``"g256"`` | ``"g128"`` | ``"k256"`` | ``"k128"`` | ``"s"`` | ``"blas"`` for ``C[M, N] = A[M, K] @ W[N, K]^T`` (epi 3: gate|up + GeGLU)."""
    m = _state["mode"]
    if m == "blas":
        return "blas"
    if m == "tb":
        return fill_choice(M, N)
    if not _state["loaded"]:
        load_table()          # keyed by (N, K, epilogue): shapes of other models simply miss it
    tab = _state["table"]
    if tab is not None:
        ent = tab.get((N, K, epi))
        if ent is not None:
            ms, cs = ent
            i = bisect.bisect_left(ms, M)
            return cs[min(i, len(cs) - 1)]
    return "blas"


def has_entry(N: int, K: int, epi: int, M: Optional[int] = None) -> bool:
    """Whether the loaded dispatch table measured ``(N, K, epi)`` (auto mode), up to row count ``M`` if given."""
    if _state["mode"] != "auto":
        return False
    if not _state["loaded"]:
        load_table()
    tab = _state["table"]
    if tab is None or (N, K, epi) not in tab:
        return False
    return M is None or M <= tab[(N, K, epi)][0][-1]


def describe() -> dict:
    return {"mode": _state["mode"], "kernel": _state["kernel"],
            "table": os.path.relpath(_state["table_path"], REPO) if _state["table_path"] else None}
