"""Per-shape GEMM selection between the in-tree MFMA kernels (four-wave, ring) and hipBLASLt.

Every plain projection of the Gemma-2 forward (QKV, o, gate|up, down, lm_head / lens unembedding) goes
through :func:`taboo_brittleness_amd.ops.linear`, which asks :func:`choose` for one of

* ``"g256"`` / ``"g128"`` — ``csrc/gemm4.hip``'s four-wave kernel (128x128 wave tiles) with 256- or 128-row output
  tiles (the 128-row tile doubles the workgroup count for the N = 3584 projections at moderate M), bit-identical; ``"gs"`` — the four-wave kernel with its tile height(s) from a rounds model
  of the persistent grid (:func:`split_rows`: 256-row tiles, 128-row tiles, or both as two launches split by rows);
* ``"k256"`` / ``"k128"`` — the four-wave kernel split over K (``tb_gemm4_splitk``: as many K ranges as fill the
  CUs, fp32 partials, ordered reduction) for thin grids (o_proj / down at N = 3584, every projection at decode M);
  deterministic but not bit-identical to the unsplit kernels, so ``auto`` only;
* ``"r<bm>x<bn>"`` / ``"r<bm>x<bn>b"`` / ``"r<bm>x<bn>c"`` — ``csrc/gemm_ring.hip``'s narrow-tile ring GEMM (bm x bn
  output tiles, a 64 KB or 144 KB LDS-DMA ring; ``c``: deeper stages for the small tiles): fills the chip at decode / mid row counts WITHOUT splitting K, bit-identical to the
  four-wave kernel at every M (batch-invariant);
* ``"blas"`` — ``torch.matmul`` (hipBLASLt, with the TunableOp solution table the bench loads).

Modes (``TB_GEMM``):

* ``tb`` (default) — in-tree batch-invariant kernels only (``g*``, ``gs``, ``r*``; never split-K or hipBLASLt), per row count the fastest of them as measured (the table's ``tb_shapes``; without one the fill
  heuristic).  All of them accumulate every output element over K in the same order with the same MFMA, so a row's
  result does not depend on M or on the tile choice: the whole forward is batch-invariant, which is what makes the
  sweep's reuse levels (shared prefixes, layer resume, ride-along baselines, trie decode) exact -- every cell's
  records equal a from-scratch generation of that cell (the GPU equivalence tests require bit-equal records).
* ``auto`` — the fastest of in-tree / split-K / hipBLASLt per ``(N, K, epilogue, M)`` as measured on an MI355X by
  ``tools/ring_bench.py`` / ``tools/gemm_dispatch_tune.py`` (``configs/gemm_dispatch/<arch>.json``); shapes the
  table does not cover use hipBLASLt.  NOT batch-invariant: a row's bf16 projections depend on the batch's row
  count, so reused and from-scratch results can differ in the last bits and then in greedy tokens
  (``tests/test_drift_gpu.py`` measures how often).
* ``blas`` — hipBLASLt only (the round-2 path).
"""
from __future__ import annotations

import bisect
import functools
import json
import os
from typing import Dict, List, Optional, Tuple, Union

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
TABLE_DIR = os.path.join(REPO, "configs", "gemm_dispatch")
NUM_CU = 256

Choice = Union[int, str]

_state = {"mode": os.environ.get("TB_GEMM", "tb"), "table": None, "tb_table": None, "table_path": None,
          "loaded": False}


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

    def parse(sec):
        tab: Dict[Tuple[int, int, int], Tuple[List[int], List[Choice]]] = {}
        for key, rows in raw.get(sec, {}).items():
            n, k, e = (int(v) for v in key.split(","))
            rows = sorted(rows, key=lambda r: r[0])
            tab[(n, k, e)] = ([int(r[0]) for r in rows], [r[1] if isinstance(r[1], str) else int(r[1]) for r in rows])
        return tab
    _state["table"], _state["tb_table"], _state["table_path"] = parse("shapes"), parse("tb_shapes") or None, path
    _state["loaded"] = True
    return path


def fill_choice(M: int, N: int) -> Choice:
    """Four-wave kernel tile rows without a measured entry: 256 unless the grid fills less than half the CUs (the
    128-row tile runs its MFMAs at ~0.78x the 256-row tile's rate, profiles/r4/gemm4/pmc_counted_waits_gate_up_4096.txt,
    so it only pays where it doubles a very thin grid)."""
    return "g128" if (N // 256) * (-(-M // 256)) < NUM_CU // 2 else "g256"


def choose(M: int, N: int, K: int, epi: int = 0) -> Choice:
    """``"g256"`` | ``"g128"`` | ``"gs"`` | ``"r<bm>x<bn>[b]"`` | ``"k256"`` | ``"k128"`` | ``"k64"`` | ``"blas"`` for
    ``C[M, N] = A[M, K] @ W[N, K]^T`` (epi 3: gate|up + GeGLU, 4: QKV + RoPE, 5: o / down + residual norm)."""
    m = _state["mode"]
    if m == "blas":
        return "blas"
    if not _state["loaded"]:
        load_table()          # keyed by (N, K, epilogue): shapes of other models simply miss it
    if m == "tb":
        ent = _tb_entry(N, K, epi)
        if ent is not None:
            ms, cs = ent
            return cs[min(bisect.bisect_left(ms, M), len(cs) - 1)]
        return fill_choice(M, N)
    tab = _state["table"]
    if tab is not None:
        ent = tab.get((N, K, epi))
        if ent is not None:
            ms, cs = ent
            i = bisect.bisect_left(ms, M)
            return cs[min(i, len(cs) - 1)]
    return "blas"


@functools.lru_cache(maxsize=1024)
def _tb_entry_cached(table_id: int, N: int, K: int, epi: int):
    tab = _state["tb_table"]
    if tab is None:
        return None
    for e in ((epi, 0) if epi in (4, 5) else (epi,)):
        if (N, K, e) in tab:
            return tab[(N, K, e)]
    # a LoRA-augmented projection (models/lora.py: the bank's up-projections appended to K) runs the base shape's
    # choices: the largest measured K below it with the same N (its extra K tiles are < 4 % of the work)
    for e in ((epi, 0) if epi in (4, 5) else (epi,)):
        ks = [k for (n, k, ee) in tab if n == N and ee == e and k < K]
        if ks:
            return tab[(N, max(ks), e)]
    return None


def _tb_entry(N: int, K: int, epi: int):
    return _tb_entry_cached(id(_state["tb_table"]), N, K, epi)


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


# time of a 128-row four-wave tile relative to a 256-row one (half the MFMAs at 0.538 vs 0.694 MFMA utilisation,
# profiles/r4/gemm4/pmc_counted_waits_gate_up_4096.txt)
G128_COST = 0.64


@functools.lru_cache(maxsize=4096)
def split_rows(M: int, N: int) -> int:
    """Row split of the ``"gs"`` choice: rows ``[0, M1)`` on 256-row tiles, the rest on 128-row tiles (two launches of
    the persistent four-wave kernel).  A persistent grid runs in rounds of one tile per CU, so a grid that does not
    divide into the CUs leaves its last round part-empty (e.g. o_proj at M = 6144: 14 x 24 = 336 tiles on 256 CUs);
    ``M1`` minimises the rounds-based cost ``ceil(tiles256 / CUs) + G128_COST * ceil(tiles128 / CUs)`` over the
    multiples of 256 (ties: more 256-row rows).  ``M1 = M``: plain 256-row tiles, ``0``: plain 128-row tiles.  The
    model picks the fastest of the three at 213 of 222 measured (shape, M) points above 2048 rows and is within 3 % at
    the rest (profiles/r5/gemm_dispatch/gs.jsonl).  Every tile height accumulates the same K chain, so the split keeps
    the GEMM batch-invariant."""
    nbn = max(1, N // 256)

    def cost(m1):
        c = -(-nbn * -(-m1 // 256) // NUM_CU) if m1 > 0 else 0
        return c + (G128_COST * -(-nbn * -(-(M - m1) // 128) // NUM_CU) if m1 < M else 0.0)
    cands = [min(256 * k, M) for k in range(-(-M // 256) + 1)]
    return min(cands, key=lambda m1: (cost(m1), -m1))


def is_invariant(choice: Choice) -> bool:
    """Whether a choice accumulates every output over K in the one order of the in-tree kernels (no split-K, no
    hipBLASLt): rows then get bit-identical results in any batch."""
    return isinstance(choice, str) and choice[:1] in ("g", "r")   # incl. "gs"


def ring_tile(choice: Choice) -> Optional[Tuple[int, int, int]]:
    """``(bm, bn, variant)`` of a ring-GEMM choice ``"r<bm>x<bn>"`` (variant 0, 64 KB ring) / ``"r<bm>x<bn>b"``
    (variant 1, 144 KB ring) / ``"r<bm>x<bn>c"`` (variant 2, 144 KB ring of 4-8 K tiles per stage, small tiles),
    else None."""
    if not (isinstance(choice, str) and choice[:1] == "r"):
        return None
    sfx = {"b": 1, "c": 2}.get(choice[-1], 0)
    body, var = (choice[1:-1], sfx) if sfx else (choice[1:], 0)
    bm, bn = body.split("x")
    return int(bm), int(bn), var


def describe() -> dict:
    return {"mode": _state["mode"],
            "table": os.path.relpath(_state["table_path"], REPO) if _state["table_path"] else None}
