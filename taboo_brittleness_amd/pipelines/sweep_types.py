"""Data types and small helpers shared by the sweep modules (:mod:`.sweep`, :mod:`.sweep_plan`,
:mod:`.sweep_decode`, :mod:`.sweep_readout`): a (word, prompt) pair with its baseline artifacts, a cell (one
intervention setting), a decode-tail carry record, the prefetched next batch, pinned host -> device staging."""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional, Tuple

import numpy as np
import torch

METHODS = ("sae_targeted", "sae_random", "proj_targeted", "proj_random")


@dataclass
class Pair:
    word: str
    pidx: int
    prompt: str
    ids: List[int]
    forms: List[str]
    track: List[int]                       # [secret(space), secret(bare), decoys...]
    resp: List[int] = field(default_factory=list)
    p_secret: Optional[np.ndarray] = None  # [n_resp] lens prob of the secret (space form) at the hooked layer
    spikes_rel: List[int] = field(default_factory=list)
    top_ids: List[int] = field(default_factory=list)
    resid: Optional[torch.Tensor] = None   # [n_resp, D] hooked-layer residuals (device)
    nll: float = float("nan")
    targeted: List[int] = field(default_factory=list)
    active_pool: np.ndarray = field(default_factory=lambda: np.zeros(0, dtype=np.int64))  # sorted, unique
    gen_toks: List[int] = field(default_factory=list)   # generated tokens incl. the stop token (if any)
    tok_nll: Optional[np.ndarray] = None                # per generated token NLL under the unedited model
    kv_slot: int = -1                                   # slot in the runner's pair-KV store
    lens_cum: Optional[torch.Tensor] = None             # [n_resp + 1, V] running lens sums (layer resume)
    track_probs: Optional[np.ndarray] = None            # [n_resp, K] lens probs of the tracked ids
    leak: Optional[bool] = None                         # baseline response contains the secret (cached)
    p_secret_mean: Optional[float] = None               # cached mean of p_secret (result records)
    forms_l: Optional[set] = None
    rep: int = 0                                        # replicate of this (word, prompt): seeds its random cells
    # exact per-latent activity at the edited spikes (SweepRunner._spike_activity): sorted candidate latent
    # ids and, per id, a bitmask over spikes_rel[:K] of where the edit kernel's own JumpReLU fires
    act_ids: Optional[np.ndarray] = None
    act_mask: Optional[np.ndarray] = None
    act_key: Optional[tuple] = None                     # SAE parameter identity/versions the table was built with

    @property
    def first_edit(self) -> int:
        """Response index of the first edited position (last token if there is nothing to edit)."""
        if self.spikes_rel:
            return min(self.spikes_rel)
        return max(len(self.resp) - 1, 0)

    @property
    def plen(self) -> int:
        return len(self.ids)

    @property
    def spikes_abs(self) -> List[int]:
        return [self.plen + i for i in self.spikes_rel]


@dataclass
class Cell:
    pair: int
    method: str
    budget: int
    trial: int
    seed: int

    @property
    def kind(self) -> str:
        return "sae" if self.method.startswith("sae") else "proj"


@dataclass
class _Carry:
    """A diverged cell whose decode continues in the next batch (decode-tail carry-over): its KV,
    capture-store row and edit-plan row live in the runner's carry region at ``slot``."""
    cell: Cell
    pair: Pair
    d: int                       # divergence point D
    nll: float                   # teacher-forced edit NLL of the baseline hint (already complete)
    slot: int
    tok: int                     # next token to feed, at position ``pos``
    pos: int
    prefix: List[int]            # response tokens so far (ends with ``tok``)
    prefix_nll: np.ndarray       # their NLLs
    steps: int                   # decode steps still needed
    pre: Tuple[int, int, int]    # (pair KV slot, len_lo, len_hi) of the shared prefix
    plan_row: Tuple[np.ndarray, int, np.ndarray, int]   # host (spikes, kind, idx, cnt) of the slot


class NextBatch:
    """The next :meth:`SweepRunner.run_cells` batch, for :meth:`SweepRunner.stage_next`: its pairs, and
    either its ``(cells, plan)`` prefetch future, or ``cells`` (``plan`` built when staged).  Run the
    next call with ``nb.cells`` (the same list object) so the staged work is used."""

    def __init__(self, pairs, methods=METHODS, cells=None, plan=None, future=None):
        self.pairs, self.methods, self.cells, self.plan, self.future = pairs, methods, cells, plan, future

    def resolve(self, runner) -> None:
        if self.future is not None:
            self.cells, self.plan = self.future.result()
            self.future = None
        if self.cells is None:
            self.cells = runner.make_cells(self.pairs, self.methods)


def _h2d(a, dev):
    """Host array -> pinned CPU tensor for a non-blocking upload (plain tensor on CPU devices)."""
    t = a if isinstance(a, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(a))
    return t.pin_memory() if dev.type == "cuda" else t


class _Deferred:
    """Result records of :meth:`SweepRunner.run_cells_async` (lists and/or futures, in cell order)."""

    def __init__(self, parts):
        self.parts = parts

    def result(self) -> List[dict]:
        out: List[dict] = []
        for p in self.parts:
            out += p.result() if hasattr(p, "result") else p
        return out


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False
