"""One-shot peer-to-peer all-reduce over xGMI (``csrc/p2p.hip``).

TP's all-reduces are small (2 × ``[M, 3584]`` bf16 per block), so they are latency-bound.  On the
MI355X's point-to-point xGMI fabric every GPU is one hop from each of its 7 peers; a ring pays
2(N-1) dependent hops over one link each, a one-shot reduce pays one: every rank stages its input in
an IPC-exported region, a barrier of release/acquire flags says "all staged", and each rank reads
the N inputs straight out of the peers' HBM (N-1 links in parallel) and sums them in rank order —
the result is bit-identical on every rank, which TP's replicated readouts rely on.

The IPC handles are exchanged once through the process group (RCCL or gloo); afterwards no
collective library is involved.  Messages larger than the staging area fall back to RCCL.

The reference has no collectives at all (SURVEY §2.4 "Collective / NCCL call sites: none").
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.distributed as dist


def _ext():
    from ..ops._ext import kernels

    return kernels()


class P2PAllReduce:
    """Per-process state of the one-shot all-reduce for one (TP) group.

    ``max_bytes`` sizes each rank's staging area (a decode step of a few hundred rows is ≈1-3 MB;
    prefill chunks above the size use RCCL).  ``blocks`` workgroups each own a grid-stride share of
    16-byte vectors and a private pair of barrier slots; ``spin_max`` bounds every wait (a missing
    peer sets the error word instead of hanging the GPU — :meth:`check` raises on it).
    """

    def __init__(self, group=None, device: Optional[torch.device] = None, max_bytes: int = 8 << 20,
                 blocks: int = 64, spin_max: int = 1 << 22, uncached: bool = True):
        ext = _ext()
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        if self.world > int(ext.p2p_max_ranks()):
            raise ValueError(f"p2p all-reduce supports at most {ext.p2p_max_ranks()} ranks")
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        self.max_bytes = int(max_bytes)
        self.blocks = int(blocks)
        self.spin_max = int(spin_max)
        with torch.cuda.device(self.device):
            self.own = int(ext.p2p_alloc(int(ext.p2p_header_bytes()) + self.max_bytes, uncached))
            handle = ext.p2p_get_handle(self.own)
        handles: List[bytes] = [b""] * self.world
        if self.world > 1:
            dist.all_gather_object(handles, handle, group=group)
        else:
            handles = [handle]
        self.opened: List[int] = []
        bases = []
        with torch.cuda.device(self.device):
            for r, h in enumerate(handles):
                if r == self.rank:
                    bases.append(self.own)
                else:
                    p = int(ext.p2p_open_handle(h))
                    self.opened.append(p)
                    bases.append(p)
        self.bases = bases
        self.calls = 0
        self.fallbacks = 0
        # persistent zero-padded staging views for small messages, one per (op, dtype, padded size): allocated once
        # (also inside a captured decode graph the same buffers are replayed), never per call
        self._stage: dict = {}

    @staticmethod
    def _align_bytes(dtype) -> int:
        """The kernel's vector size per dtype: 16 B of bf16, 32 B of fp32 (csrc/p2p.hip)."""
        return 16 if dtype == torch.bfloat16 else 32

    def supports(self, t: torch.Tensor) -> bool:
        nbytes = t.numel() * t.element_size()
        return (t.is_cuda and t.dtype in (torch.bfloat16, torch.float32) and nbytes <= self.max_bytes
                and nbytes % self._align_bytes(t.dtype) == 0 and t.is_contiguous())

    def _staging(self, key, shape, dtype, device) -> torch.Tensor:
        b = self._stage.get(key)
        if b is None:
            b = self._stage[key] = torch.zeros(shape, dtype=dtype, device=device)
        return b

    def all_reduce_(self, t: torch.Tensor) -> torch.Tensor:
        """In-place sum over the group (stream-ordered on the current stream).  A small message whose size is not
        a multiple of the kernel's vector is zero-padded (exact: x + 0 = x)."""
        if self.world == 1:
            return t
        if not self.supports(t):
            n = t.numel()
            align = self._align_bytes(t.dtype) // t.element_size()     # elements per kernel vector
            npad = -(-n // align) * align
            if (t.is_cuda and t.dtype in (torch.bfloat16, torch.float32) and npad != n
                    and npad * t.element_size() <= self.max_bytes):
                buf = self._staging(("ar", t.dtype, npad), (npad,), t.dtype, t.device)   # tail stays zero
                buf[:n].copy_(t.reshape(-1))
                _ext().p2p_allreduce(self.bases, self.rank, buf, buf, self.blocks, self.spin_max, True)
                self.calls += 1
                t.copy_(buf[:n].view_as(t))
                return t
            self.fallbacks += 1
            dist.all_reduce(t, group=self.group)
            return t
        _ext().p2p_allreduce(self.bases, self.rank, t, t, self.blocks, self.spin_max, True)
        self.calls += 1
        return t

    def all_gather(self, t: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """``[world, *t.shape]`` of every rank's ``t`` in rank order (stream-ordered, capturable; any dtype whose
        byte size is a multiple of 16; larger messages than the staging area go through RCCL)."""
        out = out if out is not None else torch.empty((self.world,) + tuple(t.shape), dtype=t.dtype, device=t.device)
        if self.world == 1:
            out[0].copy_(t)
            return out
        nbytes = t.numel() * t.element_size()
        pad = -(-nbytes // 16) * 16
        if not (t.is_cuda and pad <= self.max_bytes):
            self.fallbacks += 1
            dist.all_gather_into_tensor(out, t.contiguous(), group=self.group)
            return out
        if pad != nbytes:       # a small message padded to the kernel's 16-byte vectors
            src = self._staging(("ag", pad), (pad,), torch.uint8, t.device)             # tail stays zero
            src[:nbytes].copy_(t.contiguous().view(-1).view(torch.uint8))
            g = self._staging(("agout", pad), (self.world, pad), torch.uint8, t.device)
            _ext().p2p_allgather(self.bases, self.rank, src, g, self.blocks, self.spin_max, True)
            out.view(self.world, -1).view(torch.uint8).copy_(g[:, :nbytes])
        else:
            _ext().p2p_allgather(self.bases, self.rank, t.contiguous(), out, self.blocks, self.spin_max, True)
        self.calls += 1
        return out

    def check(self) -> None:
        """Raise if any barrier wait of this rank timed out since the last check (synchronises)."""
        torch.cuda.synchronize(self.device)
        err = int(_ext().p2p_read_error(self.own))
        if err:
            raise RuntimeError(f"p2p all-reduce rank {self.rank}: barrier timed out waiting for ranks "
                               f"{[r for r in range(32) if err >> r & 1]}")

    def close(self) -> None:
        if not self.bases:
            return
        ext = _ext()
        torch.cuda.synchronize(self.device)
        for p in self.opened:
            ext.p2p_close_handle(p)
        ext.p2p_free(self.own)
        self.bases, self.opened = [], []


def reduce_local(inputs: List[torch.Tensor], blocks: int = 64) -> torch.Tensor:
    """Single-process check of the reduction math: ``inputs`` (same shape, on one GPU) are staged into
    per-"rank" regions and summed by the kernel with its barriers off.  Returns rank 0's output."""
    ext = _ext()
    n = len(inputs)
    nbytes = inputs[0].numel() * inputs[0].element_size()
    hdr = int(ext.p2p_header_bytes())
    bases = [int(ext.p2p_alloc(hdr + nbytes, True)) for _ in range(n)]
    try:
        out = torch.empty_like(inputs[0])
        for r, x in enumerate(inputs):
            # stage rank r's input: its own call with barriers off writes the staging area (the output
            # of these calls is discarded; only the final rank-0 call below is returned)
            ext.p2p_allreduce(bases[:r + 1], r, x.contiguous(), torch.empty_like(x), blocks, 1, False)
        ext.p2p_allreduce(bases, 0, inputs[0].contiguous(), out, blocks, 1, False)
        torch.cuda.synchronize()
        return out
    finally:
        for b in bases:
            ext.p2p_free(b)


def gather_local(inputs: List[torch.Tensor], blocks: int = 64) -> torch.Tensor:
    """Single-process check of the all-gather kernel (as :func:`reduce_local`): ``inputs`` staged into per-"rank"
    regions of one GPU with barriers off, then gathered by "rank" 0.  Returns ``[len(inputs), *shape]``."""
    ext = _ext()
    n = len(inputs)
    nbytes = inputs[0].numel() * inputs[0].element_size()
    hdr = int(ext.p2p_header_bytes())
    bases = [int(ext.p2p_alloc(hdr + nbytes, True)) for _ in range(n)]
    try:
        for r, x in enumerate(inputs):
            scratch = torch.empty((r + 1,) + tuple(x.shape), dtype=x.dtype, device=x.device)
            ext.p2p_allgather(bases[:r + 1], r, x.contiguous(), scratch, blocks, 1, False)
        out = torch.empty((n,) + tuple(inputs[0].shape), dtype=inputs[0].dtype, device=inputs[0].device)
        ext.p2p_allgather(bases, 0, inputs[0].contiguous(), out, blocks, 1, False)
        torch.cuda.synchronize()
        return out
    finally:
        for b in bases:
            ext.p2p_free(b)
