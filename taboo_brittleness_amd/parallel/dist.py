"""Process groups and data-parallel helpers.

One process per GPU; ``torch.distributed`` with the ``nccl`` backend, which is
RCCL over xGMI on ROCm, or ``gloo`` on CPU.  The sweep is embarrassingly
parallel: ranks own whole (word, prompt) pairs (``pipelines.run_sweep.pair_owners``)
and only small result records (and, for pooled PCA, spike residuals) cross
ranks, so collectives are latency-bound all-gathers issued once per sweep stage.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import Any, List, Optional, Sequence

import torch
import torch.distributed as dist


@dataclass
class DistInfo:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    backend: str = "none"
    device: torch.device = torch.device("cpu")

    @property
    def is_main(self) -> bool:
        return self.rank == 0


def init_distributed(backend: str = "auto", device: str = "auto", timeout_s: int = 1800) -> DistInfo:
    """Initialise from torchrun env vars (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_ADDR/PORT)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    use_gpu = (device in ("auto", "cuda")) and torch.cuda.is_available()
    shared = False
    if use_gpu:
        # more local ranks than GPUs (e.g. a 2-rank rehearsal on a 1-GPU box): ranks share devices round-robin.
        # RCCL needs one GPU per rank, so shared devices take gloo collectives (CPU staging of device tensors)
        n_dev = torch.cuda.device_count()
        shared = int(os.environ.get("LOCAL_WORLD_SIZE", world)) > n_dev
        dev = torch.device(f"cuda:{local % n_dev}")
        torch.cuda.set_device(dev)
    else:
        dev = torch.device("cpu")
    be = "none"
    if world > 1:
        be = ("gloo" if shared or not use_gpu else "nccl") if backend == "auto" else backend
        if be == "nccl" and shared:
            raise RuntimeError(f"{world} local ranks on {torch.cuda.device_count()} GPU(s): RCCL needs one GPU per "
                               "rank; use the gloo backend to rehearse more ranks than GPUs")
        if not dist.is_initialized():
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            kw = dict(backend=be, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=timeout_s))
            if be == "nccl":
                kw["device_id"] = dev
            dist.init_process_group(**kw)
    return DistInfo(rank, world, local, be, dev)


def shard(items: Sequence[Any], rank: int, world: int) -> List[Any]:
    return list(items[rank::world])


def barrier(info: DistInfo) -> None:
    if info.world > 1 and dist.is_initialized():
        if info.backend == "nccl":
            dist.barrier(device_ids=[info.local_rank])
        else:
            dist.barrier()


def all_gather_objects(obj: Any, info: DistInfo) -> List[Any]:
    if info.world <= 1 or not dist.is_initialized():
        return [obj]
    out: List[Any] = [None] * info.world
    dist.all_gather_object(out, obj)
    return out


def all_reduce_max(x: float, info: DistInfo) -> float:
    if info.world <= 1 or not dist.is_initialized():
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=info.device if info.backend == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def all_gather_tensor(x: torch.Tensor, info: DistInfo) -> torch.Tensor:
    """Same-shape all-gather into one ``[world * n, ...]`` tensor (one RCCL all-gather over xGMI on GPU;
    gloo on CPU)."""
    if info.world <= 1 or not dist.is_initialized():
        return x
    if _host_staged(x, info):
        return all_gather_tensor(x.cpu(), info).to(x.device)
    out = torch.empty((info.world * x.shape[0],) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    dist.all_gather_into_tensor(out, x.contiguous())
    return out


def _host_staged(x: torch.Tensor, info: DistInfo) -> bool:
    """Device tensors under gloo (ranks sharing a GPU, CPU tests) go through host copies."""
    return x.is_cuda and info.backend != "nccl"


def all_gather_tensor_async(x: torch.Tensor, info: DistInfo):
    """:func:`all_gather_tensor` issued asynchronously: returns ``(out, work)``; ``work.wait()`` (or
    ``None`` on one rank) before reading ``out``.  On RCCL the collective runs on the process group's own
    stream, so the compute stream does not wait for it (and ranks do not lock-step on it)."""
    if info.world <= 1 or not dist.is_initialized():
        return x, None
    if _host_staged(x, info):            # gloo: synchronous host all-gather (rehearsal path, not the RCCL one)
        return all_gather_tensor(x, info), None
    out = torch.empty((info.world * x.shape[0],) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    work = dist.all_gather_into_tensor(out, x.contiguous(), async_op=True)
    return out, work


def all_gather_rows(x: torch.Tensor, info: DistInfo) -> torch.Tensor:
    """Variable-length row all-gather (e.g. spike residuals for pooled PCA): pad, gather, trim."""
    if info.world <= 1 or not dist.is_initialized():
        return x
    if _host_staged(x, info):
        return all_gather_rows(x.cpu(), info).to(x.device)
    n = torch.tensor([x.shape[0]], device=x.device)
    ns = [torch.zeros_like(n) for _ in range(info.world)]
    dist.all_gather(ns, n)
    mx = int(max(int(v) for v in ns))
    pad = torch.zeros((mx,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    pad[: x.shape[0]] = x
    bufs = [torch.zeros_like(pad) for _ in range(info.world)]
    dist.all_gather(bufs, pad)
    return torch.cat([b[: int(k)] for b, k in zip(bufs, ns)], 0)


def destroy(info: DistInfo) -> None:
    if info.world > 1 and dist.is_initialized():
        dist.destroy_process_group()
