"""Data parallelism over graphs: one process per GPU, one all-reduce per step.

The reference is single-device (`main.py:34` pins CUDA_VISIBLE_DEVICES=1;
there is no collective anywhere).  SURVEY.md §8e: graphs are independent, so
the batch is sharded contiguously over ranks; every loss term is a mean over
equal-size per-graph sets, hence the global gradient is the mean of the rank
gradients.  The exchange is ONE all-reduce(sum) of the flat fp32 gradient
buffer with the loss terms appended; the 1/world scale is folded into the
Adam kernel.  Frozen-stat BN needs no cross-rank sync.  Backend "nccl" is
RCCL over xGMI on MI355X; "gloo" serves the CPU tests.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import torch


@dataclass
class DistInfo:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    group: object = None


def init_from_env(backend: str = "nccl", force: bool = False) -> DistInfo:
    """torchrun-style init; single process when WORLD_SIZE is unset or 1, unless
    ``force`` (a torchrun world of 1: the N>1 code path, collectives included,
    rehearsed on one GPU)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1 and not (force and "RANK" in os.environ):
        return DistInfo()
    import torch.distributed as dist
    rank = int(os.environ["RANK"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if backend == "nccl":
        torch.cuda.set_device(local)
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    if not dist.is_initialized():
        dist.init_process_group(backend=backend, rank=rank, world_size=world,
                                device_id=torch.device("cuda", local) if backend == "nccl" else None)
    return DistInfo(rank, world, local, dist.group.WORLD)


def allreduce_mean_(flat: torch.Tensor, info: DistInfo) -> torch.Tensor:
    """In-place mean over ranks of a flat buffer (one collective)."""
    if info.world > 1:
        import torch.distributed as dist
        dist.all_reduce(flat, group=info.group)
        flat.div_(info.world)
    return flat


def max_over_ranks(x: float, info: DistInfo, device="cpu") -> float:
    if info.world <= 1:
        return x
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=info.group)
    return float(t.item())
