"""Data parallelism over graphs: one process per GPU, bucketed gradient exchange.

The reference is single-device (`main.py:34` pins CUDA_VISIBLE_DEVICES=1;
there is no collective anywhere).  SURVEY.md §8e: graphs are independent, so
the batch is sharded contiguously over ranks; every loss term is a mean over
equal-size per-graph sets, hence the global gradient is the mean of the rank
gradients.  The exchange is a sum over ranks of the flat fp32 gradient buffer
with the loss terms appended; the 1/world scale is folded into the Adam kernel.
It runs in buckets (plan_buckets / run_buckets): a block whose gradient one
kernel completes early in the backward pass (the graph-latent head and
d_sg_lin1 weights, 216 MB at C4) starts its exchange on a communication stream
while the backward pass goes on, and large buckets are reduce-scattered, updated
as per-rank shards (1/world of the Adam traffic) and all-gathered; the rest (all
of C2's ~245 KB) is ONE all-reduce at the end of the step.  Frozen-stat BN needs
no cross-rank sync.  Backend "nccl" is RCCL over xGMI on MI355X; "gloo"
serves the CPU tests.
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


# buckets at least this many floats are reduce-scattered and updated as per-rank
# shards (ZeRO-1); smaller ones are all-reduced and updated on every rank
SHARD_MIN = 1 << 20


@dataclass
class Bucket:
    """A contiguous range [lo, hi) of the flat gradient / parameter buffer whose
    gradient is complete at one point of the step: `point` 0 = after the step's final
    reduction, k > 0 = the plan's k-th early point (snd_plan_grad_event)."""
    lo: int
    hi: int
    point: int
    sharded: bool

    def shard(self, world: int, rank: int):
        """[lo, lo + c) of this rank's chunk of a sharded bucket."""
        c = (self.hi - self.lo) // world
        return self.lo + rank * c, c


def plan_buckets(blocks, points, param_count: int, total: int, world: int,
                 shard_min: int = SHARD_MIN):
    """Buckets of the flat buffer [0, total) (parameters, then the loss tail).

    blocks: [(offset, padded_length)] in layout order (contiguous, lengths % 64 == 0);
    points[i]: completion point of block i.  A bucket is a maximal run of consecutive
    blocks with one point; a run of at least `shard_min` floats whose length splits
    into world 16-byte-aligned chunks is sharded.  The loss tail [param_count, total)
    joins the last run when that run is all-reduced, else it is a bucket of its own
    (every rank reads the summed loss terms).  Issue order: the early points in the
    order the step reaches them, then the end of the step."""
    runs = []
    for (off, n), pt in zip(blocks, points):
        if runs and runs[-1][2] == pt and runs[-1][1] == off:
            runs[-1][1] = off + n
        else:
            runs.append([off, off + n, pt])
    if not runs or runs[-1][1] != param_count:
        raise ValueError("plan_buckets: blocks do not tile [0, param_count)")
    out = []
    for lo, hi, pt in runs:
        n = hi - lo
        sharded = n >= shard_min and n % (4 * world) == 0
        out.append(Bucket(lo, hi, pt, sharded))
    last = out[-1]
    if total > param_count:
        if last.point == 0 and not last.sharded:
            last.hi = total
        else:
            out.append(Bucket(param_count, total, 0, False))
    out.sort(key=lambda b: (b.point == 0, b.point, b.lo))
    return out


def run_buckets(buckets, grads, params, param_count: int, world: int, rank: int, adam,
                shard_grads, reduce_scatter, all_gather, all_reduce, wait=None):
    """The data-parallel exchange + update of one step over `buckets`:

      sharded bucket:  reduce-scatter(sum) its gradient -> this rank's chunk,
                       adam(lo, n, chunk gradient) on the chunk's parameters,
                       all-gather the updated chunks (in place) into every rank;
      other bucket:    all-reduce(sum) its gradient, adam over its parameters.

    adam(lo, n, g, bucket) updates params/m/v[lo:lo+n] with gradient g (1/world folded
    in by the caller); shard_grads[i]: the chunk buffer of bucket i, or None for an
    in-place reduce-scatter into this rank's chunk of the gradient buffer (no copy,
    a no-op at world 1); wait(bucket) orders
    the bucket after its gradient is complete (the GPU path: a stream wait on the
    bucket's event).  The collectives are parameters so the same schedule runs on
    RCCL (product) and gloo (CPU tests)."""
    for i, b in enumerate(buckets):
        if wait is not None:
            wait(b)
        if b.sharded:
            lo, c = b.shard(world, rank)
            out = grads[lo:lo + c] if shard_grads is None else shard_grads[i]
            reduce_scatter(out, grads[b.lo:b.hi])
            n = max(0, min(lo + c, param_count) - lo)
            if n:
                adam(lo, n, out[:n], b)
            all_gather(params[b.lo:b.hi], params[lo:lo + c])
        else:
            all_reduce(grads[b.lo:b.hi])
            n = max(0, min(b.hi, param_count) - b.lo)
            if n:
                adam(b.lo, n, grads[b.lo:b.lo + n], b)


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
