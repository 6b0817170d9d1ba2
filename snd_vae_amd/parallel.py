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


# ---------------------------------------------------------------- row sharding (§8e)
# One graph too large for one device's step (C5: N = 16384, 2.7e8 logits) split by
# ROWS over the ranks instead of by graphs.  zz^T: every rank owns a contiguous
# 128-row-aligned row range, all-gathers z once, evaluates its rows against every
# column (snd_zzt_ce_rows) and keeps its dz rows -- L is symmetric, so dz needs no
# reduction; only the two loss scalars are all-reduced.  Encoder SpMM: under the
# RCM row order every neighbour of a row lies within +-beta rows, so a rank needs
# only a halo of beta rows from each neighbouring range (halo_rows).

def row_ranges(n: int, world: int, block: int = 128):
    """Contiguous row ranges of one n-row graph over `world` ranks, cut on `block`-row
    boundaries (the zz^T kernel's row blocks); the last range ends at n."""
    nb = -(-n // block)
    out = []
    for r in range(world):
        b0, b1 = r * nb // world, (r + 1) * nb // world
        out.append((min(n, b0 * block), min(n, b1 * block)))
    return out


def allgather_rows(x_local: torch.Tensor, ranges, group) -> torch.Tensor:
    """The whole [n, ...] matrix from every rank's contiguous row range (ranges may
    differ in size by a block: shards are padded to the largest for the collective)."""
    import torch.distributed as dist
    world = len(ranges)
    rmax = max(r1 - r0 for r0, r1 in ranges)
    pad = torch.zeros((rmax,) + tuple(x_local.shape[1:]), dtype=x_local.dtype, device=x_local.device)
    pad[:x_local.shape[0]] = x_local
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad, group=group)
    return torch.cat([parts[r][:r1 - r0] for r, (r0, r1) in enumerate(ranges)])


def reducescatter_rows(x_full: torch.Tensor, ranges, group) -> torch.Tensor:
    """Sum over ranks of x_full [n, ...], returned as THIS rank's rows of its contiguous
    range: one reduce-scatter over the ranges padded to the largest (allgather_rows'
    layout), so each rank receives only its own rows instead of all n."""
    import torch.distributed as dist
    world = len(ranges)
    rmax = max(r1 - r0 for r0, r1 in ranges)
    tail = tuple(x_full.shape[1:])
    inp = torch.zeros((world * rmax,) + tail, dtype=x_full.dtype, device=x_full.device)
    for r, (r0, r1) in enumerate(ranges):
        inp[r * rmax:r * rmax + (r1 - r0)] = x_full[r0:r1]
    out = torch.empty((rmax,) + tail, dtype=x_full.dtype, device=x_full.device)
    dist.reduce_scatter_tensor(out, inp, group=group)
    r0, r1 = ranges[dist.get_rank(group)]
    return out[:r1 - r0].contiguous()


def halo_rows(x_local: torch.Tensor, ranges, rank: int, halo: int, group) -> torch.Tensor:
    """Rows [row0 - halo, row1 + halo) clipped to [0, n) of a contiguously row-sharded
    matrix, on this rank: its own rows plus `halo` boundary rows from each side
    (every rank contributes its first and last `halo` rows to one all-gather)."""
    import torch.distributed as dist
    world = len(ranges)
    h = halo
    rows = x_local.shape[0]
    tail = tuple(x_local.shape[1:])
    edge = torch.zeros((2, h) + tail, dtype=x_local.dtype, device=x_local.device)
    k = min(h, rows)
    edge[0, :k] = x_local[:k]                # first rows (the lower neighbour's upper halo)
    edge[1, h - k:] = x_local[rows - k:]     # last rows, right-aligned
    parts = [torch.empty_like(edge) for _ in range(world)]
    dist.all_gather(parts, edge, group=group)
    r0, r1 = ranges[rank]
    lo = max(0, r0 - h)
    hi = min(ranges[-1][1], r1 + h)
    below = parts[rank - 1][1][h - (r0 - lo):] if rank > 0 and r0 > lo else x_local[:0]
    above = parts[rank + 1][0][:hi - r1] if rank + 1 < world and hi > r1 else x_local[:0]
    if rank > 0 and (r0 - lo) > ranges[rank - 1][1] - ranges[rank - 1][0]:
        raise ValueError("halo wider than the neighbouring range")
    if rank + 1 < world and (hi - r1) > ranges[rank + 1][1] - ranges[rank + 1][0]:
        raise ValueError("halo wider than the neighbouring range")
    return torch.cat([below, x_local, above]), lo


def row_sharded_adj_ce(z_local: torch.Tensor, ranges, rank: int, rowptr, colidx, group,
                       compute=None, **kw):
    """The structure decoder's CE (layers.py:407-409, optimizer.py:142-144) of ONE
    graph row-sharded over the ranks: all-gather z, this rank's rows against every
    column, all-reduce (sum) of [ce_sum, n_correct].  rowptr/colidx: this rank's
    rows of the graph's CSR (global column ids).  Returns (stats, dz_rows) with
    stats the global [ce_sum, n_correct] and dz_rows this rank's rows of d ce_sum/dz.
    compute(z_full, row0, row1, rowptr, colidx, **kw) -> (stats, dz_rows) defaults to
    the HIP kernel (layers.inner_product_ce_rows)."""
    import torch.distributed as dist
    if compute is None:
        from .layers import inner_product_ce_rows as compute
    z_full = allgather_rows(z_local, ranges, group)
    r0, r1 = ranges[rank]
    stats, dz = compute(z_full, r0, r1, rowptr, colidx, **kw)
    dist.all_reduce(stats, group=group)
    return stats, dz
