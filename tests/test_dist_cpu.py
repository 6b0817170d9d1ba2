"""Data-parallel correctness on CPU (gloo, world_size 2).

SURVEY.md §8e: the global batch is sharded contiguously over ranks, each rank
computes the mean-loss gradient of its shard, and ONE all-reduce (mean) of the
flat gradient buffer gives the full-batch gradient.  Here every rank computes
its shard's gradient with the oracle (float64), packs it into the product's
flat layout, and the product's all-reduce helper combines them; the result
must equal the single-process gradient of the whole batch.

Noise is drawn the way the product draws it: each rank takes the device Philox
stream from its first global head row on (oracle/ref_rng.py, the restatement of
snd_common.hpp's generator; snd_plan_set_rng_offset), never a slice of a
global array, so the test fails if shards share or misplace their normals.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import ref_numpy as R
from oracle import ref_rng
from snd_vae_amd.config import tscale
from snd_vae_amd.data import shard, synthetic_batch
from snd_vae_amd.params import flat_layout, init_blocks


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


SEED, STEP = 1234, 3


def _case():
    cfg = tscale(30, 8, mean_degree=5.0)
    batch = synthetic_batch(cfg, 4, seed=2)
    p = init_blocks(cfg, 3)
    return cfg, batch, p


def _grads(cfg, b, p, eps):
    adj = [b.dense_adj(i) for i in range(b.n_graphs)]
    losses, g, _ = R.forward_backward(p, adj, b.features, b.feature_truth, b.spatial_truth, eps, cfg)
    return losses, g


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from snd_vae_amd.parallel import allreduce_mean_, init_from_env, max_over_ranks
    info = init_from_env("gloo")
    cfg, batch, p = _case()
    part = shard(batch, rank, world)
    rows = part.features.shape[0]
    eps = ref_rng.eps(SEED, STEP, rows, cfg.latent, row0=rank * rows)   # this rank's own draw
    losses, g = _grads(cfg, part, p, eps)
    lay = flat_layout(cfg)
    flat = torch.from_numpy(np.concatenate([lay.pack(g, np.float64), [losses["cost"]]]))
    allreduce_mean_(flat, info)
    mx = max_over_ranks(float(rank + 1), info)
    if rank == 0:
        out.put((flat.numpy(), mx))
    eps_all = [torch.zeros(rows, cfg.latent, dtype=torch.float64) for _ in range(world)]
    dist.all_gather(eps_all, torch.from_numpy(eps))
    if rank == 0:
        out.put(torch.cat(eps_all).numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_dp_allreduce_equals_full_batch_gradient():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    flat, mx = q.get(timeout=180)
    eps_shards = q.get(timeout=60)
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    cfg, batch, p = _case()
    eps = ref_rng.eps(SEED, STEP, batch.features.shape[0], cfg.latent)    # one device, whole batch
    assert np.array_equal(eps_shards, eps)       # shards draw disjoint, correctly placed normals
    losses, g = _grads(cfg, batch, p, eps)
    lay = flat_layout(cfg)
    ref = lay.pack(g, np.float64)
    assert np.allclose(flat[:-1], ref, rtol=1e-12, atol=1e-15)
    assert flat[-1] == pytest.approx(losses["cost"], rel=1e-12)   # mean of shard means
    assert mx == 2.0


def _force_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from snd_vae_amd.parallel import init_from_env, max_over_ranks
    info = init_from_env("gloo", force=True)
    t = max_over_ranks(1.5 + rank, info)
    flat = torch.full((4,), float(rank + 1))
    dist.all_reduce(flat, group=info.group)
    q.put((info.world, info.group is not None, t, flat.tolist()))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [1, 2])
def test_force_dist_init(world):
    """bench.py --force-dist: under a torchrun environment even a world of 1
    initialises the process group, so the collective code path (all-reduce,
    max-over-ranks timing) runs on one device; without force a world of 1 stays
    single-process."""
    from snd_vae_amd.parallel import init_from_env
    old = {k: os.environ.get(k) for k in ("RANK", "WORLD_SIZE")}
    os.environ.pop("RANK", None)
    os.environ["WORLD_SIZE"] = "1"
    try:
        assert init_from_env("gloo", force=True).group is None        # no torchrun env: no group
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_force_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for w, has_group, t, flat in res:
        assert w == world and has_group
        assert t == 1.5 + (world - 1)
        assert flat == [world * (world + 1) / 2] * 4


# ---------------------------------------------------------------- bucketed exchange
def _adam_tf1(p, m, v, g, t, lr=1e-3, b1=0.9, b2=0.999, eps=1e-8, scale=1.0):
    """TF1 Adam in float32 torch ops, the snd_adam_tf1 formula (optimizer.py:125,197)."""
    lrt = lr * np.sqrt(1.0 - b2 ** t) / (1.0 - b1 ** t)
    gc = g * scale
    m.mul_(b1).add_((1.0 - b1) * gc)
    v.mul_(b2).add_((1.0 - b2) * gc * gc)
    p.sub_(np.float32(lrt) * m / (v.sqrt() + eps))


def _bucket_case(world):
    """A flat layout with a d_sg_lin1-like early pair (point 1), a head-like early
    block (point 2) and small end-of-step blocks between them, plus the loss tail."""
    from snd_vae_amd.parallel import plan_buckets
    lens = [64, 128, 4096, 64, 192, 2048, 64, 128]
    pts = [0, 0, 2, 0, 0, 1, 1, 0]
    offs = np.cumsum([0] + lens[:-1]).tolist()
    P = sum(lens)
    return P, plan_buckets(list(zip(offs, lens)), pts, P, P + 8, world, shard_min=1024)


def _bucket_worker(rank, world, port, q, inplace):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from snd_vae_amd.parallel import init_from_env, run_buckets
    info = init_from_env("gloo")
    P, buckets = _bucket_case(world)
    gen = torch.Generator().manual_seed(7)
    params = torch.randn(P + 8, generator=gen)            # the same initial state on every rank
    m = torch.randn(P + 8, generator=gen).abs() * 1e-3
    v = torch.randn(P + 8, generator=gen).abs() * 1e-6
    grads = torch.randn(P + 8, generator=torch.Generator().manual_seed(100 + rank))
    g0 = grads.clone()
    shard_grads = [torch.empty((b.hi - b.lo) // world if b.sharded else 0) for b in buckets]
    order = []

    def adam(off, n, g, b):
        _adam_tf1(params[off:off + n], m[off:off + n], v[off:off + n], g, t=3, scale=1.0 / world)

    run_buckets(buckets, grads, params, P, world, rank, adam, shard_grads if inplace is False else None,
                lambda out, inp: dist.reduce_scatter_tensor(out, inp, group=info.group),
                lambda out, inp: dist.all_gather_into_tensor(out, inp, group=info.group),
                lambda t: dist.all_reduce(t, group=info.group), wait=lambda b: order.append(b.point))
    # the sharded buckets' moments are current on the owner's chunk only: gather them
    for b in buckets:
        if b.sharded:
            lo, c = b.shard(world, rank)
            for t in (m, v):
                dist.all_gather_into_tensor(t[b.lo:b.hi], t[lo:lo + c].clone(), group=info.group)
    q.put((rank, g0.numpy(), params[:P].numpy(), m[:P].numpy(), v[:P].numpy(),
           grads[P:].numpy(), order))
    dist.barrier()
    dist.destroy_process_group()


def test_bucket_plan_shapes():
    """Early points first (in the order the step reaches them), runs of one point
    merged, large runs sharded, the loss tail on an all-reduced bucket."""
    P, bk = _bucket_case(2)
    got = [(b.lo, b.hi, b.point, b.sharded) for b in bk]
    assert got == [(4544, 6656, 1, True), (192, 4288, 2, True), (0, 192, 0, False),
                   (4288, 4544, 0, False), (6656, P + 8, 0, False)]
    # a model without early points or large blocks (C2): one all-reduce of everything
    from snd_vae_amd.parallel import plan_buckets
    one = plan_buckets([(0, 64), (64, 128)], [0, 0], 192, 200, 8)
    assert [(b.lo, b.hi, b.point, b.sharded) for b in one] == [(0, 200, 0, False)]


@pytest.mark.parametrize("world,inplace", [(2, True), (2, False)])
def test_bucketed_exchange_equals_allreduce_adam(world, inplace):
    """parallel.run_buckets (reduce-scatter + per-rank shard Adam + all-gather for
    large buckets, all-reduce + Adam for the rest, the order OptimizerVAE issues them)
    gives every rank exactly the parameters of one all-reduce of the whole gradient
    followed by one Adam pass, and the summed loss tail."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bucket_worker, args=(r, world, port, q, inplace)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = sorted([q.get(timeout=180) for _ in range(world)], key=lambda x: x[0])
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    P, buckets = _bucket_case(world)
    gsum = sum(torch.from_numpy(r[1]) for r in res)
    gen = torch.Generator().manual_seed(7)
    params = torch.randn(P + 8, generator=gen)
    m = torch.randn(P + 8, generator=gen).abs() * 1e-3
    v = torch.randn(P + 8, generator=gen).abs() * 1e-6
    _adam_tf1(params[:P], m[:P], v[:P], gsum[:P], t=3, scale=1.0 / world)
    for r in res:
        assert np.array_equal(r[2], params[:P].numpy())
        assert np.array_equal(r[3], m[:P].numpy())
        assert np.array_equal(r[4], v[:P].numpy())
        assert np.array_equal(r[5], gsum[P:].numpy())       # loss terms summed everywhere
        assert len(r[6]) == len(buckets)
        assert r[6] == [b.point for b in buckets] == [1, 2, 0, 0, 0]
