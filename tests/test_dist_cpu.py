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
