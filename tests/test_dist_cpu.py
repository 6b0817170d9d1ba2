"""Data-parallel correctness on CPU (gloo, world_size 2).

SURVEY.md §8e: the global batch is sharded contiguously over ranks, each rank
computes the mean-loss gradient of its shard, and ONE all-reduce (mean) of the
flat gradient buffer gives the full-batch gradient.  Here every rank computes
its shard's gradient with the oracle (float64), packs it into the product's
flat layout, and the product's all-reduce helper combines them; the result
must equal the single-process gradient of the whole batch.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import ref_numpy as R
from snd_vae_amd.config import tscale
from snd_vae_amd.data import shard, synthetic_batch
from snd_vae_amd.params import flat_layout, init_blocks


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _case():
    cfg = tscale(30, 8, mean_degree=5.0)
    batch = synthetic_batch(cfg, 4, seed=2)
    p = init_blocks(cfg, 3)
    eps = np.random.default_rng(4).standard_normal((batch.features.shape[0], cfg.latent))
    return cfg, batch, p, eps


def _grads(cfg, b, p, eps):
    adj = [b.dense_adj(i) for i in range(b.n_graphs)]
    losses, g, _ = R.forward_backward(p, adj, b.features, b.feature_truth, b.spatial_truth, eps, cfg)
    return losses, g


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from snd_vae_amd.parallel import allreduce_mean_, init_from_env, max_over_ranks
    info = init_from_env("gloo")
    cfg, batch, p, eps = _case()
    part = shard(batch, rank, world)
    rows = part.features.shape[0]
    losses, g = _grads(cfg, part, p, eps[rank * rows:(rank + 1) * rows])
    lay = flat_layout(cfg)
    flat = torch.from_numpy(np.concatenate([lay.pack(g, np.float64), [losses["cost"]]]))
    allreduce_mean_(flat, info)
    mx = max_over_ranks(float(rank + 1), info)
    if rank == 0:
        out.put((flat.numpy(), mx))
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
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    cfg, batch, p, eps = _case()
    losses, g = _grads(cfg, batch, p, eps)
    lay = flat_layout(cfg)
    ref = lay.pack(g, np.float64)
    assert np.allclose(flat[:-1], ref, rtol=1e-12, atol=1e-15)
    assert flat[-1] == pytest.approx(losses["cost"], rel=1e-12)   # mean of shard means
    assert mx == 2.0
