"""The row-sharded training step (snd_vae_amd/rowshard.py) on CPU: gloo, world 2 and 3.

ONE graph (SURVEY §8e "beyond DP", C5's regime at a CPU size) split by rows over the
ranks; every rank runs rowshard.forward_backward with a float64 torch restatement of
the ops (``RefOps`` below, test infrastructure: the oracle's own conv / CE helpers and
the formulas of oracle/ref_numpy.py) in place of the HIP calls, so this test checks
the ORCHESTRATION -- row ranges, the all-gathers of H1 and z, the decoder windows with
their 6 halo rows, the reduce-scatters of dH1 and dJ, the whole-graph denominators,
the all-reduced gradient -- against the whole-graph float64 oracle
(``ref_numpy.forward_backward``): losses and every gradient block to 1e-10.  The HIP
ops are checked against the same oracle on the GPU (tests/test_gpu_row_shard_step.py).
"""
import os
import socket

import numpy as np
import pytest
import scipy.sparse as sp
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import ref_numpy as R
from snd_vae_amd.config import tscale
from snd_vae_amd.data import synthetic_batch
from snd_vae_amd.params import init_blocks

N, D = 700, 16            # 6 row blocks of 128, the last one partial
C = R.BN_C


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class RefOps:
    """float64 CPU restatement of the HipOps interface (test infrastructure)."""

    def mm(self, a, b, bias=None):
        return a @ b + (0 if bias is None else bias)

    def linear(self, x, w, b):
        return x @ w + b

    def mm_tn(self, a, b):
        return a.T @ b

    def mm_nt(self, a, b):
        return a @ b.T

    def colsum(self, a):
        return a.sum(0)

    def spmm(self, csr, h):
        A = sp.csr_matrix((np.ones(len(csr.colidx)), csr.colidx.numpy(), csr.rowptr.numpy()),
                          shape=(csr.n_out, h.shape[0]))
        return torch.from_numpy(A @ h.numpy())

    def bn_act(self, y, g, b, act, act_first):
        if act_first:
            return torch.maximum(y, 0.2 * y) * (g * C) + b
        t = y * (g * C) + b
        return torch.maximum(t, 0.2 * t) if act else t

    def bn_act_bwd(self, dx, y, g, b, act, act_first):
        lg = lambda v: torch.where(v >= 0, torch.ones_like(v), 0.2 * torch.ones_like(v))
        if act_first:   # x = BN(lrelu(y))
            a = torch.maximum(y, 0.2 * y)
            return dx * (g * C) * lg(y), (dx * a).sum(0) * C, dx.sum(0)
        t = y * (g * C) + b
        dt = dx * lg(t) if act else dx
        return dt * (g * C), (dt * y).sum(0) * C, dt.sum(0)

    def conv_bn_lrelu(self, x, w, b, g, beta):
        y = torch.from_numpy(R.per_graph_conv(x.numpy(), w.numpy(), b.numpy(), len(x)))
        t = y * (g * C) + beta
        return y, torch.maximum(t, 0.2 * t)

    def conv_bwd(self, x, w, dy):
        dx, dw, _ = R.per_graph_conv_bwd(x.numpy(), w.numpy(), dy.numpy(), len(x))
        return torch.from_numpy(dx), torch.from_numpy(dw)

    def sigmoid_mse(self, u, w, b, t, count):
        yh = torch.sigmoid(u @ w + b)
        dp = 2.0 * (yh - t) / count * yh * (1 - yh)
        return float(((yh - t) ** 2).sum()), dp @ w.T, u.T @ dp, dp.sum(0)

    def reparam(self, mu, s, eps):
        return mu + eps * torch.exp(s), float((1 + 2 * s - mu ** 2 - torch.exp(2 * s)).sum())

    def reparam_bwd(self, mu, s, eps, dz, c):
        return dz + c * mu, dz * eps * torch.exp(s) + c * (torch.exp(2 * s) - 1)

    def adj_ce_rows(self, z_full, plan, pw, norm):
        ce, dz, correct = R.adj_ce_rows(z_full.numpy(), plan.A, plan.n, plan.r0, plan.r1, pw, norm, row_chunk=256)
        return ce, float(correct), torch.from_numpy(dz)


def _case():
    cfg = tscale(N, D, mean_degree=8.0)
    b = synthetic_batch(cfg, 1, seed=11)
    p0 = {k: v.astype(np.float64) for k, v in init_blocks(cfg, 3).items()}
    eps = np.random.default_rng(4).standard_normal((N, D))
    return cfg, b, p0, eps


def _worker(rank, world, port, q):
    try:
        from snd_vae_amd.rowshard import RowShardPlan, TorchComm, forward_backward
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        torch.set_num_threads(1)
        cfg, b, p0, eps = _case()
        plan = RowShardPlan(b.rowptr, b.colidx, N, rank, world, "cpu", index_dtype=torch.int64)
        plan.A = sp.csr_matrix((np.ones(len(b.colidx)), b.colidx, b.rowptr), shape=(N, N))
        p = {k: torch.from_numpy(v) for k, v in p0.items()}
        X = torch.from_numpy(np.asarray(b.features, np.float64))
        own = slice(plan.r0, plan.r1)
        losses, g = forward_backward(p, plan, X, torch.from_numpy(np.asarray(b.feature_truth, np.float64)[own]),
                                     torch.from_numpy(np.asarray(b.spatial_truth, np.float64)[own]),
                                     torch.from_numpy(eps[own]), cfg, RefOps(), TorchComm())
        q.put((rank, losses, {k: v.numpy() for k, v in g.items()}))
    except Exception as e:   # surface the worker's failure in the test
        import traceback
        q.put((rank, "ERROR", traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_row_sharded_step_equals_whole_graph(world):
    cfg, b, p0, eps = _case()
    A = sp.csr_matrix((np.ones(len(b.colidx)), b.colidx, b.rowptr), shape=(N, N))
    ref, rg, _ = R.forward_backward(p0, [A], b.features, b.feature_truth, b.spatial_truth, eps, cfg,
                                    row_chunk=256)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    out = [q.get(timeout=300) for _ in range(world)]
    for pr in procs:
        pr.join(60)
    for rank, losses, g in out:
        assert losses != "ERROR", g
        for k in ("cost", "adj_cost", "node_cost", "spatial_cost", "kl"):
            assert losses[k] == pytest.approx(ref[k], rel=1e-10, abs=1e-14), (rank, k)
        assert losses["correct"] == ref["correct"]
        for k in rg:
            err = np.abs(g[k].reshape(rg[k].shape) - rg[k]).max() / max(np.abs(rg[k]).max(), 1e-30)
            assert err < 1e-10, (rank, k, err)
