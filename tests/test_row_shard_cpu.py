"""Row-sharded zz^T and the encoder halo on CPU (gloo, world_size 2 and 3).

SURVEY §8e "beyond DP": ONE graph split by rows over the ranks (C5's N = 16384
graph).  Every rank owns a contiguous 128-row-aligned range (parallel.row_ranges),
all-gathers z and evaluates its rows against all columns; the row blocks'
[ce_sum, n_correct] all-reduce to the whole graph's and the dz rows concatenate to
the whole graph's dz with no reduction (L symmetric).  The per-rank compute here is
the oracle's row restriction (oracle.ref_numpy.adj_ce_rows, float64) in place of the
HIP kernel; the GPU kernel (snd_zzt_ce_rows) is checked against the same oracle in
tests/test_gpu_row_shard.py.  The encoder's halo: under the RCM row order every
neighbour lies within +-beta rows, so a rank's rows of A @ H need only beta rows
from each neighbouring range (parallel.halo_rows).
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
from snd_vae_amd.data import synthetic_batch


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


N, D = 700, 16          # 6 row blocks of 128, the last one partial


def _case():
    """One RGG graph relabelled in RCM order (bandwidth beta) and a latent z."""
    import scipy.sparse as sp
    from scipy.sparse.csgraph import reverse_cuthill_mckee
    cfg = tscale(N, D, mean_degree=8.0)
    b = synthetic_batch(cfg, 1, seed=11)
    A = b.sparse_adj(0)
    perm = reverse_cuthill_mckee(A.tocsr(), symmetric_mode=True)
    A = sp.csr_matrix(A[perm][:, perm])
    rows, cols = A.nonzero()
    beta = int(np.abs(rows - cols).max())
    z = 0.3 * np.random.default_rng(3).standard_normal((N, D))
    h = np.random.default_rng(4).standard_normal((N, 8))
    return A, beta, z, h


def _oracle_rows(z_full, r0, r1, rowptr, colidx, A=None):
    ce, dz, correct = R.adj_ce_rows(z_full.numpy(), A, N, r0, r1, row_chunk=128)
    return torch.tensor([ce, float(correct)], dtype=torch.float64), torch.from_numpy(dz)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from snd_vae_amd.parallel import (halo_rows, init_from_env, reducescatter_rows, row_ranges,
                                      row_sharded_adj_ce)
    info = init_from_env("gloo")
    A, beta, z, h = _case()
    ranges = row_ranges(N, world)
    r0, r1 = ranges[rank]
    A_loc = A[r0:r1]
    rp, ci = torch.from_numpy(A_loc.indptr.astype(np.int32)), torch.from_numpy(A_loc.indices.astype(np.int32))
    stats, dz = row_sharded_adj_ce(torch.from_numpy(z[r0:r1]), ranges, rank, rp, ci, info.group,
                                   compute=_oracle_rows, A=A)
    xh, lo = halo_rows(torch.from_numpy(h[r0:r1]), ranges, rank, beta, info.group)
    spmm_loc = A_loc[:, lo:lo + xh.shape[0]] @ xh.numpy()        # this rank's rows of A @ H
    # reduce-scatter of per-rank [N, w] contributions (rank r adds (r + 1) * h): own rows
    rs = reducescatter_rows(torch.from_numpy(h * (rank + 1.0)), ranges, info.group)
    q.put((rank, stats.numpy(), dz.numpy(), lo, xh.numpy(), spmm_loc, rs.numpy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_row_sharded_ce_and_halo_equal_whole_graph(world):
    from snd_vae_amd.parallel import row_ranges
    ranges = row_ranges(N, world)
    assert ranges[0][0] == 0 and ranges[-1][1] == N
    assert all(a[1] == b[0] for a, b in zip(ranges, ranges[1:]))
    assert all(r0 % 128 == 0 for r0, _ in ranges)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    got = dict((res[0], res[1:]) for res in (q.get(timeout=180) for _ in range(world)))
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    A, beta, z, h = _case()
    ce, dJ, correct = R.adj_ce(z, [A], N, row_chunk=128)
    for r in range(world):
        stats, dz, lo, xh, spmm_loc, rs = got[r]
        r0, r1 = ranges[r]
        # all-reduced loss terms = the whole graph's; dz rows = its rows of the full dz
        assert stats[0] == pytest.approx(ce, rel=1e-12)
        assert stats[1] == correct
        assert np.allclose(dz, dJ[r0:r1], rtol=1e-12, atol=1e-14)
        # halo: exactly rows [r0 - beta, r1 + beta) of H, and the local SpMM rows
        assert lo == max(0, r0 - beta)
        assert np.array_equal(xh, h[lo:min(N, r1 + beta)])
        assert np.allclose(spmm_loc, (A @ h)[r0:r1], rtol=1e-12, atol=1e-12)
        assert rs.shape == (r1 - r0, h.shape[1])
        assert np.allclose(rs, h[r0:r1] * (world * (world + 1) / 2), rtol=1e-12, atol=0)


def test_row_shard_plan_rejects_empty_ranks():
    """More ranks than 128-row blocks would leave a rank without rows: a clear error at
    plan time, not an argument error deep inside snd_zzt_ce_rows."""
    from snd_vae_amd.rowshard import RowShardPlan
    A, _, _, _ = _case()
    with pytest.raises(ValueError, match="without rows"):
        RowShardPlan(A.indptr, A.indices, N, 0, -(-N // 128) + 1, "cpu")


def test_torchcomm_rccl_scalars_go_to_the_device(monkeypatch):
    """A non-staged RCCL group without an explicit device sends the loss-stats all-reduce
    from the current GPU (RCCL rejects CPU tensors); gloo keeps host tensors."""
    import torch.distributed as tdist
    from snd_vae_amd.rowshard import TorchComm
    monkeypatch.setattr(tdist, "is_initialized", lambda: True)
    monkeypatch.setattr(tdist, "get_world_size", lambda group=None: 2)
    monkeypatch.setattr(torch.cuda, "current_device", lambda: 3)
    monkeypatch.setattr(tdist, "get_backend", lambda group=None: "nccl")
    assert TorchComm().scalar_device == torch.device("cuda", 3)
    assert TorchComm(staged=True).scalar_device == torch.device("cpu")
    assert TorchComm(device="cuda:1").scalar_device == torch.device("cuda", 1)
    monkeypatch.setattr(tdist, "get_backend", lambda group=None: "gloo")
    assert TorchComm().scalar_device == torch.device("cpu")
