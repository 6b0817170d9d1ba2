"""snd_zzt_ce_rows (the row-sharded zz^T of SURVEY §8e) on the GPU.

* Against the float64 oracle's row restriction (oracle.ref_numpy.adj_ce_rows): the
  range's CE sum, correct count and dz rows, at C5 (N = 16384, d = 128) and at a size
  with a partial last row block (N = 1000).
* The row ranges of a partition sum to the whole-graph kernel (snd_zzt_ce).
* The world-1 forced-RCCL rehearsal of parallel.row_sharded_adj_ce (all-gather of z,
  the kernel on the rank's rows, all-reduce of the loss scalars over RCCL) and of
  parallel.halo_rows: unmeasured at world > 1 (no multi-GPU box here); the
  arithmetic of world 2 and 3 is tests/test_row_shard_cpu.py.
"""
import socket

import numpy as np
import pytest
import torch

from oracle import ref_numpy as R
from snd_vae_amd.config import tscale
from snd_vae_amd.data import synthetic_batch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu(lib_built):
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm device")


def _graph(n, d, seed):
    b = synthetic_batch(tscale(n, d), 1, seed=seed)
    z = (0.1 * np.random.default_rng(seed).standard_normal((n, d))).astype(np.float32)
    return b, z


def _rows_csr(b, r0, r1):
    rp = torch.from_numpy(b.rowptr[r0:r1 + 1].astype(np.int32)).cuda()
    ci = torch.from_numpy(b.colidx.astype(np.int32)).cuda()
    return rp, ci


@pytest.mark.timeout(300)
@pytest.mark.parametrize("n,d,ranges", [
    (16384, 128, [(0, 2048), (14336, 16384)]),
    (1000, 64, [(0, 384), (384, 896), (896, 1000)]),
])
@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_zzt_ce_rows_vs_oracle(n, d, ranges, dtype):
    from snd_vae_amd.layers import inner_product_ce_rows
    b, z = _graph(n, d, 7)
    A = b.sparse_adj(0)
    zd = torch.from_numpy(z).cuda()
    for r0, r1 in ranges:
        rp, ci = _rows_csr(b, r0, r1)
        stats, dz = inner_product_ce_rows(zd, r0, r1, rp, ci, dtype=dtype)
        ce, rdz, correct = R.adj_ce_rows(z.astype(np.float64), A, n, r0, r1, row_chunk=1024)
        s = stats.cpu().numpy()
        err = np.abs(dz.cpu().numpy() - rdz).max() / np.abs(rdz).max()
        if dtype == "f32":
            assert s[0] == pytest.approx(ce, rel=2e-6), (r0, r1)
            assert abs(s[1] - correct) <= 2, (r0, r1, s[1], correct)
            assert err < 1e-5, (r0, r1, err)
        else:
            assert s[0] == pytest.approx(ce, rel=2e-3), (r0, r1)
            assert abs(s[1] - correct) <= 1e-3 * (r1 - r0) * n
            assert err < 2e-2, (r0, r1, err)


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_zzt_ce_rows_partition_equals_whole_graph(dtype):
    from snd_vae_amd import layers
    from snd_vae_amd.parallel import row_ranges
    n, d = 4096, 64
    b, z = _graph(n, d, 3)
    zd = torch.from_numpy(z).cuda()
    rp_all = torch.from_numpy(b.rowptr.astype(np.int32)).cuda()
    ci = torch.from_numpy(b.colidx.astype(np.int32)).cuda()
    ce, correct, dz = layers.inner_product_ce(zd, 1, rp_all, ci, dtype=dtype)
    tot = np.zeros(2)
    parts = []
    for r0, r1 in row_ranges(n, 8):
        rp, _ = _rows_csr(b, r0, r1)
        stats, dzr = layers.inner_product_ce_rows(zd, r0, r1, rp, ci, dtype=dtype)
        tot += stats.cpu().numpy()
        parts.append(dzr)
    assert tot[0] == pytest.approx(ce, rel=1e-6)
    assert abs(tot[1] - correct) <= (0 if dtype == "f32" else 1e-4 * n * n)
    dzp = torch.cat(parts)
    err = float((dzp - dz).abs().max() / dz.abs().max())
    assert err < (1e-6 if dtype == "f32" else 1e-2), err


def test_row_sharded_world1_rccl_rehearsal():
    """parallel.row_sharded_adj_ce and halo_rows over a world-1 RCCL group: the
    collectives run (all-gather, all-reduce on device tensors) and the result is the
    whole-graph kernel's."""
    import torch.distributed as dist

    from snd_vae_amd import layers
    from snd_vae_amd.parallel import halo_rows, row_ranges, row_sharded_adj_ce
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        n, d = 2048, 64
        b, z = _graph(n, d, 5)
        zd = torch.from_numpy(z).cuda()
        ranges = row_ranges(n, 1)
        rp, ci = _rows_csr(b, 0, n)
        stats, dz = row_sharded_adj_ce(zd, ranges, 0, rp, ci, dist.group.WORLD, dtype="bf16")
        torch.cuda.synchronize()
        ce, correct, dz_full = layers.inner_product_ce(zd, 1, rp, ci, dtype="bf16")
        assert float(stats[0]) == pytest.approx(ce, rel=1e-9)
        assert float(stats[1]) == correct
        assert torch.equal(dz, dz_full)
        h = torch.randn(n, 8, device="cuda")
        xh, lo = halo_rows(h, ranges, 0, 100, dist.group.WORLD)
        assert lo == 0 and torch.equal(xh, h)
    finally:
        dist.destroy_process_group()
