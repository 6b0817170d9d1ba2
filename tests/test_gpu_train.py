"""Train loop on device-resident batches, HIP-graph replay per batch, checkpoints.

* A Trainer epoch (one captured graph per batch) reproduces, bit for bit, the
  same sequence of eager OptimizerVAE steps over the same batches.
* save -> restore -> continue equals uninterrupted training (params, Adam
  state and the Philox step counter all travel in the checkpoint).
* The first step of a Trainer fed from the reference on-disk format equals
  the float64 oracle on the same graphs (fp32 engine, injected eps).
"""
import os

import numpy as np
import pytest
import torch

from oracle import ref_numpy as R
from snd_vae_amd.config import tscale
from snd_vae_amd.input_data import load_data_syn, write_synthetic_dataset
from snd_vae_amd.params import init_blocks

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu(lib_built):
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm device")


@pytest.fixture(scope="module")
def dataset(tmp_path_factory):
    cfg = tscale(96, 16, mean_degree=6.0)
    root = str(tmp_path_factory.mktemp("ds"))
    write_synthetic_dataset(root, cfg, 6, seed=11)
    np.random.seed(1)
    return cfg, load_data_syn("train", root, sampling_num=2)


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_trainer_graphs_equal_eager(dataset, dtype):
    from snd_vae_amd.trainer import Trainer
    cfg, ds = dataset
    t = Trainer(cfg, ds, batch_size=2, dtype=dtype)
    e = Trainer(cfg, ds, batch_size=2, dtype=dtype, use_graphs=False)
    assert t.batch_num == 3
    for _ in range(2):
        ht, he = t.train_epoch(), e.train_epoch()
        for k in ("loss", "adj_loss", "node_loss", "spatial_loss", "sg_kl", "adj_acc"):
            np.testing.assert_array_equal(ht[k], he[k], err_msg=k)
    assert torch.equal(t.model.params, e.model.params)
    assert torch.equal(t.opt.m, e.opt.m) and torch.equal(t.opt.v, e.opt.v)
    assert t.opt.global_step == 6


def test_checkpoint_resume(dataset, tmp_path):
    from snd_vae_amd.trainer import Trainer
    cfg, ds = dataset
    a = Trainer(cfg, ds, batch_size=3, dtype="f32")
    a.train(1)
    fn = str(tmp_path / "ck.safetensors")
    a.save(fn)
    ha = a.train(2)
    b = Trainer(cfg, ds, batch_size=3, dtype="f32", blocks=init_blocks(cfg, 99))
    assert b.restore(fn) == 2
    hb = b.train(2)
    for x, y in zip(ha, hb):
        np.testing.assert_array_equal(x["loss"], y["loss"])
    assert torch.equal(a.model.params, b.model.params)


@pytest.mark.parametrize("weighted", [False, True])
def test_first_step_matches_oracle(dataset, weighted):
    """weighted: row a15 -- the weighted-BCE structure loss with the dataset's
    pos_weight / norm (`main.py:246-247` over the spanning trees)."""
    from snd_vae_amd.input_data import dataset_class_balance
    from snd_vae_amd.model import DeviceBatch
    from snd_vae_amd.trainer import Trainer
    cfg, ds = dataset
    p0 = {k: v.astype(np.float32).astype(np.float64) for k, v in init_blocks(cfg, 0).items()}
    t = Trainer(cfg, ds, batch_size=2, dtype="f32", blocks=p0, use_graphs=False, weighted=weighted)
    if weighted:
        pw, nm = dataset_class_balance(ds)
        assert pw > 1.0 and t.cfg.pos_weight == pw and t.cfg.norm == nm
        cfg = t.cfg
    hb = ds.batch(cfg, [0, 1])
    eps = np.random.default_rng(4).standard_normal((2 * cfg.n_nodes, cfg.latent)).astype(np.float32)
    t.opt.step(t.batches[0], torch.from_numpy(eps).cuda())
    got = t.opt.loss_dict()
    ref, _, _ = R.forward_backward(p0, [hb.dense_adj(b) for b in range(2)], hb.features,
                                   hb.feature_truth, hb.spatial_truth, eps.astype(np.float64), cfg,
                                   want_grads=False)
    for k in ("cost", "adj_cost", "node_cost", "spatial_cost", "kl"):
        assert abs(got[k] - ref[k]) <= 1e-5 * abs(ref[k]) + 1e-7, (k, got[k], ref[k])
    assert isinstance(t.batches[0], DeviceBatch)
