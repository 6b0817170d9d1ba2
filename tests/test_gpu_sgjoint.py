"""The SND-VAE spatial-graph model as a plan (SND_SGJOINT):
two SpatialGraphConvolution layers over B x sampling_num spanning-tree copies,
flat heads per copy, z averaged over the copies after d_sg_lin1, the graph-latent
decoders -- one snd_train_step against the literal float64 oracle
(oracle/ref_sg.py sgjoint_forward_backward: the reference's dense B x N^3 message
tensors, torch autograd) at the reference's own scale (synthetic2: N=25, S=10).

Tolerances: fp32 -- ELBO terms 1e-5 relative, gradient blocks 2e-4
of max-abs, parameters after 3 TF1-Adam steps within 5 % of the step size; bf16
GEMM operands -- losses 2e-2, gradients 1e-1.
"""
import numpy as np
import pytest
import torch

from oracle import ref_numpy as R
from oracle import ref_sg as RS
from snd_vae_amd.config import PRESETS
from snd_vae_amd.data import sgjoint_batch
from snd_vae_amd.params import init_blocks

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu(lib_built):
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm device")


def dense_trees(b):
    S, n, B = b.sampling_num, b.n_nodes, b.n_graphs
    out = np.zeros((B * S, n, n))
    rp, ci = b.tree_rowptr.astype(np.int64), b.tree_colidx.astype(np.int64)
    for r in range(B * S * n):
        out[r // n, r % n, ci[rp[r]:rp[r + 1]] % n] = 1.0
    return out


def oracle_inputs(b):
    n, B, S = b.n_nodes, b.n_graphs, b.sampling_num
    return (dense_trees(b), b.features.reshape(B * S, n, -1), b.rel,
            np.stack([b.dense_adj(g) for g in range(B)]), b.feature_truth.reshape(B, n, -1),
            b.spatial_truth.reshape(B, n, -1))


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_sgjoint_steps_vs_oracle(dtype):
    from snd_vae_amd.model import DeviceBatch, SGCNModelVAE
    from snd_vae_amd.optimizer import OptimizerVAE
    cfg = PRESETS["SG25"]
    B = 2
    batch = sgjoint_batch(cfg, B, seed=3)
    p = {k: v.astype(np.float32).astype(np.float64) for k, v in init_blocks(cfg, 0).items()}
    model = SGCNModelVAE(cfg, B, dtype=dtype, blocks=p)
    opt = OptimizerVAE(model, fuse_adam=False)
    db = DeviceBatch(batch)
    ins = oracle_inputs(batch)
    rng = np.random.default_rng(5)
    m = {k: np.zeros_like(v) for k, v in p.items()}
    v = {k: np.zeros_like(x) for k, x in p.items()}
    ltol, gtol = (1e-5, 2e-4) if dtype == "f32" else (2e-2, 1e-1)
    for t in range(1, 4 if dtype == "f32" else 2):
        eps = rng.standard_normal((B * cfg.sampling_num, cfg.latent)).astype(np.float32)
        opt.step(db, torch.from_numpy(eps).cuda())
        got = opt.loss_dict()
        ref, rg = RS.sgjoint_forward_backward(p, *ins, eps.astype(np.float64), cfg)
        for k in ("cost", "spatial_cost", "adj_cost", "node_cost", "kl"):
            # kl ~ 1e-8 at the first steps: a mean of (1 + 2s - mu^2 - e^2s) terms of size ~1
            # cancelling, whose fp32 rounding floor is ~1e-7 absolute
            assert got[k] == pytest.approx(ref[k], rel=ltol, abs=1e-7), (t, k, got[k], ref[k])
        assert abs(got["acc"] - ref["acc"]) <= 1e-9 + (0 if dtype == "f32" else 1e-2)
        g = opt.grad_blocks()
        for k in rg:
            err = np.abs(g[k] - rg[k]).max() / max(np.abs(rg[k]).max(), 1e-30)
            assert err < gtol, (t, k, err)
        R.adam_tf1(p, rg, m, v, t, cfg.learning_rate, cfg.adam_beta1, cfg.adam_beta2, cfg.adam_eps)
        if dtype == "f32":
            blocks = model.blocks()
            for k in p:   # Adam normalises each update to ~lr: compare against the step size
                assert np.abs(blocks[k] - p[k]).max() < 0.05 * t * cfg.learning_rate, (t, k)
    # the latent per tree copy, the decoder input per graph (model.py:148-151,177-180)
    assert model.z_sg.shape == (B * cfg.sampling_num, cfg.latent)
    assert model.joint_h.shape == (B * cfg.n_nodes, cfg.node_h_size)


def test_sgjoint_graph_replay_and_trainer(tmp_path):
    """The SG-joint step captured in a HIP graph replays bit-identically to eager steps,
    and the Trainer feeds it from the reference on-disk format (2D_rel.npy and the
    sampled spanning trees of load_data_syn)."""
    from snd_vae_amd.input_data import load_data_syn, write_synthetic_dataset
    from snd_vae_amd.model import DeviceBatch, SGCNModelVAE
    from snd_vae_amd.optimizer import OptimizerVAE
    from snd_vae_amd.trainer import Trainer
    cfg = PRESETS["SG25"].replace(sampling_num=3)
    batch = sgjoint_batch(cfg, 2, seed=8)
    p0 = init_blocks(cfg, 2)
    runs = []
    for graph in (False, True):
        m = SGCNModelVAE(cfg, 2, dtype="f32", blocks=p0)
        o = OptimizerVAE(m)
        db = DeviceBatch(batch)
        if graph:
            o.capture(db, warmup=1)
            for _ in range(3):
                o.replay()
        else:
            for _ in range(3):
                o.step(db)
        torch.cuda.synchronize()
        runs.append((m, o))
    assert torch.equal(runs[0][0].params, runs[1][0].params)
    assert torch.equal(runs[0][1].losses, runs[1][1].losses)
    root = str(tmp_path)
    d = write_synthetic_dataset(root, cfg, 4, seed=3)
    rel = np.stack([np.sqrt(((sp[:, None] - sp[None]) ** 2).sum(-1))
                    for sp in np.load(f"{d}/2D_geometry.npy") / 600.0]) * 600.0
    np.save(f"{d}/2D_rel.npy", rel)
    np.random.seed(1)
    ds = load_data_syn("train", root, sampling_num=cfg.sampling_num)
    tr = Trainer(cfg, ds, batch_size=2, dtype="f32")
    h = tr.train(2)
    assert len(h) == 2 and np.isfinite(h[-1]["loss"]).all()
    assert tr.opt.global_step == 4
