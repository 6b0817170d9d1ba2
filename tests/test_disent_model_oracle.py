"""The disentangled-model oracle (oracle/ref_disent_model.py: SGCNModelVAE of
model.py:19-222 with the optimizer.py:123-203 costs, float64 torch ops) on CPU:

* every variable of snd_vae_amd.disent_model.block_shapes is read by the oracle (the
  layouts agree) and receives a gradient;
* autograd gradients == central finite differences of the oracle's own cost, for each
  model_type branch;
* its pieces agree with the per-piece oracles it composes (KL / regulariser values of
  ref_disent.group_reg).
"""
import numpy as np
import pytest

from oracle import ref_disent as RD
from oracle import ref_disent_model as RM


def dense_trees(b):
    S, n, B = b.sampling_num, b.n_nodes, b.n_graphs
    out = np.zeros((B * S, n, n))
    rp, ci = b.tree_rowptr.astype(np.int64), b.tree_colidx.astype(np.int64)
    for r in range(B * S * n):
        out[r // n, r % n, ci[rp[r]:rp[r + 1]] % n] = 1.0
    return out


def disent_inputs(b, spatial_dim=2):
    n, B, S = b.n_nodes, b.n_graphs, b.sampling_num
    return {"x": b.feature_truth.reshape(B, n, -1), "spatial": b.spatial_truth.reshape(B, n, spatial_dim),
            "adj": np.stack([b.dense_adj(g) for g in range(B)]), "x_sg": b.features.reshape(B * S, n, -1),
            "trees": dense_trees(b), "rel": b.rel}


def small_case(model_type="disentangled", **kw):
    from snd_vae_amd.config import sgjoint
    from snd_vae_amd.data import sgjoint_batch
    from snd_vae_amd.disent_model import DisentangledConfig
    n, B, S = 6, 2, 2
    cfg = DisentangledConfig(n_nodes=n, g_conv_hidden=(3, 4), s_channel=(3, 3, 4),
                             sg_conv_hidden=((3, 4, 5), (4, 3, 5)), g_hidden=6, g_latent=3, s_hidden=6, s_latent=3,
                             sg_hidden=6, sg_latent=3, sampling_num=S, node_h=4, n_d_channel=(5, 3),
                             e_d_hidden=(4, 3), s_d_channel=(4, 3, 3), model_type=model_type, **kw)
    b = sgjoint_batch(sgjoint(n, 16, mean_degree=3.0, sampling_num=S), B, seed=1)
    rng = np.random.default_rng(2)
    eps = {"s": rng.standard_normal((B, cfg.s_latent)), "g": rng.standard_normal((B, cfg.g_latent)),
           "sg": rng.standard_normal((B * S, cfg.sg_latent))}
    return cfg, disent_inputs(b), eps


def scaled(blocks, f=5.0):
    """Larger N(0, 0.02) weights (non-trivial gradients); glorot kernels and BN kept."""
    big = lambda k: k.endswith(("/Matrix", "/w", "/w1")) or (k.startswith("g_sg") and k.endswith("_conv"))
    return {k: v * f if big(k) else v.copy() for k, v in blocks.items()}


def test_layout_covers_every_variable():
    from snd_vae_amd.disent_model import block_shapes, init_blocks
    cfg, ins, eps = small_case()
    p = scaled(init_blocks(cfg, 0))
    assert set(p) == set(block_shapes(cfg))
    losses, g = RM.disent_forward_backward(p, ins, eps, cfg)
    assert set(g) == set(p)
    for k, v in g.items():
        assert v is not None and v.shape == p[k].shape and np.isfinite(v).all(), k
        assert np.abs(v).max() > 0, k            # every variable is on the cost's path
    assert np.isfinite(losses["cost"]) and 0 <= losses["correct"] <= 2 * 6 * 6


@pytest.mark.parametrize("model_type,kw", [("disentangled", {}), ("beta-TCVAE", {}), ("NED-VAE-IP", {}),
                                           ("disentangled_C", {"capacity": 0.0, "gamma": 3.0}),
                                           ("base", {})])
def test_oracle_finite_differences(model_type, kw):
    import torch
    from snd_vae_amd.disent_model import init_blocks
    cfg, ins, eps = small_case(model_type, **kw)
    p = scaled(init_blocks(cfg, 3))
    _, g = RM.disent_forward_backward(p, ins, eps, cfg)
    tin = {k: torch.tensor(np.asarray(v, np.float64)) for k, v in ins.items()}
    te = {k: torch.tensor(v) for k, v in eps.items()}

    def cost(q):
        c, _, _ = RM.disent_loss_torch({k: torch.tensor(v) for k, v in q.items()}, tin, te, cfg)
        return float(c)
    rng = np.random.default_rng(0)
    keys = ("g_g0_conv/w", "g_bn_g1/gamma", "g_g23_lin/Matrix", "g_s1_conv/kernel", "encoder_s/beta",
            "g_sg0_conv", "g_sg23_lin/bias", "d_sg_lin1/Matrix", "d_g_lin1/bias", "n0_deconv/kernel",
            "decoder_node/gamma", "e0_deconv/w1", "d_bn_e0/gamma", "d_e_lin2/Matrix", "s2_deconv/kernel",
            "d_s_lin2/bias")
    for k in keys:
        idx = tuple(rng.integers(0, d) for d in p[k].shape)
        h = 1e-6
        qp = {kk: vv.copy() for kk, vv in p.items()}
        qm = {kk: vv.copy() for kk, vv in p.items()}
        qp[k][idx] += h
        qm[k][idx] -= h
        fd = (cost(qp) - cost(qm)) / (2 * h)
        assert abs(fd - g[k][idx]) <= 1e-6 + 1e-5 * abs(fd), (model_type, k, idx, fd, g[k][idx])


def test_regulariser_parts_match_group_oracle():
    import torch
    from snd_vae_amd.disent_model import init_blocks
    cfg, ins, eps = small_case("NED-VAE-IP")
    p = {k: torch.tensor(v) for k, v in scaled(init_blocks(cfg, 1)).items()}
    tin = {k: torch.tensor(np.asarray(v, np.float64)) for k, v in ins.items()}
    te = {k: torch.tensor(v) for k, v in eps.items()}
    cost, parts, groups = RM.disent_loss_torch(p, tin, te, cfg)
    reg = 0.0
    for name, w in RD.model_type_groups(cfg.model_type, cfg.beta, cfg.gamma, cfg.capacity).items():
        mu, ls, _ = groups[name]
        v = RD.group_reg(mu.numpy(), ls.numpy(), (mu + te[name] * torch.exp(ls)).numpy(), **w)
        assert float(parts["kl_" + name]) == pytest.approx(v["kl"], rel=1e-12)
        reg += v["term"]
    rec = float(parts["adj_cost"] + parts["node_cost"] + parts["spatial_cost"])
    assert float(cost) == pytest.approx(rec + reg, rel=1e-12)
