"""CPU tests of the float64 oracle (oracle/ref_numpy.py) -- the parity checker.

Pins: analytic known-answer constants, finite differences, an independent
torch autograd formulation of the reference graph (oracle/ref_torch.py), the
TF1 Adam formula, and the committed golden fixtures (regenerated here).
Parity against TensorFlow itself is unpinned (TF not installable; the
reference ships no tests/fixtures) -- see DESIGN.md.
"""
import os

import numpy as np
import pytest
import torch

import golden_io
from oracle import ref_numpy as R
from oracle import ref_torch as T
from snd_vae_amd.config import tref, tscale
from snd_vae_amd.data import synthetic_batch
from snd_vae_amd.params import init_blocks

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def test_kat_constants():
    # diag pair CE: logits (1, 0), label 0 -> logsumexp(1,0) - 1 = softplus(-1)
    assert abs(R.SOFTPLUS_M1 - 0.3132616875182228) < 1e-15
    assert abs(R.BN_C - 0.9995003746877732) < 1e-15
    # 2-class softmax CE with logit0 = 0 equals BCE-with-logits
    L = np.linspace(-30, 30, 121)
    for a in (0.0, 1.0):
        lse = np.logaddexp(0.0, L)
        ce = lse - (1 - a) * 0.0 - a * L
        log_sig = lambda x: -np.logaddexp(0.0, -x)
        bce = -(a * log_sig(L) + (1 - a) * log_sig(-L))
        assert np.allclose(ce, bce, rtol=1e-12, atol=1e-12)


def test_lrelu_tf_maximum_gradient():
    # tf.maximum(x, 0.2x): grad goes to x where x >= 0.2x -> 1 at x == 0
    assert R.lrelu_grad(np.array([0.0]))[0] == 1.0
    assert R.lrelu_grad(np.array([-1e-30]))[0] == 0.2


def test_conv1d_same_matches_torch():
    rng = np.random.default_rng(0)
    x, w, b = rng.standard_normal((13, 3)), rng.standard_normal((5, 3, 4)), rng.standard_normal(4)
    out = R.conv1d_same(x, w, b)
    ref = T.conv1d_same(torch.tensor(x)[None], torch.tensor(w), torch.tensor(b))[0].numpy()
    assert np.allclose(out, ref, atol=1e-12)


def _small(n=25, d=8, B=2, seed=3, topology="tscale"):
    if topology == "tref":
        cfg = tref(n, d, g_hidden=12, latent=10, mean_degree=6.0)
    else:
        cfg = tscale(n, d, mean_degree=6.0)
    batch = synthetic_batch(cfg, B, seed=seed)
    rng = np.random.default_rng(seed)
    p = {k: v + 0.3 * rng.standard_normal(v.shape) for k, v in init_blocks(cfg, 1).items()}
    eps = rng.standard_normal((B, cfg.latent) if topology == "tref" else (B * n, d))
    adj = [batch.dense_adj(i) for i in range(B)]
    return cfg, batch, p, eps, adj


@pytest.mark.parametrize("topology", ["tscale", "tref"])
def test_oracle_grads_match_torch_autograd(topology):
    cfg, batch, p, eps, adj = _small(topology=topology)
    losses, g, _ = R.forward_backward(p, adj, batch.features, batch.feature_truth,
                                      batch.spatial_truth, eps, cfg)
    tp = T.build_params(p, torch.float64)
    cost, d = T.loss_fn(tp, *T.to_tensors((adj, batch.features, batch.feature_truth,
                                           batch.spatial_truth, eps), cfg, torch.float64), cfg)
    cost.backward()
    for k in ("cost", "adj_cost", "node_cost", "spatial_cost", "kl", "acc"):
        assert abs(losses[k] - float(d[k])) <= 1e-12 * max(1.0, abs(losses[k])), k
    for k in p:
        ref = tp[k].grad.numpy()
        err = np.abs(g[k] - ref).max() / (np.abs(ref).max() + 1e-30)
        assert err < 1e-10, (k, err)


@pytest.mark.parametrize("topology", ["tscale", "tref"])
def test_oracle_finite_differences(topology):
    cfg, batch, p, eps, adj = _small(n=12, d=4, B=2 if topology == "tref" else 1, seed=7,
                                     topology=topology)
    args = (adj, batch.features, batch.feature_truth, batch.spatial_truth, eps, cfg)
    _, g, _ = R.forward_backward(p, *args)
    rng = np.random.default_rng(0)
    h = 1e-6
    keys = ["enc.W0", "enc.W1", "enc.bne.gamma", "enc.Wms", "dec.K1", "dec.K3s", "dec.bn1.beta",
            "dec.Wn"]
    if topology == "tref":
        keys += ["enc.Wh", "enc.bh", "dec.Wp", "dec.bp"]
    for k in keys:
        idx = tuple(rng.integers(0, s) for s in p[k].shape)
        pp = {a: b.copy() for a, b in p.items()}
        pm = {a: b.copy() for a, b in p.items()}
        pp[k][idx] += h
        pm[k][idx] -= h
        fd = (R.forward_backward(pp, *args, want_grads=False)[0]["cost"] -
              R.forward_backward(pm, *args, want_grads=False)[0]["cost"]) / (2 * h)
        assert abs(fd - g[k][idx]) < 1e-6 * max(1.0, abs(fd)), (k, fd, g[k][idx])


def test_tf1_adam_formula():
    p = {"w": np.array([1.0, -2.0])}
    g = {"w": np.array([0.5, 0.25])}
    m = {"w": np.zeros(2)}
    v = {"w": np.zeros(2)}
    R.adam_tf1(p, g, m, v, 1, 0.001)
    # t=1: m = 0.1 g, v = 0.001 g^2, lr_t = lr sqrt(0.001)/0.1 -> step = lr*g/(|g| + eps/sqrt(.001)...)
    lr_t = 0.001 * np.sqrt(1 - 0.999) / (1 - 0.9)
    exp = np.array([1.0, -2.0]) - lr_t * 0.1 * g["w"] / (np.sqrt(0.001 * g["w"] ** 2) + 1e-8)
    assert np.allclose(p["w"], exp, rtol=0, atol=1e-15)


@pytest.mark.parametrize("name", golden_io.NAMES)
def test_golden_fixture_reproduces(name):
    z, cfg, fixture_batch, p0 = golden_io.load(name)
    B = fixture_batch.n_graphs
    batch = synthetic_batch(cfg, B, seed=int(z["seed"]))
    assert np.array_equal(batch.rowptr, z["rowptr"]) and np.array_equal(batch.colidx, z["colidx"])
    assert np.array_equal(batch.features, z["features"])
    adj = [batch.dense_adj(b) for b in range(B)]
    losses, g, _ = R.forward_backward(p0, adj, z["features"], z["feature_truth"],
                                      z["spatial_truth"], z["eps"][0].astype(np.float64), cfg)
    assert losses["cost"] == pytest.approx(float(z["s0/loss/cost"]), rel=1e-13)
    for k in p0:
        err, nerr = golden_io.block_error(z, "s0/grad", k, g[k])
        assert err < 1e-10 and (nerr is None or nerr < 1e-12), (k, err, nerr)


def test_c1_fixture_is_the_reference_topology():
    """BASELINE configs[0]: graph latent, F_in = num_feature (model.py:104), L = 100."""
    z, cfg, batch, p0 = golden_io.load("tref_c1_n200_d16")
    assert cfg.topology == "tref" and cfg.f_in == 1 and cfg.latent == 100
    assert p0["enc.Wh"].shape == (200 * 17, 100) and p0["dec.Wp"].shape == (100, 200 * 16)


def test_adj_ce_chunked_sparse_equals_dense():
    """adj_ce over scipy-sparse adjacencies in row chunks (the large-N oracle, N = 16384)
    equals the dense one-shot form: same CE sum, dJ and correct count."""
    from snd_vae_amd.config import tscale
    from snd_vae_amd.data import synthetic_batch
    cfg = tscale(300, 8, mean_degree=8.0)
    b = synthetic_batch(cfg, 2, seed=3)
    J = np.random.default_rng(1).standard_normal((600, 8))
    dense = [b.dense_adj(g).astype(np.float64) for g in range(2)]
    sparse = [b.sparse_adj(g) for g in range(2)]
    for g in range(2):
        assert np.array_equal(sparse[g].toarray(), dense[g])
    ce0, dj0, c0 = R.adj_ce(J, dense, 300, 1.7, 0.6)
    ce1, dj1, c1, amb = R.adj_ce(J, sparse, 300, 1.7, 0.6, row_chunk=64, amb_tol=1e-3)
    assert abs(ce1 - ce0) <= 1e-12 * abs(ce0)
    np.testing.assert_allclose(dj1, dj0, rtol=1e-12, atol=1e-12)
    assert c1 == c0 and amb >= 0



def test_lrelu_override_changes_exactly_the_overridden_derivatives():
    """forward_backward(lrelu_override=...) evaluates the backward pass with the given
    lrelu' at the given elements (NaN elsewhere = the oracle's own choice): overriding every
    element with the oracle's own derivative changes nothing, and flipping ONE element of
    the decoder's layer-1 pre-activation moves dec.b1 by exactly 0.8 dU1 gamma c there."""
    import oracle.ref_numpy as RN
    from snd_vae_amd.config import tscale
    from snd_vae_amd.data import synthetic_batch
    from snd_vae_amd.params import init_blocks
    cfg = tscale(60, 16, mean_degree=5.0)
    b = synthetic_batch(cfg, 2, seed=4)
    p = {k: v.astype(np.float64) for k, v in init_blocks(cfg, 1).items()}
    eps = np.random.default_rng(3).standard_normal((2 * 60, 16))
    adj = [b.dense_adj(i) for i in range(2)]
    args = (p, adj, b.features, b.feature_truth, b.spatial_truth, eps, cfg)
    _, g, cache = RN.forward_backward(*args)
    same = {k: RN.lrelu_grad(cache[k]) for k in ("P0", "P1", "T1", "T2s", "T3s", "T2n")}
    _, g_same, _ = RN.forward_backward(*args, lrelu_override=same)
    assert all(np.array_equal(g[k], g_same[k]) for k in g)
    T1 = cache["T1"]
    r, col = np.unravel_index(np.argmin(np.abs(T1)), T1.shape)
    o = np.full(T1.shape, np.nan)
    o[r, col] = 1.2 - RN.lrelu_grad(T1[r, col])      # the other side: 1 <-> 0.2
    _, g_flip, c2 = RN.forward_backward(*args, lrelu_override={"T1": o})
    # dU1 at (r, col) from the flipped run's own backward: recompute it from dT1 = dU1 * d
    gam = p["dec.bn1.gamma"][col] * RN.BN_C
    delta = g_flip["dec.b1"] - g["dec.b1"]
    assert np.count_nonzero(delta) == 1 and delta[col] != 0
    d_old, d_new = RN.lrelu_grad(T1[r, col]), o[r, col]
    dU = (g_flip["dec.bn1.beta"][col] - g["dec.bn1.beta"][col]) / (d_new - d_old)
    assert delta[col] == pytest.approx(dU * (d_new - d_old) * gam, rel=1e-9)
