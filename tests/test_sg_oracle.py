"""SpatialGraphConvolution oracle (oracle/ref_sg.py) and the factorised algebra
the HIP layer implements (csrc/snd_sg.hip), on CPU.

* numpy literal forward == torch literal forward (two formulations);
* torch autograd gradients == central finite differences;
* the factorised forward/backward (restated below in dense numpy, the same
  equations as the kernels) == the literal O(N^3) graph, symmetric adjacency.
"""
import numpy as np
import pytest

from oracle import ref_sg as S

lr = S.lrelu


def lrg(x):
    return np.where(x >= 0, 1.0, 0.2)


def fact_fwd(A, X, Rl, p):
    F = X.shape[1]
    LX = lr(X); d = A.sum(1); AX = A @ LX
    M1 = p["M1"]
    u, v, w = LX @ M1[:F], LX @ M1[F:2 * F], AX @ M1[2 * F:3 * F]
    LR = lr(Rl); e = (A * LR).sum(1); Q = LR @ A.T
    S3 = A[:, :, None] * (d[None, :, None] * (u[:, None] + v[None] + LR[..., None] * M1[3 * F]
                                               + p["b1"]) + w[None] + e[None, :, None] * M1[3 * F + 1]
                          + Q[..., None] * M1[3 * F + 2])
    P = (A[..., None] * lr(S3)).sum(1)
    M2 = p["M2"]
    m2 = d[:, None] * (LX @ M2[:F] + p["b2"]) + AX @ M2[F:2 * F] + e[:, None] * M2[2 * F] \
        + P @ M2[2 * F + 1:]
    return np.concatenate([LX, lr(m2)], 1) @ p["M3"] + p["b3"], (LX, d, AX, u, v, w, LR, e, Q, S3, P, m2)


def fact_bwd(A, X, Rl, p, dO):
    F = X.shape[1]
    _, (LX, d, AX, u, v, w, LR, e, Q, S3, P, m2) = fact_fwd(A, X, Rl, p)
    M1, M2 = p["M1"], p["M2"]
    g = {"M3": np.concatenate([LX, lr(m2)], 1).T @ dO, "b3": dO.sum(0)}
    dZ3 = dO @ p["M3"].T
    dLX = dZ3[:, :F].copy()
    dm2 = dZ3[:, F:] * lrg(m2)
    g["M2"] = np.concatenate([(d[:, None] * LX).T @ dm2, AX.T @ dm2, (e @ dm2)[None], P.T @ dm2])
    g["b2"] = d @ dm2
    dLX += d[:, None] * (dm2 @ M2[:F].T)
    dAX = dm2 @ M2[F:2 * F].T
    dP = dm2 @ M2[2 * F + 1:].T
    G = A[..., None] * dP[:, None, :] * lrg(S3)
    du = (G * d[None, :, None]).sum(1); dw = G.sum(0); dv = d[:, None] * dw
    g["M1"] = np.concatenate([LX.T @ du, LX.T @ dv, AX.T @ dw,
                              (G * (d[None, :, None] * LR[..., None])).sum((0, 1))[None],
                              (G * e[None, :, None]).sum((0, 1))[None],
                              (G * Q[..., None]).sum((0, 1))[None]])
    g["b1"] = du.sum(0)
    dLX += du @ M1[:F].T + dv @ M1[F:2 * F].T
    dAX += dw @ M1[2 * F:3 * F].T
    g["x"] = (dLX + A.T @ dAX) * lrg(X)
    return g


@pytest.fixture
def case():
    rng = np.random.default_rng(0)
    B, N, F = 2, 7, 3
    A = np.triu((rng.random((B, N, N)) < 0.4).astype(float), 1)
    A = A + A.transpose(0, 2, 1)
    X = rng.normal(size=(B, N, F))
    pos = rng.random((B, N, 2))
    Rl = np.linalg.norm(pos[:, :, None] - pos[:, None], axis=-1) - 0.3   # both lrelu branches
    p = S.init_sg_layer(F, (4, 5, 6), rng, stddev=0.5)
    for k, n in (("b1", 4), ("b2", 5), ("b3", 6)):
        p[k] = rng.normal(size=n)
    return A, X, Rl, p


def test_numpy_equals_torch(case):
    import torch
    A, X, Rl, p = case
    ref = S.sgconv(A, X, Rl, p)
    t = {k: torch.tensor(v) for k, v in p.items()}
    got = S.sgconv_torch(torch.tensor(A), torch.tensor(X), torch.tensor(Rl), t).numpy()
    np.testing.assert_allclose(got, ref, rtol=1e-12, atol=1e-12)


def test_autograd_vs_finite_differences(case):
    A, X, Rl, p = case
    dO = np.random.default_rng(1).normal(size=(2, 7, 6))
    _, g = S.sgconv_grads(A, X, Rl, p, dO)
    f = lambda q, x: float((S.sgconv(A, x, Rl, q) * dO).sum())
    h = 1e-6
    for key, idx in (("M1", (3 * 3 + 2, 1)), ("M1", (4, 2)), ("M2", (7, 3)), ("b1", (2,)),
                     ("M3", (5, 4))):
        q1 = {k: v.copy() for k, v in p.items()}
        q2 = {k: v.copy() for k, v in p.items()}
        q1[key][idx] += h
        q2[key][idx] -= h
        fd = (f(q1, X) - f(q2, X)) / (2 * h)
        assert abs(fd - g[key][idx]) <= 1e-6 * max(1.0, abs(fd)), (key, idx, fd, g[key][idx])
    for idx in ((0, 3, 1), (1, 5, 2)):
        x1, x2 = X.copy(), X.copy()
        x1[idx] += h
        x2[idx] -= h
        fd = (f(p, x1) - f(p, x2)) / (2 * h)
        assert abs(fd - g["x"][idx]) <= 1e-6 * max(1.0, abs(fd))


def test_factorised_equals_literal(case):
    A, X, Rl, p = case
    ref = S.sgconv(A, X, Rl, p)
    got = np.stack([fact_fwd(A[b], X[b], Rl[b], p)[0] for b in range(2)])
    np.testing.assert_allclose(got, ref, rtol=1e-12, atol=1e-12)
    dO = np.random.default_rng(2).normal(size=ref.shape)
    _, g = S.sgconv_grads(A, X, Rl, p, dO)
    gs = [fact_bwd(A[b], X[b], Rl[b], p, dO[b]) for b in range(2)]
    for k in ("M1", "b1", "M2", "b2", "M3", "b3"):
        np.testing.assert_allclose(sum(x[k] for x in gs), g[k], rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(np.stack([x["x"] for x in gs]), g["x"], rtol=1e-10, atol=1e-12)


def test_param_layout_matches_library():
    from snd_vae_amd import _lib
    from snd_vae_amd.sg import sg_param_shapes
    for f, hid in ((1, (20, 20, 20)), (20, (50, 50, 50)), (3, (4, 5, 6))):
        n = sum(int(np.prod(s)) for _, s in sg_param_shapes(f, hid))
        assert _lib.lib().snd_sg_param_count(f, *hid) == n


def test_sgjoint_oracle_finite_differences():
    """oracle.ref_sg.sgjoint_forward_backward (the whole SG-joint model in float64 torch
    ops, autograd gradients) against central differences of its own cost on a small
    case, and its decoder half against the GCN oracle's (ref_torch.decoder_losses is
    shared with the node/graph-latent oracle)."""
    import numpy as np
    import torch

    from oracle import ref_sg as RS
    from snd_vae_amd.config import sgjoint
    from snd_vae_amd.data import sgjoint_batch
    from snd_vae_amd.params import init_blocks
    cfg = sgjoint(8, 16, g_hidden=8, latent=4, sampling_num=2, sg_conv_hidden=((3, 4, 5), (4, 3, 6)),
                  mean_degree=3.0, s_d_channel=(5, 4, 3), n_d_channel=(5, 4))
    b = sgjoint_batch(cfg, 2, seed=1)
    n, B, S = 8, 2, 2
    trees = np.zeros((B * S, n, n))
    rp, ci = b.tree_rowptr.astype(np.int64), b.tree_colidx.astype(np.int64)
    for r in range(B * S * n):
        trees[r // n, r % n, ci[rp[r]:rp[r + 1]] % n] = 1.0
    ins = (trees, b.features.reshape(B * S, n, -1), b.rel, np.stack([b.dense_adj(g) for g in range(B)]),
           b.feature_truth.reshape(B, n, -1), b.spatial_truth.reshape(B, n, -1))
    p = {k: v * 5.0 for k, v in init_blocks(cfg, 3).items()}       # larger weights: non-trivial grads
    eps = np.random.default_rng(2).standard_normal((B * S, cfg.latent))
    losses, g = RS.sgjoint_forward_backward(p, *ins, eps, cfg)
    rng = np.random.default_rng(0)

    def cost(q):
        t = {k: torch.tensor(v) for k, v in q.items()}
        tt = lambda a: torch.tensor(np.asarray(a, np.float64))
        c, _ = RS.sgjoint_loss_torch(t, tt(ins[0]), tt(ins[1]), tt(ins[2]), tt(ins[3]), tt(ins[4]),
                                     tt(ins[5]), tt(eps), cfg)
        return float(c)
    for k in ("enc.sg0", "enc.sg1", "enc.Wh", "enc.Wms", "dec.Wp", "dec.K1"):
        for _ in range(3):
            idx = tuple(rng.integers(0, d) for d in p[k].shape)
            h = 1e-6
            qp = {kk: vv.copy() for kk, vv in p.items()}
            qm = {kk: vv.copy() for kk, vv in p.items()}
            qp[k][idx] += h
            qm[k][idx] -= h
            fd = (cost(qp) - cost(qm)) / (2 * h)
            assert abs(fd - g[k][idx]) <= 1e-6 + 1e-5 * abs(fd), (k, idx, fd, g[k][idx])
    assert np.isfinite(losses["cost"])
