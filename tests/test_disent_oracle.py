"""CPU checks of the disentangled-model oracle (oracle/ref_disent.py): numpy ==
torch on values, torch autograd == finite differences on gradients (SURVEY §8f
rank 4: e2e, layers.py:431-450; the regularisers of optimizer.py:7-58,159-190)."""
import numpy as np
import pytest

from oracle import ref_disent as RD


@pytest.mark.parametrize("B,N,C,O", [(2, 7, 3, 4), (1, 6, 2, 3)])
def test_e2e_numpy_matches_torch_and_fd(B, N, C, O):
    import torch
    rng = np.random.default_rng(N)
    x, w, b = rng.standard_normal((B, N, N, C)), rng.standard_normal((N, C, O)), rng.standard_normal(O)
    ref = RD.e2e(x, w, b)
    got = RD.e2e_torch(torch.tensor(x), torch.tensor(w), torch.tensor(b)).numpy()
    np.testing.assert_allclose(got, ref, rtol=1e-12, atol=1e-12)
    dout = rng.standard_normal(ref.shape)
    dx, dw, db = RD.e2e_grads(x, w, b, dout)
    eps = 1e-6
    for arr, g, idx in ((x, dx, (0, 1, 2, 1)), (w, dw, (2, 1, 3 % O)), (b, db, (1,))):
        a0 = arr[idx]
        arr[idx] = a0 + eps
        fp = (RD.e2e(x, w, b) * dout).sum()
        arr[idx] = a0 - eps
        fm = (RD.e2e(x, w, b) * dout).sum()
        arr[idx] = a0
        assert (fp - fm) / (2 * eps) == pytest.approx(g[idx], rel=1e-6, abs=1e-8)


def test_e2e_is_the_literal_sum():
    """out[b,i,j,o] = 2 b1 + sum_t sum_c w1[t,c,o] (x[i, j+t-p] + x[i+t-p, j]), p = (K-1)//2."""
    rng = np.random.default_rng(3)
    B, N, C, O = 1, 5, 2, 2
    x, w, b = rng.standard_normal((B, N, N, C)), rng.standard_normal((N, C, O)), rng.standard_normal(O)
    p = (N - 1) // 2
    ref = np.zeros((B, N, N, O))
    for i in range(N):
        for j in range(N):
            acc = 2 * b.copy()
            for t in range(N):
                if 0 <= j + t - p < N:
                    acc += x[0, i, j + t - p] @ w[t]
                if 0 <= i + t - p < N:
                    acc += x[0, i + t - p, j] @ w[t]
            ref[0, i, j] = acc
    np.testing.assert_allclose(RD.e2e(x, w, b), ref, rtol=1e-12)


CONFIGS = [
    {"w_kl": 0.7},
    {"cap_gamma": 2.0, "cap_c": 0.05},
    {"cap_gamma": 2.0, "cap_c": 50.0},
    {"w_kl": 1.0, "w_dip": 0.3, "lambda_od": 10.0, "lambda_d": 100.0},
    {"w_kl": 0.5, "w_tc": 10.0},
]


@pytest.mark.parametrize("kw", CONFIGS)
def test_group_reg_numpy_torch_fd(kw):
    rng = np.random.default_rng(7)
    B, L = 6, 4
    mu, s, eps = 0.5 * rng.standard_normal((B, L)), 0.3 * rng.standard_normal((B, L)), rng.standard_normal((B, L))
    z = mu + eps * np.exp(s)
    ref = RD.group_reg(mu, s, z, **kw)["term"]
    val, dmu, ds = RD.group_reg_torch(mu, s, eps, **kw)
    assert val == pytest.approx(ref, rel=1e-12, abs=1e-14)
    h = 1e-6
    for arr, g in ((mu, dmu), (s, ds)):
        for idx in [(0, 0), (3, 2), (5, 3)]:
            a0 = arr[idx]
            arr[idx] = a0 + h
            fp = RD.group_reg(mu, s, mu + eps * np.exp(s), **kw)["term"]
            arr[idx] = a0 - h
            fm = RD.group_reg(mu, s, mu + eps * np.exp(s), **kw)["term"]
            arr[idx] = a0
            assert (fp - fm) / (2 * h) == pytest.approx(g[idx], rel=1e-5, abs=1e-8)


def test_model_type_weights_and_capacity():
    assert RD.model_type_groups("base", beta=2.0) == {"sg": {"w_kl": 2.0}}
    g = RD.model_type_groups("disentangled_C", gamma=3.0, c=0.5)
    assert g["sg"] == {"w_kl": 0.0, "cap_gamma": 3.0, "cap_c": 0.5} and g["s"] == {"w_kl": 1.0}
    assert RD.capacity(0, 25.0, 1000, 100000) == 0.0
    assert RD.capacity(250000, 25.0, 1000, 100000) == 25.0
    assert RD.capacity(5500, 25.0, 1000, 100000) == pytest.approx(25.0 * 1000 / 100000 * 5)
    from snd_vae_amd import disent
    for mt in ("base", "disentangled", "disentangled_C", "NED-VAE-IP", "beta-TCVAE"):
        assert disent.group_weights(mt, 1.5, 2.0, 0.25) == RD.model_type_groups(mt, 1.5, 2.0, 0.25)
    assert disent.capacity(5500, 25.0, 1000, 100000) == RD.capacity(5500, 25.0, 1000, 100000)


def test_structure_decoder_oracle_fd():
    """The literal structure decoder (model.py:193-208 + optimizer.py:142-144): autograd
    gradients against central differences, and the diagonal pairs carry no gradient."""
    rng = np.random.default_rng(2)
    B, N, D = 1, 6, 2
    z = rng.standard_normal((B, N, D))
    a = np.triu((rng.random((N, N)) < 0.4).astype(float), 1)
    adj = (a + a.T)[None]
    layers = [{"gamma": 1 + 0.1 * rng.standard_normal(4), "beta": 0.1 * rng.standard_normal(4),
               "w": 0.3 * rng.standard_normal((N, 4, 3)), "b": 0.1 * rng.standard_normal(3)}]
    head = {"gamma": 1 + 0.1 * rng.standard_normal(3), "beta": 0.1 * rng.standard_normal(3),
            "w": rng.standard_normal((3, 2)), "b": 0.1 * rng.standard_normal(2)}
    import torch
    f = lambda zz: float(RD.structure_decoder_torch(torch.tensor(zz), adj, [{k: torch.tensor(v) for k, v in layers[0].items()}],
                                                   {k: torch.tensor(v) for k, v in head.items()})[0])
    ce, _, dz, _, _ = RD.structure_decoder_grads(z, adj, layers, head)
    assert ce == pytest.approx(f(z), rel=1e-12)
    h = 1e-6
    for idx in [(0, 0, 0), (0, 3, 1), (0, 5, 0)]:
        zp, zm = z.copy(), z.copy()
        zp[idx] += h
        zm[idx] -= h
        assert (f(zp) - f(zm)) / (2 * h) == pytest.approx(dz[idx], rel=1e-5, abs=1e-9)
