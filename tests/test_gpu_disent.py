"""Disentangled-model pieces (csrc/snd_disent.hip) vs the float64
oracle (oracle/ref_disent.py): the e2e edge-to-edge filter (`layers.py:431-450`,
k_h = N as `model.py:196`) forward and backward, and the latent regularisers of
every model_type branch of `optimizer.py:159-190` (KL, the 'disentangled_C'
capacity gate on both sides, DIP, total correlation) with gradients through the
reparameterised sample.  fp32 kernels: within 1e-5 of each block's max-abs."""
import numpy as np
import pytest
import torch

from oracle import ref_disent as RD

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu(lib_built):
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm device")


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


def cu(a):
    return torch.from_numpy(np.ascontiguousarray(a, np.float32)).cuda()


@pytest.mark.parametrize("B,N,C,O", [(2, 25, 8, 50), (3, 24, 16, 20), (1, 50, 4, 10), (2, 7, 3, 5)])
def test_e2e_fwd_bwd(B, N, C, O):
    from snd_vae_amd import disent
    rng = np.random.default_rng(B * N + C)
    x = rng.standard_normal((B, N, N, C)).astype(np.float32)
    w = (0.02 * rng.standard_normal((N, C, O))).astype(np.float32)   # truncated_normal(0.02), layers.py:434
    b = rng.standard_normal(O).astype(np.float32)
    out = disent.e2e(cu(x), cu(w), cu(b)).cpu().numpy()
    assert rel(out, RD.e2e(x, w, b)) < 1e-5
    dout = rng.standard_normal(out.shape).astype(np.float32)
    dx, dw, db = disent.e2e_bwd(cu(x), cu(w), cu(dout))
    rx, rw, rb = RD.e2e_grads(x, w, b, dout)
    assert rel(dx.cpu().numpy(), rx) < 1e-5
    assert rel(dw.cpu().numpy(), rw) < 1e-5
    assert rel(db.cpu().numpy(), rb) < 1e-5


CONFIGS = [
    ("kl", {"w_kl": 0.7}),
    ("capacity on", {"cap_gamma": 2.0, "cap_c": 0.01}),
    ("capacity off", {"cap_gamma": 2.0, "cap_c": 50.0}),
    ("dip", {"w_kl": 1.0, "w_dip": 0.3, "lambda_od": 10.0, "lambda_d": 100.0}),
    ("tc", {"w_kl": 0.5, "w_tc": 10.0}),
]


@pytest.mark.parametrize("B,L", [(10, 16), (50, 100), (3, 5)])
@pytest.mark.parametrize("name,kw", CONFIGS)
def test_latent_reg(B, L, name, kw):
    from snd_vae_amd import disent
    rng = np.random.default_rng(B + L)
    mu = (0.5 * rng.standard_normal((B, L))).astype(np.float32)
    s = (0.3 * rng.standard_normal((B, L))).astype(np.float32)
    eps = rng.standard_normal((B, L)).astype(np.float32)
    z = (mu + eps * np.exp(s)).astype(np.float32)
    # the oracle with the sample exactly as the kernel sees it: eps' = (z - mu) e^-s
    eps64 = (z.astype(np.float64) - mu) * np.exp(-s.astype(np.float64))
    v, dmu, ds = disent.latent_reg(cu(mu), cu(s), cu(z), **kw)
    ref = RD.group_reg(mu, s, z, **kw)
    val, rdmu, rds = RD.group_reg_torch(mu, s, eps64, **kw)
    assert v["kl"] == pytest.approx(ref["kl"], rel=1e-6, abs=1e-9)
    assert v["term"] == pytest.approx(ref["term"], rel=1e-5, abs=1e-7)
    assert v["term"] == pytest.approx(val, rel=1e-5, abs=1e-7)
    assert rel(dmu.cpu().numpy(), rdmu) < 1e-5 or np.abs(rdmu).max() == 0
    assert rel(ds.cpu().numpy(), rds) < 1e-5 or np.abs(rds).max() == 0
    if name == "capacity off":
        assert float(dmu.abs().max()) == 0.0 and v["term"] == 0.0


@pytest.mark.parametrize("mt", ["base", "disentangled", "disentangled_C", "NED-VAE-IP", "beta-TCVAE"])
def test_disentangled_cost_overall_loss(mt):
    """optimizer.py:146-203: cost = adj + node + spatial + the model_type's regulariser;
    overall_loss in the reference order [cost, spatial, adj, node, kl_g, kl_s, kl_sg]."""
    from snd_vae_amd import disent
    rng = np.random.default_rng(11)
    groups, ref_groups = {}, {}
    for g, (B, L) in {"s": (4, 6), "g": (4, 5), "sg": (8, 7)}.items():
        mu = (0.4 * rng.standard_normal((B, L))).astype(np.float32)
        s = (0.2 * rng.standard_normal((B, L))).astype(np.float32)
        z = (mu + rng.standard_normal((B, L)) * np.exp(s)).astype(np.float32)
        groups[g] = (cu(mu), cu(s), cu(z))
        ref_groups[g] = (mu, s, z)
    mse = {"spatial_cost": 0.08, "adj_cost": 0.7, "node_cost": 0.09}
    c = RD.capacity(5500, 25.0, 1000, 100000)
    loss, grads = disent.disentangled_cost(mt, groups, mse, beta=1.5, gamma=2.0, c=c)
    w = RD.model_type_groups(mt, 1.5, 2.0, c)
    reg = sum(RD.group_reg(*ref_groups[g], **kw)["term"] for g, kw in w.items())
    assert loss[0] == pytest.approx(0.87 + reg, rel=1e-5)
    assert loss[1:4] == pytest.approx([0.08, 0.7, 0.09])
    kls = {g: RD.kl(*ref_groups[g][:2]) for g in ("s", "g", "sg")}
    if mt == "base":
        assert len(loss) == 5 and loss[4] == pytest.approx(kls["sg"], rel=1e-6)
    else:
        assert loss[4:] == pytest.approx([kls["g"], kls["s"], kls["sg"]], rel=1e-6)
    assert set(grads) == set(w)


@pytest.mark.parametrize("B,N,D,hidden", [(2, 25, 6, (50, 20)), (3, 24, 4, (50, 20)), (1, 9, 3, (7, 5, 4))])
def test_structure_decoder(B, N, D, hidden):
    """The e2e structure decoder (model.py:193-208) + CE (optimizer.py:142-144) and its
    backward against the literal torch float64 graph."""
    from snd_vae_amd import disent
    rng = np.random.default_rng(N + D)
    z = rng.standard_normal((B, N, D)).astype(np.float32)
    adj = np.zeros((B, N, N), np.float32)
    for b in range(B):
        a = (rng.random((N, N)) < 0.2).astype(np.float32)
        a = np.triu(a, 1)
        adj[b] = a + a.T
    cin, layers = 2 * D, []
    for h in hidden:
        layers.append({"gamma": (1 + 0.1 * rng.standard_normal(cin)).astype(np.float32),
                       "beta": (0.1 * rng.standard_normal(cin)).astype(np.float32),
                       "w": (0.3 / np.sqrt(N * cin) * rng.standard_normal((N, cin, h))).astype(np.float32),
                       "b": (0.1 * rng.standard_normal(h)).astype(np.float32)})
        cin = h
    head = {"gamma": (1 + 0.1 * rng.standard_normal(cin)).astype(np.float32),
            "beta": (0.1 * rng.standard_normal(cin)).astype(np.float32),
            "w": (0.5 * rng.standard_normal((cin, 2))).astype(np.float32),
            "b": (0.1 * rng.standard_normal(2)).astype(np.float32)}
    ce, correct, dz, grads, hg = disent.structure_decoder(
        cu(z), cu(adj), [{k: cu(v) for k, v in l.items()} for l in layers], {k: cu(v) for k, v in head.items()})
    rce, rcorrect, rdz, rgrads, rhg = RD.structure_decoder_grads(z, adj, layers, head)
    assert ce == pytest.approx(rce, rel=1e-5)
    assert abs(correct - rcorrect) <= 2
    assert rel(dz.cpu().numpy(), rdz) < 1e-4
    for g, rg in zip(grads, rgrads):
        for k in ("gamma", "beta", "w", "b"):
            assert rel(g[k].cpu().numpy(), rg[k]) < 1e-4, k
    for k in ("gamma", "beta", "w", "b"):
        assert rel(hg[k].cpu().numpy(), rhg[k]) < 1e-4, k
