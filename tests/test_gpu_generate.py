"""snd_generate (eval / reconstruction / sampling) vs the float64 oracle.

Reference: generate_new / generate_new_train (`main.py:358-469`), get_random_z
(`model.py:163-169`), generated_adj = argmax over (0, L_ij) / (1, 0) on the
diagonal (`model.py:205-208`), accuracy (`main.py:334`).  fp32 engine: 1e-5
relative on the continuous outputs; generated_adj bit-exact except on pairs
whose float64 logit lies within fp32 rounding of 0.
"""
import numpy as np
import pytest
import torch

from oracle import ref_numpy as R
from snd_vae_amd.config import tref, tscale
from snd_vae_amd.data import synthetic_batch
from snd_vae_amd.params import init_blocks

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu(lib_built):
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm device")


CFGS = {"tscale": tscale(96, 16, mean_degree=6.0),
        "tref": tref(96, 16, mean_degree=6.0)}


def setup(name, B=2, dtype="f32"):
    from snd_vae_amd.model import DeviceBatch, SGCNModelVAE
    cfg = CFGS[name]
    batch = synthetic_batch(cfg, B, seed=21)
    p0 = {k: v.astype(np.float32).astype(np.float64) for k, v in init_blocks(cfg, 3).items()}
    model = SGCNModelVAE(cfg, B, dtype=dtype, blocks=p0)
    rh = B if cfg.topology == "tref" else B * cfg.n_nodes
    return cfg, batch, p0, model, DeviceBatch(batch), rh


def close(got, ref, rtol=1e-5):
    got = got.double().cpu().numpy() if torch.is_tensor(got) else got
    err = np.abs(got - ref).max()
    assert err <= rtol * max(1.0, np.abs(ref).max()), err


def adj_check(gen, J, n, rel=1e-5):
    pred, Lg = R.generated_adj(J, n)
    got = gen.cpu().numpy()
    bad = got != pred
    amb = np.abs(Lg) <= rel * np.abs(Lg).max()
    assert not np.any(bad & ~amb), int((bad & ~amb).sum())
    return pred


@pytest.mark.parametrize("name", ["tscale", "tref"])
def test_sample_and_mean_match_oracle(name):
    from snd_vae_amd.model import adj_accuracy
    cfg, batch, p0, model, db, rh = setup(name)
    adjs = [batch.dense_adj(b) for b in range(2)]
    eps = np.random.default_rng(7).standard_normal((rh, cfg.latent)).astype(np.float32)
    for mode, e in (("sample", eps), ("mean", np.zeros_like(eps))):
        out = model.generate(db, mode=mode, eps=torch.from_numpy(e) if mode == "sample" else None)
        ref, _, cache = R.forward_backward(p0, adjs, batch.features, batch.feature_truth,
                                           batch.spatial_truth, e.astype(np.float64), cfg,
                                           want_grads=False)
        close(out["z_mean"], cache["mu"])
        close(out["z"], cache["z"])
        close(out["generated_spatial"], cache["Shat"])
        close(out["generated_node_feat"], cache["Xhat"])
        pred = adj_check(out["generated_adj"], cache["J"], cfg.n_nodes)
        acc = adj_accuracy(out["generated_adj"], db)
        assert abs(acc - ref["acc"]) <= 1e-3, (acc, ref["acc"])
        A = np.stack(adjs)
        assert acc == float((out["generated_adj"].cpu().numpy() == A).mean())
        del pred


@pytest.mark.parametrize("name", ["tscale", "tref"])
def test_prior_and_given(name):
    cfg, batch, p0, model, db, rh = setup(name)
    z = np.random.default_rng(9).standard_normal((rh, cfg.latent)).astype(np.float32)
    J, S, X = R.decode(p0, z.astype(np.float64), cfg)
    for mode, kw in (("prior", {"eps": torch.from_numpy(z)}), ("given", {"z": torch.from_numpy(z)})):
        out = model.generate(None, mode=mode, **kw)
        close(out["z"], z)
        close(out["generated_spatial"], S)
        close(out["generated_node_feat"], X)
        adj_check(out["generated_adj"], J, cfg.n_nodes)
    # device Philox prior: standard normal draws, reproducible at the same (seed, step)
    a = model.generate(None, mode="prior", seed=5, step=3)["z"]
    b = model.generate(None, mode="prior", seed=5, step=3)["z"]
    c = model.generate(None, mode="prior", seed=5, step=4)["z"]
    assert torch.equal(a, b) and not torch.equal(a, c)
    assert abs(float(a.mean())) < 0.2 and abs(float(a.std()) - 1.0) < 0.2


def test_bf16_plan_generate_and_params_untouched():
    cfg, batch, p0, model, db, rh = setup("tscale", dtype="bf16")
    before = model.params.clone()
    eps = np.random.default_rng(7).standard_normal((rh, cfg.latent)).astype(np.float32)
    out = model.generate(db, mode="sample", eps=torch.from_numpy(eps))
    assert torch.equal(before, model.params)
    _, _, cache = R.forward_backward(p0, [batch.dense_adj(b) for b in range(2)], batch.features,
                                     batch.feature_truth, batch.spatial_truth,
                                     eps.astype(np.float64), cfg, want_grads=False)
    close(out["generated_spatial"], cache["Shat"], rtol=2e-2)
    pred, _ = R.generated_adj(cache["J"], cfg.n_nodes)
    assert (out["generated_adj"].cpu().numpy() == pred).mean() > 0.99


def test_generate_errors():
    from snd_vae_amd import _lib
    cfg, batch, p0, model, db, rh = setup("tscale")
    with pytest.raises(ValueError):
        model.generate(None, mode="mean")
    with pytest.raises(ValueError):
        model.generate(None, mode="given")
    L = _lib.lib()
    rc = L.snd_generate(model.plan, None, _lib.ptr(model.params), _lib.ptr(model.workspace), 0,
                        None, 0, None, None, _lib.stream_ptr())
    assert rc == -1 and "batch" in _lib.last_error()
