"""The disentangled SND-VAE (model.py:19-222 + optimizer.py:123-203; SURVEY.md §8f
rank 4) assembled over the C ABI (snd_vae_amd/disent_model.py) against the literal
float64 oracle (oracle/ref_disent_model.py, torch autograd) at the reference's
synthetic2 widths (N = 25, sampling_num = 10).

Tolerances (DESIGN.md §3, fp32 path): ELBO terms 1e-5 relative (1e-7 absolute for
the KLs, whose terms cancel); a gradient block within max(2e-4, 10 e32) of its max-abs,
where e32 is the same oracle's own fp32 error on that block (the conditioning: the
total-correlation and DIP terms reach some bias / BN gradients through cancellation that
costs the fp32 oracle itself up to a few %); parameters after 3 TF1-Adam steps within
5 % of the step size; the e2e accuracy count exact.
"""
import numpy as np
import pytest
import torch

from oracle import ref_disent_model as RM
from oracle import ref_numpy as R

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


def case(B, n=25, S=10, seed=3, **kw):
    from snd_vae_amd.config import sgjoint
    from snd_vae_amd.data import sgjoint_batch
    from snd_vae_amd.disent_model import DisentangledConfig
    cfg = DisentangledConfig(n_nodes=n, sampling_num=S, **kw)
    b = sgjoint_batch(sgjoint(n, 16, mean_degree=4.0, sampling_num=S), B, seed=seed)
    ins = {"x": b.feature_truth.reshape(B, n, -1), "spatial": b.spatial_truth.reshape(B, n, 2),
           "adj": np.stack([b.dense_adj(g) for g in range(B)]), "x_sg": b.features.reshape(B * S, n, -1),
           "trees": dense_trees(b), "rel": b.rel}
    return cfg, b, ins


def draw_eps(rng, cfg, B):
    return {"s": rng.standard_normal((B, cfg.s_latent)).astype(np.float32),
            "g": rng.standard_normal((B, cfg.g_latent)).astype(np.float32),
            "sg": rng.standard_normal((B * cfg.sampling_num, cfg.sg_latent)).astype(np.float32)}


def compare(got, ref, g, rg, tag, p=None, ins=None, eps=None, cfg=None):
    for k, v in got.items():
        if k == "correct":
            assert v == ref[k], (tag, k, v, ref[k])
        else:
            assert v == pytest.approx(ref[k], rel=1e-5, abs=1e-7), (tag, k, v, ref[k])
    g32 = RM.disent_forward_backward(p, ins, eps, cfg, dtype=torch.float32)[1]
    for k in rg:
        scale = max(np.abs(rg[k]).max(), 1e-30)
        err = np.abs(g[k] - rg[k]).max() / scale
        e32 = np.abs(g32[k] - rg[k]).max() / scale
        assert err < max(2e-4, 10 * e32), (tag, k, err, e32)


@pytest.mark.parametrize("model_type", ["disentangled", "beta-TCVAE"])
def test_disentangled_steps_vs_oracle(model_type):
    from snd_vae_amd.disent_model import DeviceDisentBatch, DisentangledSGCNModelVAE, init_blocks
    B = 2
    cfg, b, ins = case(B, model_type=model_type)
    p = {k: v.astype(np.float32).astype(np.float64) for k, v in init_blocks(cfg, 0).items()}
    model = DisentangledSGCNModelVAE(cfg, B, blocks=p)
    db = DeviceDisentBatch(b)
    rng = np.random.default_rng(5)
    m = {k: np.zeros_like(v) for k, v in p.items()}
    v = {k: np.zeros_like(x) for k, x in p.items()}
    # three Adam steps where every gradient is well conditioned; one under the TC term (an
    # element whose fp32 gradient sign is noise moves by +-lr there, as it would in TF)
    for t in range(1, 4 if model_type == "disentangled" else 2):
        eps = draw_eps(rng, cfg, B)
        got = model.step(db, {k: torch.from_numpy(e).cuda() for k, e in eps.items()})
        e64 = {k: e.astype(np.float64) for k, e in eps.items()}
        ref, rg = RM.disent_forward_backward(p, ins, e64, cfg)
        compare(got, ref, model.grad_blocks(), rg, (model_type, t), p, ins, e64, cfg)
        R.adam_tf1(p, rg, m, v, t, cfg.learning_rate, cfg.adam_beta1, cfg.adam_beta2, cfg.adam_eps)
        if model_type != "disentangled":
            continue    # first-step Adam moves every element by ~lr sign(g): noise-signed ones differ
        blocks = model.blocks()
        for k in p:     # Adam normalises each update to ~lr: compare against the step size
            assert np.abs(blocks[k] - p[k]).max() < 0.05 * t * cfg.learning_rate, (t, k)


@pytest.mark.parametrize("model_type,kw", [("NED-VAE-IP", {}), ("disentangled_C", {"capacity": 0.5, "gamma": 2.0}),
                                           ("base", {}), ("geoGCN", {"beta": 4.0})])
def test_model_type_gradients(model_type, kw):
    """One step of each remaining optimizer.py:159-190 branch, weights scaled up so the
    regularisers' gradients are not lost under the reconstruction terms."""
    from snd_vae_amd.disent_model import DeviceDisentBatch, DisentangledSGCNModelVAE, init_blocks
    B = 4
    cfg, b, ins = case(B, S=3, seed=11, model_type=model_type, **kw)
    big = lambda k: k.endswith(("/Matrix", "/w", "/w1"))
    p = {k: (v * 4.0 if big(k) else v).astype(np.float32).astype(np.float64) for k, v in init_blocks(cfg, 1).items()}
    model = DisentangledSGCNModelVAE(cfg, B, blocks=p)
    eps = draw_eps(np.random.default_rng(9), cfg, B)
    got = model.step(DeviceDisentBatch(b), {k: torch.from_numpy(e).cuda() for k, e in eps.items()})
    e64 = {k: e.astype(np.float64) for k, e in eps.items()}
    ref, rg = RM.disent_forward_backward(p, ins, e64, cfg)
    compare(got, ref, model.grad_blocks(), rg, model_type, p, ins, e64, cfg)
