"""Generate the golden fixtures from the float64 oracle (oracle/ref_numpy.py).

Parity is unpinned against TensorFlow (not installable here; the reference
ships no tests or logged values), so these vectors are the oracle's own
outputs for seeded inputs, committed so GPU tests compare against fixed data.
Each fixture: CSR of B seeded RGG graphs, features/targets, float32-rounded
initial parameters, per-step eps, and for 3 TF1-Adam steps the loss terms,
all gradients and the parameters after the step.

Blocks above BIG elements (the graph-latent heads / projection, up to 340 K
floats at C1) are not stored whole: the fixture keeps their initial values'
float64 sum and sum of squares (``p0sum/<k>``; tests regenerate them with
``initial_params``), and for gradients and final parameters every SAMPLE-th
element plus the float64 norm.

    python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import ref_numpy as R  # noqa: E402
from snd_vae_amd.config import PRESETS, tref, tscale  # noqa: E402
from snd_vae_amd.data import synthetic_batch  # noqa: E402
from snd_vae_amd.params import init_blocks  # noqa: E402

CASES = {
    "tscale_n25_d16": dict(topology="tscale", n=25, d=16, kbar=6.0, B=2, seed=11),
    "tscale_n200_d16": dict(topology="tscale", n=200, d=16, kbar=8.0, B=2, seed=0),
    # graph latent (model.py:113-115 + model_joint.py:97); C1 = BASELINE configs[0]
    "tref_n25_d16": dict(topology="tref", n=25, d=16, kbar=6.0, B=3, seed=21),
    "tref_c1_n200_d16": dict(topology="C1", n=200, d=16, kbar=8.0, B=2, seed=5),
}
STEPS = 3
BIG = 20000
SAMPLE = 61


def fixture_config(topology, n, d, kbar):
    if topology == "tscale":
        return tscale(n, d, mean_degree=kbar)
    if topology == "C1":
        return PRESETS["C1"]
    return tref(n, d, mean_degree=kbar)


def initial_params(cfg, seed):
    """Seeded initial parameters: reference initialisers, perturbed, float32-rounded."""
    rng = np.random.default_rng(seed + 100)
    p0 = init_blocks(cfg, seed)
    # perturb BN / biases away from 1/0 so their gradients are exercised
    p0 = {k: (v + 0.05 * rng.standard_normal(v.shape)) for k, v in p0.items()}
    return {k: v.astype(np.float32).astype(np.float64) for k, v in p0.items()}, rng


def make(name, topology, n, d, kbar, B, seed):
    cfg = fixture_config(topology, n, d, kbar)
    batch = synthetic_batch(cfg, B, seed=seed)
    p0, rng = initial_params(cfg, seed)
    eshape = (B, cfg.latent) if cfg.topology == "tref" else (B * n, d)
    eps = [rng.standard_normal(eshape).astype(np.float32) for _ in range(STEPS)]
    adj = [batch.dense_adj(b) for b in range(B)]
    p, m, v, hist = R.train_steps(p0, adj, batch.features, batch.feature_truth,
                                  batch.spatial_truth, [e.astype(np.float64) for e in eps],
                                  cfg, STEPS)
    out = dict(topology=topology, n=n, d=d, B=B, kbar=kbar, seed=seed, rowptr=batch.rowptr,
               colidx=batch.colidx, features=batch.features, feature_truth=batch.feature_truth,
               spatial_truth=batch.spatial_truth, eps=np.stack(eps))

    def put(prefix, k, val):
        if val.size > BIG:
            flat = val.reshape(-1)
            out[f"{prefix}sample/{k}"] = flat[::SAMPLE]
            out[f"{prefix}norm/{k}"] = np.float64(np.linalg.norm(flat))
        else:
            out[f"{prefix}/{k}"] = val

    for k, val in p0.items():
        if val.size > BIG:
            out["p0sum/" + k] = np.array([val.sum(), (val * val).sum()])
        else:
            out["p0/" + k] = val
    for t, (losses, grads) in enumerate(hist):
        for k in ("cost", "spatial_cost", "adj_cost", "node_cost", "kl", "acc"):
            out[f"s{t}/loss/{k}"] = np.float64(losses[k])
        for k, g in grads.items():
            put(f"s{t}/grad", k, g)
    # params after all steps
    for k, val in p.items():
        put("p_final", k, val)
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)


if __name__ == "__main__":
    for name, kw in CASES.items():
        make(name, **kw)
        print("wrote", name)
