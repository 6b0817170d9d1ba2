"""Generate the golden fixtures from the float64 oracle (oracle/ref_numpy.py).

Parity is unpinned against TensorFlow (not installable here; the reference
ships no tests or logged values), so these vectors are the oracle's own
outputs for seeded inputs, committed so GPU tests compare against fixed data.
Each fixture: CSR of B seeded RGG graphs, features/targets, float32-rounded
initial parameters, per-step eps, and for 3 TF1-Adam steps the loss terms,
all gradients and the parameters after the step.

    python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import ref_numpy as R  # noqa: E402
from snd_vae_amd.config import tscale  # noqa: E402
from snd_vae_amd.data import synthetic_batch  # noqa: E402
from snd_vae_amd.params import init_blocks  # noqa: E402

CASES = {
    "tscale_n25_d16": dict(n=25, d=16, kbar=6.0, B=2, seed=11),
    "tscale_n200_d16": dict(n=200, d=16, kbar=8.0, B=2, seed=0),
}
STEPS = 3


def make(name, n, d, kbar, B, seed):
    cfg = tscale(n, d, mean_degree=kbar)
    batch = synthetic_batch(cfg, B, seed=seed)
    rng = np.random.default_rng(seed + 100)
    p0 = init_blocks(cfg, seed)
    # perturb BN / biases away from 1/0 so their gradients are exercised
    p0 = {k: (v + 0.05 * rng.standard_normal(v.shape)) for k, v in p0.items()}
    p0 = {k: v.astype(np.float32).astype(np.float64) for k, v in p0.items()}
    eps = [rng.standard_normal((B * n, d)).astype(np.float32) for _ in range(STEPS)]
    adj = [batch.dense_adj(b) for b in range(B)]
    p, m, v, hist = R.train_steps(p0, adj, batch.features, batch.feature_truth,
                                  batch.spatial_truth, [e.astype(np.float64) for e in eps],
                                  cfg, STEPS)
    out = dict(n=n, d=d, B=B, kbar=kbar, seed=seed, rowptr=batch.rowptr, colidx=batch.colidx,
               features=batch.features, feature_truth=batch.feature_truth,
               spatial_truth=batch.spatial_truth, eps=np.stack(eps))
    for k, val in p0.items():
        out["p0/" + k] = val
    for t, (losses, grads) in enumerate(hist):
        for k in ("cost", "spatial_cost", "adj_cost", "node_cost", "kl", "acc"):
            out[f"s{t}/loss/{k}"] = np.float64(losses[k])
        for k, g in grads.items():
            out[f"s{t}/grad/{k}"] = g
    # params after all steps
    for k, val in p.items():
        out["p_final/" + k] = val
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)


if __name__ == "__main__":
    for name, kw in CASES.items():
        make(name, **kw)
        print("wrote", name)
