"""Load the committed golden fixtures (tests/golden/*.npz, written by
tests/golden/make_golden.py from the float64 oracle) and compare against them.

Blocks larger than make_golden.BIG are stored as every SAMPLE-th element plus
the float64 norm; their initial values are regenerated from the seed and
checked against the stored sum / sum of squares.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")
sys.path.insert(0, GOLDEN)

import make_golden as MG  # noqa: E402

from snd_vae_amd.data import GraphBatch  # noqa: E402

NAMES = tuple(MG.CASES)


def load(name):
    """-> (npz, cfg, GraphBatch, p0 dict of float64 blocks)."""
    z = np.load(os.path.join(GOLDEN, name + ".npz"))
    topology = str(z["topology"]) if "topology" in z.files else "tscale"
    n, d, B = int(z["n"]), int(z["d"]), int(z["B"])
    cfg = MG.fixture_config(topology, n, d, float(z["kbar"]))
    batch = GraphBatch(B, n, z["rowptr"], z["colidx"], z["features"], z["feature_truth"],
                       z["spatial_truth"])
    p0 = {k[3:]: z[k] for k in z.files if k.startswith("p0/")}
    big = [k[6:] for k in z.files if k.startswith("p0sum/")]
    if big:
        regen, _ = MG.initial_params(cfg, int(z["seed"]))
        for k in big:
            v = regen[k]
            s = z["p0sum/" + k]
            assert abs(v.sum() - s[0]) <= 1e-9 * max(1.0, abs(s[0])), k
            assert abs((v * v).sum() - s[1]) <= 1e-9 * s[1], k
            p0[k] = v
    return z, cfg, batch, p0


def block_error(z, prefix, k, got):
    """Max-abs error of block k relative to the reference max-abs (sampled for big blocks).

    prefix: e.g. "s0/grad" or "p_final".  Returns (err, norm_err or None).
    """
    got = np.asarray(got)
    if f"{prefix}/{k}" in z.files:
        ref = z[f"{prefix}/{k}"]
        return np.abs(got - ref).max() / max(np.abs(ref).max(), 1e-30), None
    ref = z[f"{prefix}sample/{k}"]
    g = got.reshape(-1)[::MG.SAMPLE]
    err = np.abs(g - ref).max() / max(np.abs(ref).max(), 1e-30)
    nref = float(z[f"{prefix}norm/{k}"])
    return err, abs(np.linalg.norm(got) - nref) / max(nref, 1e-30)


def max_abs_diff(z, prefix, k, got):
    got = np.asarray(got)
    if f"{prefix}/{k}" in z.files:
        return np.abs(got - z[f"{prefix}/{k}"]).max()
    return np.abs(got.reshape(-1)[::MG.SAMPLE] - z[f"{prefix}sample/{k}"]).max()
