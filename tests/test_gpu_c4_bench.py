"""C4 at the benchmarked shape against the float64 oracle, over three Adam steps.

bench.py's C4 workload: tref(4096, 64) (graph latent + model_joint decoders), B = 8
graphs of synthetic_batch seed 1000, the weights of init seed 0, TF1 Adam FUSED into
the two big weight-gradient streams (snd_plan_fuse_adam: enc.Wh inside tref_head_bwd,
dec.Wp inside tref_proj_bwd) exactly as the bench runs it.  Every row slot 0..7 of
the head / projection streams is therefore exercised, and the fused 54 M-parameter
update meets the oracle (`model.py:113-115`, `model_joint.py:97`,
`optimizer.py:125,197`, `main.py:315-331`).

After each step the loss terms, every parameter block and both Adam moments are
compared with the oracle's own three steps (oracle.ref_numpy.forward_backward with
row_chunk + adam_tf1, the same injected eps).  Measured errors are written to
gpurun_out/parity_errors.jsonl (DESIGN §3 records them).

Tolerances.  Parameters move by ~lr per step whatever the gradient's size (Adam
normalises), so an element whose gradient is tiny and sign-ambiguous in fp32 moves
the other way: parameters are compared in units of the learning rate (the bulk: the
99.9th percentile of |p - p_ref| / lr; every element: the Adam step bound).  Moments
are compared block-wise against max-abs, as gradients are.
"""
import json
import os

import numpy as np
import pytest
import torch

from oracle import ref_numpy as R
from snd_vae_amd.config import tref
from snd_vae_amd.data import synthetic_batch
from snd_vae_amd.params import init_blocks

pytestmark = pytest.mark.gpu
TERMS = ("cost", "spatial_cost", "adj_cost", "node_cost", "kl")
STEPS = 3
# (loss rel, moment max-abs rel, params: p99.9 / lr per step, max / lr per step)
TOL = {"f32": (1e-5, 2e-4, 0.05, 2.5), "bf16": (2e-2, 1e-1, 1.0, 2.5)}
_REF = {}


@pytest.fixture(scope="module", autouse=True)
def _gpu(lib_built):
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm device")


def log_errors(rec):
    os.makedirs("gpurun_out", exist_ok=True)
    with open(os.path.join("gpurun_out", "parity_errors.jsonl"), "a") as f:
        f.write(json.dumps(rec) + "\n")


def block_err(g, ref):
    return float(np.abs(g - ref).max() / max(np.abs(ref).max(), 1e-30))


def oracle_steps(cfg, batch, p0, eps):
    """The reference's three train steps (main.py:315-331) in float64, with the state
    after each step."""
    key = (cfg.n_nodes, batch.n_graphs)
    if key in _REF:
        return _REF[key]
    adj = [batch.sparse_adj(b) for b in range(batch.n_graphs)]
    p = {k: np.array(v, np.float64) for k, v in p0.items()}
    m = {k: np.zeros_like(v) for k, v in p.items()}
    v = {k: np.zeros_like(x) for k, x in p.items()}
    hist = []
    for t in range(1, STEPS + 1):
        losses, grads, _ = R.forward_backward(p, adj, batch.features, batch.feature_truth,
                                              batch.spatial_truth, eps[t - 1].astype(np.float64),
                                              cfg, row_chunk=1024)
        R.adam_tf1(p, grads, m, v, t, cfg.learning_rate, cfg.adam_beta1, cfg.adam_beta2,
                   cfg.adam_eps)
        hist.append((losses, {k: x.copy() for k, x in p.items()},
                     {k: x.copy() for k, x in m.items()}, {k: x.copy() for k, x in v.items()}))
    _REF[key] = hist
    return hist


@pytest.mark.timeout(900)
@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_c4_bench_batch_vs_oracle(dtype):
    from snd_vae_amd.model import DeviceBatch, SGCNModelVAE
    from snd_vae_amd.optimizer import OptimizerVAE
    cfg = tref(4096, 64)
    B = 8
    batch = synthetic_batch(cfg, B, seed=1000)          # bench.py run_workload, rank 0
    p0 = {k: v.astype(np.float32).astype(np.float64) for k, v in init_blocks(cfg, 0).items()}
    rng = np.random.default_rng(9)
    eps = [rng.standard_normal((B, cfg.latent)).astype(np.float32) for _ in range(STEPS)]
    hist = oracle_steps(cfg, batch, p0, eps)

    model = SGCNModelVAE(cfg, B, dtype=dtype, blocks=p0)
    opt = OptimizerVAE(model, fuse_adam=True)            # bench.py: fused by default
    assert opt.fused
    db = DeviceBatch(batch)
    ltol, mtol, ptol, pmax = TOL[dtype]
    lr = cfg.learning_rate
    fails = []
    for t in range(STEPS):
        opt.step(db, torch.from_numpy(eps[t]).cuda())
        torch.cuda.synchronize()
        rl, rp, rm, rv = hist[t]
        got = opt.loss_dict()
        rec = {"test": "c4_bench_batch", "dtype": dtype, "step": t + 1, "loss_rel": {},
               "param_p999_lr": {}, "param_max_lr": {}, "m_err": {}, "v_err": {}}
        for k in TERMS:
            e = abs(got[k] - rl[k]) / max(abs(rl[k]), 1e-30)
            rec["loss_rel"][k] = e
            if e > ltol:
                fails.append((t + 1, "loss", k, got[k], rl[k]))
        gp = model.blocks()
        gm, gv = opt.state_blocks()
        for k in rp:
            d = np.abs(np.asarray(gp[k], np.float64) - rp[k]) / lr
            p999 = float(np.quantile(d, 0.999)) if d.size > 1 else float(d.max())
            rec["param_p999_lr"][k] = p999
            rec["param_max_lr"][k] = float(d.max())
            if p999 > ptol * (t + 1) or d.max() > pmax * (t + 1):
                fails.append((t + 1, "param", k, p999, float(d.max())))
            for name, a, r in (("m", gm[k], rm[k]), ("v", gv[k], rv[k])):
                e = block_err(np.asarray(a, np.float64), r)
                rec[f"{name}_err"][k] = e
                if e > mtol:
                    fails.append((t + 1, name, k, e))
        log_errors(rec)
    assert opt.global_step == STEPS
    assert not fails, fails[:12]
