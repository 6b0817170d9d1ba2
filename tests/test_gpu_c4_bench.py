"""C4 at the benchmarked shape against the float64 oracle, step by step.

bench.py's C4 workload: tref(4096, 64) (graph latent + model_joint decoders), B = 8
graphs of synthetic_batch seed 1000, the weights of init seed 0, TF1 Adam FUSED into
the two big weight-gradient streams (snd_plan_fuse_adam: enc.Wh inside tref_head_bwd,
dec.Wp inside tref_proj_bwd) exactly as the bench runs it.  Every row slot 0..7 of
the head / projection streams is therefore exercised, and the fused 54 M-parameter
update meets the oracle (`model.py:113-115`, `model_joint.py:97`,
`optimizer.py:125,197`, `main.py:315-331`).

Each step t is checked from the GPU's own state: the oracle (forward_backward with
row_chunk + adam_tf1, float64) takes the parameters and Adam moments the GPU held
before step t, runs step t with the same injected eps, and the GPU's loss terms,
every parameter block and both moments after step t are compared with it.  Step 1 is
the plain from-init comparison; later steps test the carried state (step counter,
bias correction, moments) without the trajectory's own sensitivity to rounding.
Measured errors go to gpurun_out/parity_errors.jsonl (DESIGN §3 records them).

Two schedules:
* the reference learning rate, ONE step: exactly the bench's timed C4 step (bench.py
  times step 1 from a reset state).  At this lr the reference dynamics leave the fp32
  range at step 2 (cost ~4.6e25; Adam's v = g^2 overflows to inf in fp32 -- in TF's
  fp32 graph as here; only a float64 oracle stays finite);
* lr = 1e-6, THREE steps: the same kernels with every step finite.

Tolerances.  Parameters move by ~lr per step whatever the gradient's size (Adam
normalises), so an element whose gradient is near zero and sign-ambiguous in the
computing precision moves the other way (2 lr apart): fp32 -- all but 1e-4 of a
block's elements within 0.05 lr plus 4 fp32 ulps of the parameter (measured: the
worst element of enc.Wh 0.098 lr at step 1); bf16 -- at most 3 % of a block's elements
more than lr/2 apart (measured: 1.0 % of enc.W0, 1.9 % of dec.K1 at step 1), none
more than the Adam step bound 2 lr.  Moments against the block's max-abs, as
gradients: fp32 2e-3 (the decoder's conv1 / conv-bias gradients, sums over B*N = 32768
rows with cancellation: measured 3.4e-4 at step 1, 1.4e-3 for dec.K1 at step 3 of the
lr = 1e-6 schedule); bf16: the loss terms 5x and the moment blocks 2x the error measured
for each (tests/parity_bars.json, tests/parity_bars.py; fallbacks 2e-2 / 1e-1).  Blocks
of at most 32 elements in bf16 (scalar-like bias sums whose terms cancel: dec.bn, ONE
element, measured 0.15 at step 1 and 0.74 at step 2 -- bf16 operands leave only its
order of magnitude) are recorded against the oracle but NOT bounded by it: a bar on
them would be a number, not a check.  What pins them -- and the fused update of every
block -- is the self-consistency check, in every dtype: the GPU's new m and
the old m give the gradient the update used (g = (m' - b1 m) / (1 - b1), TF's float32
coefficients), and v' and the parameters must follow from it and from m', v' by TF1 Adam
to float32 rounding (`self_adam_err`: v within 1e-5 of |v'| + 1e-5 of the block's max,
parameters within 5e-4 lr + 4 ulps; measured, round 5: v 9e-8, parameters 1.25e-4 lr).
"""
import dataclasses

import numpy as np
import pytest
import torch

import parity_bars as PB
from oracle import ref_numpy as R
from snd_vae_amd.config import tref
from snd_vae_amd.data import synthetic_batch
from snd_vae_amd.params import init_blocks

pytestmark = pytest.mark.gpu
TERMS = ("cost", "spatial_cost", "adj_cost", "node_cost", "kl")
STEPS = 3
LOSS_TOL = {"f32": 1e-5, "bf16": 2e-2}
M_TOL = {"f32": 2e-3, "bf16": 1e-1}   # bf16: fallback where parity_bars.json has no entry
EPS32 = float(np.finfo(np.float32).eps)


@pytest.fixture(scope="module", autouse=True)
def _gpu(lib_built):
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm device")


def block_err(g, ref):
    return float(np.abs(g - ref).max() / max(np.abs(ref).max(), 1e-30))


def self_adam(p, m, v, gp, gm, gv, t, lr, b1, b2, eps):
    """(v error, parameter error) of the GPU's step against TF1 Adam applied to the
    gradient its own moments imply; 1.0 = the tolerance."""
    f32 = np.float32
    c1, c2 = float(f32(1) - f32(b1)), float(f32(1) - f32(b2))
    g = (gm - float(f32(b1)) * m) / c1
    sv = float(f32(b2)) * v + c2 * g * g
    ev = float(np.max(np.abs(gv - sv) / (1e-5 * np.abs(sv) + 1e-5 * np.abs(sv).max() + 1e-30)))
    lr_t = lr * np.sqrt(1 - b2 ** t) / (1 - b1 ** t)
    sp = p - lr_t * gm / (np.sqrt(gv) + eps)
    ep = float(np.max(np.abs(gp - sp) / (5e-4 * lr + 4 * EPS32 * np.abs(p))))
    return ev, ep


@pytest.mark.timeout(900)
@pytest.mark.parametrize("lr,steps", [(None, 1), (1e-6, STEPS)])
@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_c4_bench_batch_vs_oracle(dtype, lr, steps):
    from snd_vae_amd.model import DeviceBatch, SGCNModelVAE
    from snd_vae_amd.optimizer import OptimizerVAE
    cfg = tref(4096, 64)
    if lr is not None:
        cfg = dataclasses.replace(cfg, learning_rate=lr)
    B = 8
    batch = synthetic_batch(cfg, B, seed=1000)          # bench.py run_workload, rank 0
    adj = [batch.sparse_adj(b) for b in range(B)]
    p0 = {k: v.astype(np.float32).astype(np.float64) for k, v in init_blocks(cfg, 0).items()}
    rng = np.random.default_rng(9)
    eps = [rng.standard_normal((B, cfg.latent)).astype(np.float32) for _ in range(steps)]

    model = SGCNModelVAE(cfg, B, dtype=dtype, blocks=p0)
    opt = OptimizerVAE(model, fuse_adam=True)            # bench.py: fused by default
    assert opt.fused and opt.lr == cfg.learning_rate
    db = DeviceBatch(batch)
    lr = cfg.learning_rate
    fails = []
    for t in range(1, steps + 1):
        # the GPU's state before step t, as the oracle's starting point
        p = {k: np.asarray(v, np.float64) for k, v in model.blocks().items()}
        m, v = opt.state_blocks()
        m = {k: np.asarray(x, np.float64) for k, x in m.items()}
        v = {k: np.asarray(x, np.float64) for k, x in v.items()}
        p0s, m0s, v0s = ({k: x.copy() for k, x in d.items()} for d in (p, m, v))   # adam_tf1 updates in place
        opt.step(db, torch.from_numpy(eps[t - 1]).cuda())
        torch.cuda.synchronize()
        rl, rg, _ = R.forward_backward(p, adj, batch.features, batch.feature_truth,
                                       batch.spatial_truth, eps[t - 1].astype(np.float64),
                                       cfg, row_chunk=1024)
        R.adam_tf1(p, rg, m, v, t, lr, cfg.adam_beta1, cfg.adam_beta2, cfg.adam_eps)
        got = opt.loss_dict()
        bars = PB.Bars(f"c4_bench_{'reflr' if steps == 1 else 'lr1e-6'}/{dtype}", dtype=dtype, lr=lr, step=t)
        for k in TERMS:
            e = abs(got[k] - rl[k]) / max(abs(rl[k]), 1e-30)
            if dtype == "f32":
                bars.rec.setdefault("loss", {})[k] = e
                if e > LOSS_TOL[dtype]:
                    fails.append((t, "loss", k, got[k], rl[k]))
            else:
                bars.check("loss", k, e, LOSS_TOL[dtype], tag=t)
        gp = model.blocks()
        gm, gv = opt.state_blocks()
        for k in p:
            d = np.abs(np.asarray(gp[k], np.float64) - p[k])
            far = float(np.mean(d > 0.5 * lr))
            bars.rec.setdefault("param_far_frac", {})[k] = far
            bars.rec.setdefault("param_max_lr", {})[k] = float(d.max() / lr)
            if dtype == "f32":
                off = float(np.mean(d > 0.05 * lr + 4 * EPS32 * np.abs(p[k])))
                bars.rec.setdefault("param_off_frac", {})[k] = off
                if off > 1e-4 or d.max() > 2.05 * lr:
                    fails.append((t, "param", k, off, float(d.max() / lr)))
            elif far > 0.03 or d.max() > 2.05 * lr:
                fails.append((t, "param", k, far, float(d.max() / lr)))
            ev, ep = self_adam(p0s[k], m0s[k], v0s[k], np.asarray(gp[k], np.float64), np.asarray(gm[k], np.float64),
                               np.asarray(gv[k], np.float64), t, lr, cfg.adam_beta1, cfg.adam_beta2, cfg.adam_eps)
            bars.rec.setdefault("self_adam_err", {})[k] = [ev, ep]
            if ev > 1 or ep > 1:
                fails.append((t, "self_adam", k, ev, ep))
            mt = M_TOL[dtype]
            for name, a, r, tol in (("m", gm[k], m[k], mt), ("v", gv[k], v[k], min(2 * mt, 1.0))):
                e = block_err(np.asarray(a, np.float64), r)
                if dtype == "f32":
                    bars.rec.setdefault(name, {})[k] = e
                    if e > tol:
                        fails.append((t, name, k, e))
                elif p[k].size <= 32:      # recorded; pinned by self_adam above
                    bars.rec.setdefault(name + "_small", {})[k] = e
                else:
                    bars.check(name, k, e, tol, tag=t)
        bars.flush()
        fails += bars.fails
    assert opt.global_step == steps
    assert not fails, fails[:12]
