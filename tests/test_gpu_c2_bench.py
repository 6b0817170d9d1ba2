"""C2, the headline, at the benchmarked shape with the SHIPPED update path, step by step.

bench.py's C2 step: tscale(4096, 64), B = 8 graphs of synthetic_batch seed 1000, the
weights of init seed 0, and TF1 Adam fused into the step's final slab reduction
(snd_plan_fuse_adam + plan option "reduce_adam" on: every block of the node-latent plan
is updated inside `reduce_kernel`, ABI 16) -- exactly what the bench times.  Reference:
`model.py:104-161`, `model_joint.py:112-145`, `optimizer.py:125,135-197`,
`main.py:315-331`.

Every step t starts the float64 oracle (forward_backward with row_chunk + adam_tf1) from
the parameters and Adam moments the GPU held before step t, with the same injected eps,
and compares after step t:
* the loss terms: f32 1e-5 relative (the north_star's ELBO bar); bf16 against the
  measured bars of tests/parity_bars.json (5x the measured error per term: cost ~7e-5,
  kl ~8e-3; round 5 used a flat 2e-2);
* bf16 only: the structure term on the step's OWN bf16 operands (parity_bars.
  own_structure): the CE sum within 1e-6 of sum |terms| and the accuracy count exact
  away from |L| < 1e-4 -- a wrong logit anywhere in zz^T or the per-edge terms fails here;
* the gradient blocks the step wrote, against the oracle's, as max-abs error over the
  block's max-abs: f32 max(2e-4, 10 e32), e32 being the reference formulation's own
  float32 error on that block (oracle/ref_torch.py, autograd); where the fp32 step's
  lrelu' differs from the oracle's at a pre-activation that is zero to within 1e-6 of
  its layer's scale (a rounding tie at the kink, layers.py:112-113), the oracle takes the
  GPU's side (gpu_kink_choices) -- measured: one element at step 3, T = 5e-8, which alone
  moved dec.K1 / dec.b1 / dec.bn1.beta by 1.3-2.0e-3 of their max-abs; a disagreement
  farther from 0 fails; bf16 2x the measured error per block
  (parity_bars.json; the bf16 gap to the float64 oracle is the bf16 operands' rounding
  and is parity-unpinned against TF, which has no bf16 path);
* the fused update against the GPU's OWN gradient, in float64: m, v and the parameters
  after the step must equal TF1 Adam applied to the GPU gradient up to fp32 rounding
  (m, v 1e-6 relative per element + an absolute floor of 1e-6 of the block's max, the
  parameters within 1e-3 lr + 4 fp32 ulps).  This pins the reduction-fused Adam tightly
  in BOTH precisions: a wrong bias correction, step index, moment order or a skipped /
  doubled block fails here whatever the gradient's precision;
* fp32 only: the parameters against the oracle's update in units of lr (Adam moves every
  element by ~lr, so a sign-ambiguous near-zero gradient moves it up to 2 lr the other
  way): all but 1e-4 of a block's elements within 0.05 lr + 4 ulps.
Measured errors go to gpurun_out/parity_errors.jsonl.
"""
import numpy as np
import pytest
import torch

import parity_bars as PB
from oracle import ref_numpy as R
from snd_vae_amd.config import tscale
from snd_vae_amd.data import synthetic_batch
from snd_vae_amd.params import init_blocks

pytestmark = pytest.mark.gpu
TERMS = ("cost", "spatial_cost", "adj_cost", "node_cost", "kl")
STEPS = 3
LOSS_TOL = {"f32": 1e-5, "bf16": 2e-2}   # bf16: fallback where parity_bars.json has no entry
GRAD_TOL = {"f32": 2e-4, "bf16": 1e-1}
EPS32 = float(np.finfo(np.float32).eps)


@pytest.fixture(scope="module", autouse=True)
def _gpu(lib_built):
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm device")


def block_err(g, ref):
    return float(np.abs(g - ref).max() / max(np.abs(ref).max(), 1e-30))


# a derivative disagreement with the oracle is a rounding tie only where the oracle's own
# pre-activation is this close to 0 (relative to its layer's max |value|); measured, round
# 6: ONE element over the three fp32 steps, at 1.7e-8 (tools/diag_kink.py)
KINK_REL = 1e-6
KINK_LAYERS = {"P0": ("P0", None), "P1": ("P1", None), "T1": ("Y1", "dec.bn1"),
               "T2s": ("Y2S", "dec.bn2s"), "T2n": ("Y2N", "dec.bn2n"), "T3s": ("Y3S", "dec.bn3s")}


def gpu_kink_choices(model, p, cache, cfg, B):
    """The lrelu derivative the fp32 step actually used wherever it differs from the
    oracle's.  lrelu' is discontinuous at 0 (layers.py:112-113), so a pre-activation that
    is zero to within rounding may land on either side in any finite-precision evaluation:
    at such an element the oracle takes the GPU's side (ref_numpy lrelu_override), and the
    gradients are then held to the unchanged bars.  Any disagreement at a pre-activation
    NOT within KINK_REL of zero is reported as a failure ("beyond_rounding")."""
    R_ = B * cfg.n_nodes
    over, info = {}, {}
    for name, (buf, bn) in KINK_LAYERS.items():
        ref = cache[name]
        w = ref.shape[1]
        y = model.buffer(buf)[:R_ * w].view(R_, w).double().cpu().numpy()
        gpu = y if bn is None else y * (p[bn + ".gamma"] * R.BN_C) + p[bn + ".beta"]
        scale = max(np.abs(ref).max(), 1e-30)
        assert np.abs(gpu - ref).max() <= 1e-4 * scale, (name, "GPU pre-activation buffer layout")
        diff = (gpu >= 0) != (ref >= 0)
        if diff.any():
            o = np.full(ref.shape, np.nan)
            o[diff] = np.where(gpu[diff] >= 0, 1.0, 0.2)
            over[name] = o
            info[name] = {"n": int(diff.sum()), "max_rel": float(np.abs(ref[diff]).max() / scale),
                          "beyond_rounding": bool(np.abs(ref[diff]).max() > KINK_REL * scale)}
    return over, info


def adam_from(p, g, m, v, t, lr, b1, b2, eps):
    """TF1 Adam (optimizer.py:125 -> tf.train.AdamOptimizer) in float64 on one block, with
    TF's float32 coefficients: its ApplyAdam kernel forms 1 - beta1 and 1 - beta2 in the
    variable's dtype, and float32(1 - 0.999f) is 1.3e-5 relative off 0.001 -- the
    fused update does the same (adam_elem), a float64 (1 - b2) would not."""
    f32 = np.float32
    c1, c2 = float(f32(1) - f32(b1)), float(f32(1) - f32(b2))
    m2 = float(f32(b1)) * m + c1 * g
    v2 = float(f32(b2)) * v + c2 * g * g
    lr_t = lr * np.sqrt(1 - b2 ** t) / (1 - b1 ** t)
    return p - lr_t * m2 / (np.sqrt(v2) + eps), m2, v2


@pytest.mark.timeout(900)
@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_c2_bench_batch_steps_vs_oracle(dtype):
    from snd_vae_amd.model import DeviceBatch, SGCNModelVAE
    from snd_vae_amd.optimizer import OptimizerVAE
    cfg = tscale(4096, 64)
    B = 8
    batch = synthetic_batch(cfg, B, seed=1000)          # bench.py run_workload, rank 0
    adj = [batch.sparse_adj(b) for b in range(B)]
    p0 = {k: v.astype(np.float32).astype(np.float64) for k, v in init_blocks(cfg, 0).items()}
    rng = np.random.default_rng(9)
    eps = [rng.standard_normal((B * cfg.n_nodes, cfg.latent)).astype(np.float32) for _ in range(STEPS)]

    model = SGCNModelVAE(cfg, B, dtype=dtype, blocks=p0)
    opt = OptimizerVAE(model)                            # bench.py: fused by default
    assert opt.fused and not opt._adam_ranges, "every C2 block must be reduce-fused"
    db = DeviceBatch(batch)
    lr, b1, b2, ae = cfg.learning_rate, cfg.adam_beta1, cfg.adam_beta2, cfg.adam_eps
    fails = []
    for t in range(1, STEPS + 1):
        p = {k: np.asarray(v, np.float64) for k, v in model.blocks().items()}
        m, v = opt.state_blocks()
        m = {k: np.asarray(x, np.float64) for k, x in m.items()}
        v = {k: np.asarray(x, np.float64) for k, x in v.items()}
        opt.step(db, torch.from_numpy(eps[t - 1]).cuda())
        torch.cuda.synchronize()
        rl, rg, rc = R.forward_backward(p, adj, batch.features, batch.feature_truth,
                                        batch.spatial_truth, eps[t - 1].astype(np.float64),
                                        cfg, row_chunk=1024)
        kinks = {}
        if dtype == "f32":   # lrelu' at pre-activations that are zero within fp32 rounding
            over, kinks = gpu_kink_choices(model, p, rc, cfg, B)
            if over:
                rg = R.forward_backward(p, adj, batch.features, batch.feature_truth, batch.spatial_truth,
                                        eps[t - 1].astype(np.float64), cfg, row_chunk=1024,
                                        lrelu_override=over)[1]
        pr = {k: x.copy() for k, x in p.items()}
        mr = {k: x.copy() for k, x in m.items()}
        vr = {k: x.copy() for k, x in v.items()}
        R.adam_tf1(pr, rg, mr, vr, t, lr, b1, b2, ae)
        got = opt.loss_dict()
        gg = {k: np.asarray(x, np.float64) for k, x in opt.grad_blocks().items()}
        gp = {k: np.asarray(x, np.float64) for k, x in model.blocks().items()}
        gm, gv = opt.state_blocks()
        gm = {k: np.asarray(x, np.float64) for k, x in gm.items()}
        gv = {k: np.asarray(x, np.float64) for k, x in gv.items()}
        bars = PB.Bars(f"c2_bench_steps/{dtype}", dtype=dtype, step=t)
        if kinks:
            bars.note("kink_choices", kinks)
            fails += [(t, "kink", k, v) for k, v in kinks.items() if v["beyond_rounding"]]
        for k in TERMS:
            e = abs(got[k] - rl[k]) / max(abs(rl[k]), 1e-30)
            if dtype == "f32":
                bars.rec.setdefault("loss", {})[k] = e
                if e > LOSS_TOL[dtype]:
                    fails.append((t, "loss", k, got[k], rl[k]))
            else:
                bars.check("loss", k, e, LOSS_TOL[dtype], tag=t)
        if dtype == "bf16":   # the structure term on the step's own bf16 operands
            ce, absum, correct, amb = PB.own_structure(model, batch, cfg)
            e = abs(got["adj_sum"] - ce) / absum
            bars.note("own_structure", {"ce_rel_abs": e, "correct_diff": got["correct"] - correct,
                                        "ambiguous": amb})
            if e > 1e-6 or abs(got["correct"] - correct) > amb:
                fails.append((t, "own_structure", got["adj_sum"], ce, e, got["correct"], correct, amb))
        else:                 # the fp32 conditioning of each block (reference formulation)
            e32 = PB.e32_grads(p, [batch.dense_adj(b) for b in range(B)], batch.features,
                               batch.feature_truth, batch.spatial_truth, eps[t - 1], cfg, rg)
            bars.note("e32", e32)
        for k in p:
            e = block_err(gg[k], rg[k])
            if dtype == "f32":
                bars.rec.setdefault("grad", {})[k] = e
                if e > max(GRAD_TOL[dtype], 10 * e32[k]):
                    fails.append((t, "grad", k, e, e32[k]))
            else:
                bars.check("grad", k, e, GRAD_TOL[dtype], tag=t)
            # the fused update vs TF1 Adam on the GPU's own gradient (tight, any dtype)
            sp, sm, sv = adam_from(p[k], gg[k], m[k], v[k], t, lr, b1, b2, ae)
            em = float(np.max(np.abs(gm[k] - sm) / (1e-6 * np.abs(sm) + 1e-6 * np.abs(sm).max() + 1e-30)))
            ev = float(np.max(np.abs(gv[k] - sv) / (1e-6 * np.abs(sv) + 1e-6 * np.abs(sv).max() + 1e-30)))
            dp = np.abs(gp[k] - sp)
            ep = float(np.max(dp / (1e-3 * lr + 4 * EPS32 * np.abs(p[k]))))
            bars.rec.setdefault("self_adam_err", {})[k] = [em, ev, ep]
            if em > 1 or ev > 1 or ep > 1:
                fails.append((t, "self_adam", k, em, ev, ep))
            if dtype == "f32":
                d = np.abs(gp[k] - pr[k])
                off = float(np.mean(d > 0.05 * lr + 4 * EPS32 * np.abs(p[k])))
                bars.rec.setdefault("param_off_frac", {})[k] = off
                if off > 1e-4 or d.max() > 2.05 * lr:
                    fails.append((t, "param", k, off, float(d.max() / lr)))
        bars.flush()
        fails += bars.fails
    assert opt.global_step == STEPS
    assert not fails, fails[:12]
