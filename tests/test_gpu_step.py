"""Full train-step parity: snd_train_step + snd_adam_tf1 vs the golden fixtures
(float64 oracle) and vs the oracle at the C2 size.

fp32 mode is the parity mode (north_star: ELBO within 1e-5 of the reference
formula); bf16 mode (the throughput mode) is checked at a looser tolerance.
"""
import os

import numpy as np
import pytest
import torch

import golden_io
from oracle import ref_numpy as R
from snd_vae_amd.config import tref, tscale
from snd_vae_amd.data import synthetic_batch

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
LOSS_KEYS = ("cost", "spatial_cost", "adj_cost", "node_cost", "kl", "acc")


@pytest.fixture(scope="module", autouse=True)
def _gpu(lib_built):
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm device")


load_fixture = golden_io.load


def make(cfg, batch, p0, dtype, fuse_adam=False):
    """fuse_adam off by default: the parity tests read every block's gradient back."""
    from snd_vae_amd.model import DeviceBatch, SGCNModelVAE
    from snd_vae_amd.optimizer import OptimizerVAE
    model = SGCNModelVAE(cfg, batch.n_graphs, dtype=dtype, blocks=p0)
    return model, OptimizerVAE(model, fuse_adam=fuse_adam), DeviceBatch(batch)


def block_err(g, ref):
    return np.abs(g - ref).max() / max(np.abs(ref).max(), 1e-30)


def check_terms_grads(case, dtype, got, ref, g, rg, ltol, gtol):
    """Loss terms and gradient blocks: fp32 at the fixed bars, bf16 at the measured ones
    (tests/parity_bars.json; ltol / gtol are the fallbacks)."""
    import parity_bars as PB
    bars = PB.Bars(case, dtype=dtype)
    for k in ("cost", "spatial_cost", "adj_cost", "node_cost", "kl"):
        e = abs(got[k] - ref[k]) / max(abs(ref[k]), 1e-30)
        if dtype == "f32":
            bars.rec.setdefault("loss", {})[k] = e
            assert e <= ltol, (k, got[k], ref[k])
        else:
            bars.check("loss", k, e, ltol)
    for k in rg:
        e = float(block_err(g[k], rg[k]))
        if dtype == "f32":
            bars.rec.setdefault("grad", {})[k] = e
            if e > gtol:
                bars.fails.append(("grad", k, e))
        else:
            bars.check("grad", k, e, gtol)
    bars.flush()
    assert not bars.fails, bars.fails


@pytest.mark.parametrize("name", golden_io.NAMES)
def test_train_steps_f32_vs_golden(name):
    z, cfg, batch, p0 = load_fixture(name)
    model, opt, db = make(cfg, batch, p0, "f32")
    for t in range(3):
        eps = torch.from_numpy(z["eps"][t]).cuda()
        opt.step(db, eps)
        got = opt.loss_dict()
        for k in LOSS_KEYS:
            ref = float(z[f"s{t}/loss/{k}"])
            assert got[k] == pytest.approx(ref, rel=1e-5, abs=1e-7), (t, k, got[k], ref)
        grads = opt.grad_blocks()
        for k, g in grads.items():
            err, nerr = golden_io.block_error(z, f"s{t}/grad", k, g)
            assert err < 2e-4 and (nerr is None or nerr < 1e-4), (t, k, err, nerr)
    final = model.blocks()
    for k, v in final.items():
        # Adam normalises each update to ~lr: compare against the step size
        assert golden_io.max_abs_diff(z, "p_final", k, v) < 0.05 * 3 * cfg.learning_rate, k
    assert opt.global_step == 3


@pytest.mark.parametrize("name", ["tscale_n200_d16", "tref_c1_n200_d16"])
def test_train_step_bf16_vs_golden(name):
    import parity_bars as PB
    z, cfg, batch, p0 = load_fixture(name)
    model, opt, db = make(cfg, batch, p0, "bf16")
    opt.step(db, torch.from_numpy(z["eps"][0]).cuda())
    got = opt.loss_dict()
    bars = PB.Bars(f"golden_{name}/bf16", dtype="bf16")
    for k in ("cost", "spatial_cost", "adj_cost", "node_cost", "kl"):
        ref = float(z[f"s0/loss/{k}"])
        bars.check("loss", k, abs(got[k] - ref) / max(abs(ref), 1e-30), 2e-2)
    grads = opt.grad_blocks()
    # bf16 operands (8-bit mantissa) in sums with cancellation: compare norm-wise, each
    # block against 2x its measured error (parity_bars.json); fallbacks: the decoder-conv
    # gradients sit at 3-5 % on both the fast and the generic bf16 engines
    # (tools/bf16_errors.py), encoder blocks at ~0.3 %
    for k, g in grads.items():
        if f"s0/grad/{k}" not in z.files:     # sampled big block: sampled max-abs check
            err, nerr = golden_io.block_error(z, "s0/grad", k, g)
            bars.check("grad", k, float(err), 5e-2)
            bars.check("gradn", k, float(nerr), 2e-2)
            continue
        ref = z[f"s0/grad/{k}"]
        err = np.linalg.norm(g - ref) / max(np.linalg.norm(ref), 1e-30)
        bars.check("gradn", k, float(err), 1e-1 if k.startswith("dec.") else 2e-2)
    bars.flush()
    assert not bars.fails, bars.fails


@pytest.mark.parametrize("dtype,ltol,gtol", [("f32", 1e-5, 2e-4), ("bf16", 2e-2, 1e-1)])
def test_train_step_c2_size_vs_oracle(dtype, ltol, gtol):
    """N=4096 d=64 (the bench config) with B=2 graphs, one step vs the oracle."""
    cfg = tscale(4096, 64)
    batch = synthetic_batch(cfg, 2, seed=0)
    from snd_vae_amd.params import init_blocks
    p0 = {k: v.astype(np.float32).astype(np.float64) for k, v in init_blocks(cfg, 0).items()}
    eps = np.random.default_rng(9).standard_normal((2 * 4096, 64)).astype(np.float32)
    model, opt, db = make(cfg, batch, p0, dtype)
    opt.step(db, torch.from_numpy(eps).cuda())
    got = opt.loss_dict()
    adj = [batch.dense_adj(b) for b in range(2)]
    ref, rg, _ = R.forward_backward(p0, adj, batch.features, batch.feature_truth,
                                    batch.spatial_truth, eps.astype(np.float64), cfg)
    assert abs(got["acc"] - ref["acc"]) < (1e-6 if dtype == "f32" else 1e-3)
    check_terms_grads(f"c2_size_b2/{dtype}", dtype, got, ref, opt.grad_blocks(), rg, ltol, gtol)


@pytest.mark.parametrize("dtype,ltol,gtol", [("f32", 1e-5, 2e-4), ("bf16", 2e-2, 1e-1)])
def test_train_step_c4_size_vs_oracle(dtype, ltol, gtol):
    """C4: graph latent + model_joint decoders at N=4096 d=64 (B=2), one step vs the oracle.

    Exercises the 27 M-row-element head stream (flat(G) [2, 274432]) and the
    26 M-element d_sg_lin1 projection at the BASELINE size."""
    cfg = tref(4096, 64)
    batch = synthetic_batch(cfg, 2, seed=0)
    from snd_vae_amd.params import init_blocks
    p0 = {k: v.astype(np.float32).astype(np.float64) for k, v in init_blocks(cfg, 0).items()}
    eps = np.random.default_rng(9).standard_normal((2, cfg.latent)).astype(np.float32)
    model, opt, db = make(cfg, batch, p0, dtype)
    opt.step(db, torch.from_numpy(eps).cuda())
    got = opt.loss_dict()
    adj = [batch.dense_adj(b) for b in range(2)]
    ref, rg, _ = R.forward_backward(p0, adj, batch.features, batch.feature_truth,
                                    batch.spatial_truth, eps.astype(np.float64), cfg)
    assert abs(got["acc"] - ref["acc"]) < (1e-6 if dtype == "f32" else 1e-3)
    check_terms_grads(f"c4_size_b2/{dtype}", dtype, got, ref, opt.grad_blocks(), rg, ltol, gtol)
    # decoder input J and the graph latent read back under the reference names
    assert model.joint_h.shape == (2 * 4096, 64) and model.z_sg.shape == (2, cfg.latent)
    assert model.z_mean_sg.shape == (2, cfg.latent)


@pytest.mark.parametrize("kind", ["tref", "tscale"])
@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_fused_adam_matches_separate_update(dtype, kind):
    """Adam inside the step (snd_plan_fuse_adam) -- in the graph-latent head / d_sg_lin1
    weight streams (kind 1) and in the final slab reduction (kind 2, every block of the
    node-latent plans) -- gives the parameters and Adam moments of the separate
    snd_adam_tf1 pass, bit for bit over three steps, eager and graph-replayed."""
    from snd_vae_amd import _lib
    from snd_vae_amd.params import init_blocks
    cfg = tref(1024, 64) if kind == "tref" else tscale(2048, 64)
    batch = synthetic_batch(cfg, 2, seed=4)
    p0 = init_blocks(cfg, 0)
    runs = []
    for fuse in (False, True):
        m, o, b = make(cfg, batch, p0, dtype, fuse_adam=fuse)
        o.step(b)
        o.capture(b)
        o.replay()
        o.replay()
        torch.cuda.synchronize()
        runs.append((m, o))
    (m0, o0), (m1, o1) = runs
    assert o1.fused and not o0.fused and o1.global_step == 3
    names = list(m1.layout.shapes)
    kinds = {k: _lib.lib().snd_plan_block_fused(m1.plan, i) for i, k in enumerate(names)}
    if kind == "tref":
        assert kinds["enc.Wh"] == 1 and kinds["dec.Wp"] == 1 and kinds["dec.bp"] == 1
    else:   # every block in the reduction
        assert set(kinds.values()) == {2}
    assert o1._adam_ranges == []   # no separate Adam launch at all
    p_a, p_b = m0.blocks(), m1.blocks()
    # same gradients and one shared element update with explicit roundings (snd_common.hpp
    # adam_elem): the fused and the separate update agree bit for bit, over three steps
    for k in p_a:
        assert np.array_equal(p_a[k], p_b[k]), (k, np.abs(p_a[k] - p_b[k]).max())
    for a, b in ((o0.m, o1.m), (o0.v, o1.v)):
        assert torch.equal(a, b)
    g_a, g_b = o0.grad_blocks(), o1.grad_blocks()
    for k in names:   # the reduction-fused blocks still store their gradient
        if kinds[k] != 1:
            assert np.array_equal(g_a[k], g_b[k]), k
    assert o0.loss_dict()["cost"] == o1.loss_dict()["cost"]


def test_device_rng_same_draw_on_both_engines():
    """Philox eps (seed, step) is the same stream on the bf16 fast path and the fp32
    generic engine: standard-normal moments, bitwise-equal draws."""
    from snd_vae_amd.params import init_blocks
    cfg = tscale(512, 64)
    batch = synthetic_batch(cfg, 2, seed=6)
    eps = []
    for dtype in ("bf16", "f32"):
        m, o, b = make(cfg, batch, init_blocks(cfg, 0), dtype)
        o.forward_backward(b)
        torch.cuda.synchronize()
        eps.append(m.buffer("EPS")[:2 * 512 * 64].clone())
    assert torch.equal(eps[0], eps[1])
    e = eps[0].double()
    assert abs(float(e.mean())) < 0.02 and abs(float(e.std()) - 1.0) < 0.02


def test_graph_replay_is_deterministic():
    """A captured step replays bit-identically to eager steps (no atomics)."""
    cfg = tscale(512, 64)
    batch = synthetic_batch(cfg, 4, seed=1)
    from snd_vae_amd.params import init_blocks
    p0 = init_blocks(cfg, 0)
    m1, o1, b1 = make(cfg, batch, p0, "bf16")
    for _ in range(5):
        o1.step(b1)
    m2, o2, b2 = make(cfg, batch, p0, "bf16")
    init = [t.clone() for t in (m2.params, o2.m, o2.v, o2.step_counter)]
    o2.step(b2)                    # a non-trivial state to capture from (moments, step 1)
    snap = [t.clone() for t in (m2.params, o2.m, o2.v, o2.step_counter, o2.grads, o2.losses)]
    o2.capture(b2, warmup=2)       # 2 eager warm-up steps + the capture; state restored
    # capture leaves every piece of training state bit-identical
    for name, a, b in zip(("params", "m", "v", "step", "grads", "losses"), snap,
                          (m2.params, o2.m, o2.v, o2.step_counter, o2.grads, o2.losses)):
        assert torch.equal(a, b), name
    # one replay == one eager step from the same state
    m3, o3, b3 = make(cfg, batch, p0, "bf16")
    for dst, src in zip((m3.params, o3.m, o3.v, o3.step_counter), snap):
        dst.copy_(src)
    o3.step(b3)
    o2.replay()
    torch.cuda.synchronize()
    assert torch.equal(m2.params, m3.params) and torch.equal(o2.v, o3.v)
    assert torch.equal(o2.losses, o3.losses)
    for dst, src in zip((m2.params, o2.m, o2.v, o2.step_counter), init):
        dst.copy_(src)             # back to the initial state: 5 replays == 5 eager steps
    for _ in range(5):
        o2.replay()
    torch.cuda.synchronize()
    assert o1.global_step == o2.global_step == 5
    assert torch.equal(m1.params, m2.params)
    assert torch.equal(o1.losses, o2.losses)


@pytest.mark.parametrize("B", [1, 2])
def test_concurrent_decoder_replays_like_eager(B):
    """Plan option "conc_decoder" (the fused decoder on a side stream beside zz^T, whose
    column splits then leave the decoder's tiles their CUs): captured replays equal eager
    steps bit for bit, and the step equals the serial step's up to the zz^T split sums'
    fp32 re-association."""
    from snd_vae_amd.params import init_blocks
    cfg = tscale(4096, 64)
    batch = synthetic_batch(cfg, B, seed=8)
    p0 = init_blocks(cfg, 0)
    runs = []
    for conc in (0, 1):
        m, o, b = make(cfg, batch, p0, "bf16")
        assert m.set_option("conc_decoder", conc) == bool(conc)   # explicit, not the auto default
        for _ in range(3):
            o.step(b)                 # eager (the first creates the side stream)
        torch.cuda.synchronize()
        runs.append((m, o, b))
    (ms, os_, _), (mc, oc, bc) = runs
    for k in ("cost", "adj_cost", "kl", "spatial_cost"):
        assert oc.loss_dict()[k] == pytest.approx(os_.loss_dict()[k], rel=1e-4), k
    gs, gc = os_.grads[:ms.param_count], oc.grads[:mc.param_count]
    assert float((gs - gc).abs().max()) <= 2e-2 * float(gs.abs().max())
    # replay == eager from the same state
    m2, o2, b2 = make(cfg, batch, p0, "bf16")
    m2.set_option("conc_decoder", 1)
    o2.step(b2)
    o2.capture(b2, warmup=1)
    snap = [t.clone() for t in (m2.params, o2.m, o2.v, o2.step_counter)]
    o2.replay()
    m3, o3, b3 = make(cfg, batch, p0, "bf16")
    m3.set_option("conc_decoder", 1)
    o3.step(b3)                       # creates the side stream; then reset to the snapshot
    for dst, src in zip((m3.params, o3.m, o3.v, o3.step_counter), snap):
        dst.copy_(src)
    o3.step(b3)
    torch.cuda.synchronize()
    assert torch.equal(m2.params, m3.params) and torch.equal(o2.losses, o3.losses)


def test_training_reduces_cost():
    cfg = tscale(1024, 64)
    batch = synthetic_batch(cfg, 4, seed=3)
    from snd_vae_amd.params import init_blocks
    m, o, b = make(cfg, batch, init_blocks(cfg, 0), "bf16")
    o.step(b)
    first = o.loss_dict()["cost"]
    for _ in range(60):
        o.step(b)
    last = o.loss_dict()["cost"]
    assert np.isfinite(last) and last < first


def test_device_rng_matches_restatement_and_rank_offset():
    """Device normals equal the oracle's Philox4x32-10 + Box-Muller restatement
    (oracle/ref_rng.py; fast f32 log/sincos on the device, float64 here), and a
    data-parallel shard (snd_plan_set_rng_offset at its first global row) draws
    bit-for-bit the rows one device draws for the whole batch."""
    from oracle import ref_rng
    from snd_vae_amd import _lib
    from snd_vae_amd.data import shard
    from snd_vae_amd.params import init_blocks
    cfg = tscale(512, 64)
    batch = synthetic_batch(cfg, 2, seed=6)
    p0 = init_blocks(cfg, 0)
    m, o, b = make(cfg, batch, p0, "bf16")
    o.forward_backward(b)
    torch.cuda.synchronize()
    full = m.buffer("EPS")[:2 * 512 * 64].view(1024, 64).clone()
    ref = ref_rng.eps(o.seed, 0, 1024, 64)
    d = np.abs(full.double().cpu().numpy() - ref)
    assert np.median(d) < 1e-6 and d.max() < 5e-3, (np.median(d), d.max())
    for dtype in ("bf16", "f32"):
        m1, o1, b1 = make(cfg, shard(batch, 1, 2), p0, dtype)
        _lib.check(_lib.lib().snd_plan_set_rng_offset(m1.plan, 512))
        o1.forward_backward(b1)
        torch.cuda.synchronize()
        assert torch.equal(m1.buffer("EPS")[:512 * 64].view(512, 64), full[512:])


def test_forced_world1_process_group_runs_the_distributed_step():
    """with a process group present -- even a world of 1 -- the step
    always runs the RCCL all-reduce and never fuses Adam.  Its result must equal
    an eager single-process run with fuse_adam off, bit for bit (all-reduce of one
    rank and grad_scale 1/world = 1 are identities), on the graph-latent plan
    where fusion matters."""
    import socket

    import torch.distributed as dist

    from snd_vae_amd.model import DeviceBatch, SGCNModelVAE
    from snd_vae_amd.optimizer import OptimizerVAE
    from snd_vae_amd.params import init_blocks
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        cfg = tref(64, 16, mean_degree=6.0)
        batch = synthetic_batch(cfg, 2, seed=4)
        p0 = init_blocks(cfg, 0)
        ma = SGCNModelVAE(cfg, 2, dtype="bf16", blocks=p0)
        oa = OptimizerVAE(ma, process_group=dist.group.WORLD, bucketed=True)
        assert oa.distributed and not oa.fused
        mb, ob, bb = make(cfg, batch, p0, "bf16", fuse_adam=False)
        ba = DeviceBatch(batch)
        calls = []
        real = dist.all_reduce
        dist.all_reduce = lambda t, **kw: (calls.append(t.numel()), real(t, **kw))[1]
        try:
            for _ in range(3):
                oa.step(ba)
                ob.step(bb)
        finally:
            dist.all_reduce = real
        torch.cuda.synchronize()
        # the bucketed exchange (parallel.plan_buckets): every bucket is all-reduced once per
        # step at this size (no bucket reaches SHARD_MIN), together exactly grads || loss terms
        nb = len(oa.buckets)
        assert nb > 1 and not any(b.sharded for b in oa.buckets)
        assert len(calls) == 3 * nb and sum(calls) == 3 * (ma.param_count + 8)
        assert torch.equal(ma.params, mb.params)
        assert torch.equal(oa.losses, ob.losses)
    finally:
        dist.destroy_process_group()


DEC_BUFS = (("FY1", torch.float32), ("FU1", torch.bfloat16), ("FY2", torch.float32),
            ("FU2", torch.bfloat16), ("FDY3", torch.bfloat16), ("FDY2", torch.bfloat16),
            ("FDY1", torch.bfloat16), ("DZDEC", torch.float32), ("SHAT", torch.float32),
            ("XHAT", torch.float32))


@pytest.mark.parametrize("topology,n,d,B", [("tscale", 512, 64, 2), ("tscale", 200, 16, 3),
                                            ("tref", 300, 32, 2), ("tscale", 4096, 64, 4),
                                            ("tscale", 1000, 128, 2)])
def test_fused_decoder_matches_row_engine(topology, n, d, B):
    """The fused decoder (snd_dec.hip: conv chain + heads in one launch, the
    backward data chain in another, halos recomputed in LDS) against the row
    engine's seven launches (debug bit 32768): every activation, data gradient
    and head output is bitwise equal; the parameter gradients built from
    column partials (biases, BN, heads) agree to fp32 reassociation, and the
    conv weight gradients (same operands) are bitwise equal.  Covers partial
    tiles (N = 200, 300: 128-row tiles never span graphs) and the graph latent; N = 4096,
    B = 4 the 128-row tiles of a full chip (128 tiles), the bench's tiling; d = 128 (C5's
    width) the streamed kernels: 64-row tiles, every conv's weights through two one-tap
    LDS buffers (N = 1000: a partial last tile)."""
    from snd_vae_amd import _lib
    from snd_vae_amd.params import init_blocks
    cfg = tscale(n, d) if topology == "tscale" else tref(n, d, g_hidden=16, latent=8)
    batch = synthetic_batch(cfg, B, seed=11)
    p0 = init_blocks(cfg, 2)
    runs = []
    for flags in (32768, 0):
        _lib.check(_lib.lib().snd_debug_set(flags))
        try:
            m, o, b = make(cfg, batch, p0, "bf16")
        finally:
            _lib.check(_lib.lib().snd_debug_set(0))
        o.forward_backward(b)
        torch.cuda.synchronize()
        runs.append((m, o))
    (m0, o0), (m1, o1) = runs
    R = B * n
    for name, dt in DEC_BUFS:
        a, c = m0.buffer(name, dt), m1.buffer(name, dt)
        assert torch.equal(a, c), name
    g0, g1 = o0.grad_blocks(), o1.grad_blocks()
    for k in g0:
        if not k.startswith("dec."):
            continue
        if k.startswith("dec.K"):
            assert np.array_equal(g0[k], g1[k]), k
        else:
            np.testing.assert_allclose(g1[k], g0[k], rtol=1e-4, atol=1e-7 * max(1.0, np.abs(g0[k]).max()),
                                       err_msg=k)
    l0, l1 = o0.loss_dict(), o1.loss_dict()
    for k in ("spatial_cost", "node_cost", "cost"):
        assert l1[k] == pytest.approx(l0[k], rel=1e-6), k
    # the forward kernel zeroes only the LDS it must: rerun with every activation byte
    # of its LDS set to NaN first (debug bit 1 << 23) -- same buffers, bit for bit
    ctr = o1.step_counter.clone()            # the device Philox stream is keyed by the step
    o1.forward_backward(b)
    torch.cuda.synchronize()
    snap = {name: m1.buffer(name, dt).clone() for name, dt in DEC_BUFS}
    o1.step_counter.copy_(ctr)
    _lib.check(_lib.lib().snd_debug_set(1 << 23))
    try:
        o1.forward_backward(b)
        torch.cuda.synchronize()
    finally:
        _lib.check(_lib.lib().snd_debug_set(0))
    for name, dt in DEC_BUFS:
        assert torch.equal(m1.buffer(name, dt), snap[name]), f"{name} with NaN-poisoned LDS"


def test_edge_terms_in_reparam_backward_launch():
    """d = 128 (no fused backward head, C5's width): the per-edge terms computed inside the
    reparameterisation backward (edge_reparam_bwd_kernel) against edge_bf16 before zz^T +
    reparam_bwd_fast (debug bit 1 << 27 at plan creation): d[mu | s], every gradient but
    the [mu | s] bias (its column sums group rows by the fused kernel's 32-row blocks) and
    every loss term bitwise equal."""
    from snd_vae_amd import _lib
    from snd_vae_amd.params import init_blocks
    cfg = tscale(2048, 128)
    batch = synthetic_batch(cfg, 2, seed=41)
    p0 = init_blocks(cfg, 4)
    runs = []
    for flags in (1 << 27, 0):
        _lib.check(_lib.lib().snd_debug_set(flags))
        try:
            m, o, b = make(cfg, batch, p0, "bf16")
        finally:
            _lib.check(_lib.lib().snd_debug_set(0))
        o.forward_backward(b)
        torch.cuda.synchronize()
        runs.append((m, o))
    (m0, o0), (m1, o1) = runs
    for name, dt in (("FDMS", torch.bfloat16), ("FDH", torch.bfloat16), ("FDP1", torch.bfloat16)):
        assert torch.equal(m0.buffer(name, dt), m1.buffer(name, dt)), name
    g0, g1 = o0.grad_blocks(), o1.grad_blocks()
    for k in g0:
        if k == "enc.bms":
            np.testing.assert_allclose(g1[k], g0[k], rtol=1e-5, atol=1e-7 * max(1.0, np.abs(g0[k]).max()), err_msg=k)
        else:
            np.testing.assert_array_equal(g1[k], g0[k], err_msg=k)
    assert torch.equal(o0.losses, o1.losses)


@pytest.mark.parametrize("n,B", [(2048, 2), (1000, 1)])
def test_weight_images_inside_gcn0_launch(n, B):
    """d = 128 (C5's widths: the encoder front is not fused, gcn0 runs): the step's packed
    weight images built by extra workgroups of the gcn0 launch against pack_kernel before
    it (debug bit 1 << 28 at plan creation).  Two Adam steps (the second packs the updated
    parameters): every gradient block, the parameters and every loss term bitwise equal."""
    from snd_vae_amd import _lib
    from snd_vae_amd.params import init_blocks
    cfg = tscale(n, 128)
    batch = synthetic_batch(cfg, B, seed=43)
    p0 = init_blocks(cfg, 5)
    runs = []
    for flags in (1 << 28, 0):
        _lib.check(_lib.lib().snd_debug_set(flags))
        try:
            m, o, b = make(cfg, batch, p0, "bf16")
        finally:
            _lib.check(_lib.lib().snd_debug_set(0))
        losses = []
        for _ in range(2):
            o.step(b)
            torch.cuda.synchronize()
            losses.append(o.losses.clone())
        runs.append((m, o, losses))
    (m0, o0, l0), (m1, o1, l1) = runs
    for a, c in zip(l0, l1):
        assert torch.equal(a, c)
    g0, g1 = o0.grad_blocks(), o1.grad_blocks()
    for k in g0:
        np.testing.assert_array_equal(g1[k], g0[k], err_msg=k)
    assert torch.equal(m0.params, m1.params)


HEAD_BUFS = (("FP1", torch.float32), ("FG", torch.bfloat16), ("FHH", torch.bfloat16), ("MS", torch.float32),
             ("Z", torch.float32), ("ZB", torch.bfloat16), ("EPS", torch.float32), ("ZSTAGE", torch.uint8),
             ("DJD", torch.float32), ("FDP1", torch.bfloat16))


@pytest.mark.parametrize("n,d,B", [(512, 64, 2), (300, 32, 3), (4096, 64, 2)])
def test_fused_encoder_head_matches_chain(n, d, B):
    """The fused encoder forward tail (snd_head.hip: GraphConvolution 1 gather + epilogue,
    h = G Wh + bh, [mu | s] = h Wms + bms, reparameterisation and the zz^T staging images in
    one launch) against the four-launch chain (debug bit 65536): P1, G, h, [mu | s], z,
    eps and the staging images are bitwise equal, so is everything downstream (dJ, dP1);
    the KL partials group rows differently (fp64 sums: the losses agree to 1e-12; the KL term
    alone to 1e-9 since round 5, whose per-element KL is the cancellation-free
    -(expm1(2s) - 2s) - mu^2 with full fp32 mantissas instead of values quantized to the
    O(1) terms' ulp, so the grouping of the fp64 sums shows: 2.5e-11 measured).
    N = 300 covers partial 128-row tiles, d = 32 the narrower heads."""
    from snd_vae_amd import _lib
    from snd_vae_amd.params import init_blocks
    cfg = tscale(n, d)
    batch = synthetic_batch(cfg, B, seed=12)
    p0 = init_blocks(cfg, 3)
    runs = []
    for flags in (65536, 0):
        _lib.check(_lib.lib().snd_debug_set(flags))
        try:
            m, o, b = make(cfg, batch, p0, "bf16")
        finally:
            _lib.check(_lib.lib().snd_debug_set(0))
        o.forward_backward(b)
        torch.cuda.synchronize()
        runs.append((m, o))
    (m0, o0), (m1, o1) = runs
    for name, dt in HEAD_BUFS:
        assert torch.equal(m0.buffer(name, dt), m1.buffer(name, dt)), name
    l0, l1 = o0.loss_dict(), o1.loss_dict()
    for k in ("cost", "adj_cost", "kl", "acc"):
        assert l1[k] == pytest.approx(l0[k], rel=1e-9 if k == "kl" else 1e-12, abs=1e-15), k
    g0, g1 = o0.grad_blocks(), o1.grad_blocks()
    for k in g0:
        np.testing.assert_allclose(g1[k], g0[k], rtol=1e-5, atol=1e-6 * max(1.0, np.abs(g0[k]).max()), err_msg=k)


@pytest.mark.parametrize("n,d,B", [(512, 64, 2), (300, 32, 3), (200, 16, 2), (4096, 64, 8)])
def test_fused_backward_head_matches_chain(n, d, B):
    """The fused backward head (snd_head.hip: per-edge CE terms, the reparameterisation /
    KL backward, dh = d[mu | s] Wms^T and the encoder BN / lrelu backward to dP1 in one
    launch) against edge_bf16 + reparam_bwd_fast + two row-engine launches (debug bit
    262144): d[mu | s], dh and dP1 are bitwise equal and so is every weight gradient
    computed from them; the bias gradient of the [mu | s] head and the edge loss partials
    group rows differently (agree to fp32 / fp64 reassociation), and so do the bias / BN
    gradients from column partials when the kernel runs 64-row tiles (small batches)."""
    from snd_vae_amd import _lib
    from snd_vae_amd.params import init_blocks
    cfg = tscale(n, d)
    batch = synthetic_batch(cfg, B, seed=13)
    p0 = init_blocks(cfg, 4)
    runs = []
    for flags in (262144, 0):
        _lib.check(_lib.lib().snd_debug_set(flags))
        try:
            m, o, b = make(cfg, batch, p0, "bf16")
        finally:
            _lib.check(_lib.lib().snd_debug_set(0))
        o.forward_backward(b)
        torch.cuda.synchronize()
        runs.append((m, o))
    (m0, o0), (m1, o1) = runs
    for name, dt in (("FDMS", torch.bfloat16), ("FDH", torch.bfloat16), ("FDP1", torch.bfloat16)):
        assert torch.equal(m0.buffer(name, dt), m1.buffer(name, dt)), name
    l0, l1 = o0.loss_dict(), o1.loss_dict()
    for k in ("cost", "adj_cost", "kl", "acc"):
        assert l1[k] == pytest.approx(l0[k], rel=1e-9 if k == "kl" else 1e-12, abs=1e-15), k
    g0, g1 = o0.grad_blocks(), o1.grad_blocks()
    # below 128 tiles of 128 rows the fused kernel runs 64-row tiles (head_bwd_rows): the
    # column partials behind the bias / BN gradients then group rows differently too
    tiled = {"enc.bms"}
    if B * ((n + 127) // 128) < 128:
        tiled |= {"enc.bh", "enc.bn1.gamma", "enc.bn1.beta", "enc.bne.gamma", "enc.bne.beta"}
    for k in g0:
        if k in tiled:
            np.testing.assert_allclose(g1[k], g0[k], rtol=1e-4, atol=1e-6 * max(1.0, np.abs(g0[k]).max()), err_msg=k)
        else:
            assert np.array_equal(g0[k], g1[k]), k


FRONT_BUFS = (("FH1", torch.bfloat16), ("AX", torch.float32), ("AXB", torch.bfloat16), ("FXW1", torch.bfloat16),
              ("PK1F", torch.uint8), ("PK2F", torch.uint8), ("PK3F", torch.uint8), ("PK3B", torch.uint8),
              ("PK2B", torch.uint8), ("PK1B", torch.uint8), ("PW1F", torch.uint8), ("PW1B", torch.uint8))


@pytest.mark.parametrize("topology,n,d,B", [("tscale", 512, 64, 2), ("tscale", 300, 32, 3),
                                            ("tscale", 200, 16, 2), ("tref", 300, 32, 2)])
def test_fused_encoder_front_matches_chain(topology, n, d, B):
    """The fused encoder front (snd_head.hip: the gcn0 gather, H1 = [BN0(lrelu(AX W0)) | X],
    XW1 = H1 W1 and the step's packed weight images in one launch) against pack + gcn0 +
    a row-engine launch (debug bit 1048576): H1, AX, XW1 and every weight image are
    bitwise equal, and so is the whole step downstream."""
    from snd_vae_amd import _lib
    from snd_vae_amd.params import init_blocks
    cfg = tscale(n, d) if topology == "tscale" else tref(n, d, g_hidden=16, latent=8)
    batch = synthetic_batch(cfg, B, seed=14)
    p0 = init_blocks(cfg, 5)
    runs = []
    for flags in (1048576, 0):
        _lib.check(_lib.lib().snd_debug_set(flags))
        try:
            m, o, b = make(cfg, batch, p0, "bf16")
        finally:
            _lib.check(_lib.lib().snd_debug_set(0))
        o.forward_backward(b)
        torch.cuda.synchronize()
        runs.append((m, o))
    (m0, o0), (m1, o1) = runs
    names = [nm for nm in FRONT_BUFS if not (topology == "tref" and nm[0] in ("PWHF",))]
    for name, dt in names:
        assert torch.equal(m0.buffer(name, dt), m1.buffer(name, dt)), name
    l0, l1 = o0.loss_dict(), o1.loss_dict()
    for k in l0:
        assert l1[k] == l0[k], k
    g0, g1 = o0.grad_blocks(), o1.grad_blocks()
    for k in g0:
        assert np.array_equal(g0[k], g1[k]), k


@pytest.mark.parametrize("n,B", [(4096, 8), (4096, 1), (1000, 3)])
def test_step_window_spmm_matches_row_tiles(n, B):
    """The step's GraphConvolution backward SpMM A @ dP1 on the window kernel (the batch
    carries a window plan, snd_window_plan_t) against the row-tile kernel (debug bit
    1 << 22): the same fp32 sums in colidx order -- dXW1 and every gradient equal."""
    from snd_vae_amd import _lib
    from snd_vae_amd.params import init_blocks
    cfg = tscale(n, 64)
    batch = synthetic_batch(cfg, B, seed=21)
    p0 = init_blocks(cfg, 1)
    runs = []
    for flags in (1 << 22, 0):
        m, o, b = make(cfg, batch, p0, "bf16")
        assert b.window is not None and b.tiles is not None
        _lib.check(_lib.lib().snd_debug_set(flags))
        try:
            o.forward_backward(b)
            torch.cuda.synchronize()
        finally:
            _lib.check(_lib.lib().snd_debug_set(0))
        runs.append((m, o))
    (m0, o0), (m1, o1) = runs
    a, c = m0.buffer("FDXW1", torch.bfloat16), m1.buffer("FDXW1", torch.bfloat16)
    diff = int((a.view(torch.int16) != c.view(torch.int16)).sum())
    assert diff <= 1e-5 * a.numel(), diff       # dot2c adds: within one fp32 ulp, bitwise in practice
    g0, g1 = o0.grad_blocks(), o1.grad_blocks()
    for k in g0:
        np.testing.assert_allclose(g1[k], g0[k], rtol=1e-3, atol=1e-6 * max(1.0, np.abs(g0[k]).max()), err_msg=k)
