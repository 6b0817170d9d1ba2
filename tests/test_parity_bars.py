"""CPU checks of the GPU tests' parity references (tests/parity_bars.py): the own-operand
structure term against an independent dense evaluation, the fp32-conditioning estimate
of the reference formulation, and the measured-bar table's shape."""
import json
import math

import numpy as np
import pytest
import torch

import parity_bars as PB
from oracle import ref_numpy as R
from snd_vae_amd.config import tscale
from snd_vae_amd.data import synthetic_batch
from snd_vae_amd.params import init_blocks


class _FakeModel:
    """The two plan buffers own_structure reads, laid out as the plan holds them."""

    def __init__(self, bufs):
        self.bufs = bufs

    def buffer(self, name, dtype=torch.float32):
        return self.bufs[name].to(dtype)


def test_own_structure_matches_dense_evaluation():
    n, d, B = 200, 64, 2
    cfg = tscale(n, d, mean_degree=8.0)
    batch = synthetic_batch(cfg, B, seed=3)
    z = np.random.default_rng(0).standard_normal((B * n, d)).astype(np.float32)
    npad = 256
    c = math.sqrt(1.0 / math.log(2.0))
    img = torch.zeros(B, npad, d, dtype=torch.bfloat16)
    img[:, :n] = (torch.from_numpy(z) * c).to(torch.bfloat16).view(B, n, d)
    zb = torch.from_numpy(z).to(torch.bfloat16)
    m = _FakeModel({"ZSTAGE": img.reshape(-1), "ZB": zb.reshape(-1)})
    ce, absum, correct, amb = PB.own_structure(m, batch, cfg)
    # independent dense evaluation with the same two roundings
    ref_ce, ref_correct = 0.0, 0
    for b in range(B):
        J = img[b, :n].double().numpy()
        Zb = zb[b * n:(b + 1) * n].double().numpy()
        Ld = (J @ J.T) * math.log(2.0)
        Le = Zb @ Zb.T
        A = batch.dense_adj(b)
        off = ~np.eye(n, dtype=bool)
        ref_ce += float((R.softplus(Ld) - A * Le)[off].sum()) + n * PB.SOFTPLUS_M1
        pred = np.where(A > 0, Le > 0, Ld > 0) & off
        ref_correct += int((pred == (A > 0)).sum())
    assert ce == pytest.approx(ref_ce, rel=1e-12)
    assert absum >= abs(ce)
    assert abs(correct - ref_correct) <= amb


def test_e32_is_the_fp32_rounding_of_the_reference_formulation():
    n, d, B = 25, 16, 2
    cfg = tscale(n, d, mean_degree=4.0)
    batch = synthetic_batch(cfg, B, seed=1)
    p = {k: v.astype(np.float32).astype(np.float64) for k, v in init_blocks(cfg, 0).items()}
    eps = np.random.default_rng(2).standard_normal((B * n, d)).astype(np.float32)
    adj = [batch.dense_adj(b) for b in range(B)]
    _, rg, _ = R.forward_backward(p, adj, batch.features, batch.feature_truth, batch.spatial_truth,
                                  eps.astype(np.float64), cfg)
    e32 = PB.e32_grads(p, adj, batch.features, batch.feature_truth, batch.spatial_truth, eps, cfg, rg)
    assert set(e32) == set(rg)
    assert all(0 <= e < 1e-3 for e in e32.values()), e32
    assert max(e32.values()) > 0            # it is an fp32 evaluation, not the float64 one


def test_bar_table_is_never_looser_than_the_fallback_and_rounds_up():
    table = json.load(open(PB.TABLE))
    assert table["factor"]["loss"] == 5.0 and table["factor"]["grad"] == 2.0
    for case, bars in table["bars"].items():
        assert case.endswith("/bf16"), case
        assert all(v > 0 for v in bars.values()), case
    b = PB.Bars("c2_bench_steps/bf16")
    assert b.bar("loss", "cost", 2e-2) <= 1e-4          # 5x the measured 1.3e-5
    assert b.bar("grad", "no.such.block", 0.1) == 0.1
    assert PB.round_up2(1.231e-5) == 1.3e-5 and PB.round_up2(0.05) == 0.05
