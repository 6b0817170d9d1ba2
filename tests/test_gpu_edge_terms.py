"""The bf16 step's per-edge CE terms against a float64 evaluation on the step's own bf16 z.

The weighted cross entropy of the A = 1 pairs (optimizer.py:142-144 with main.py:246's
pos_weight) is evaluated per edge by the fused backward head (`head_bwd_kernel`, or
`edge_bf16_kernel` on the unfused path): logit L_ij = z_i . z_j over the bf16 z of the
step (plan buffer ZB), loss (pos_weight - 1) softplus(L) - pos_weight L, and the count
of L > 0 for the accuracy.  Both land in the plan's per-tile partials (PEDGE, float64
{loss, count}).  Here they are recomputed in float64 from the same bf16 z (products of
bf16 values are exact, so the only device error is the fp32 sum of 64 products and the
fp32 transcendentals): the loss within 1e-6 of sum |term|, the count exact away from
|L| < 1e-3.  The end-to-end step tests cannot see a wrong logit at pos_weight = 1 (the
reference's effective value): the edge gradient is then -sum z_j,
independent of L, and the edge loss sum -L is a small part of adj_cost.
"""
import dataclasses

import numpy as np
import pytest
import torch

from snd_vae_amd.config import tscale
from snd_vae_amd.data import synthetic_batch
from snd_vae_amd.params import init_blocks

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu(lib_built):
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm device")


@pytest.mark.timeout(300)
@pytest.mark.parametrize("pos_weight", [1.0, 37.5])
@pytest.mark.parametrize("debug", [0, 262144])   # fused backward head | edge_bf16_kernel chain
def test_edge_terms_vs_float64(pos_weight, debug):
    from snd_vae_amd import _lib
    from snd_vae_amd.model import DeviceBatch, SGCNModelVAE
    from snd_vae_amd.optimizer import OptimizerVAE
    n, B = 1024, 2
    cfg = dataclasses.replace(tscale(n, 64), pos_weight=pos_weight)
    batch = synthetic_batch(cfg, B, seed=21)
    p0 = init_blocks(cfg, 4)
    _lib.check(_lib.lib().snd_debug_set(debug))
    try:
        model = SGCNModelVAE(cfg, B, dtype="bf16", blocks=p0)
    finally:
        _lib.check(_lib.lib().snd_debug_set(0))
    opt = OptimizerVAE(model, fuse_adam=False)
    opt.forward_backward(DeviceBatch(batch))
    torch.cuda.synchronize()
    R, L = B * n, cfg.latent
    z = model.buffer("ZB", torch.bfloat16)[:R * L].view(R, L).double().cpu().numpy()
    # backward-head tile rows as head_bwd_rows (snd_head.hip): 128; 64 below 128 tiles of
    # 128 rows; 32 below 128 tiles of 64 rows
    rows = 128 if (R + 127) // 128 >= 128 else (32 if (R + 63) // 64 < 128 else 64)
    tiles = (R + rows - 1) // rows
    pe = model.buffer("PEDGE", torch.float64).cpu().numpy()
    got_loss = float(pe[0:2 * tiles:2].sum()) if debug == 0 else float(pe[0::2].sum())
    got_tp = float(pe[1:2 * tiles:2].sum()) if debug == 0 else float(pe[1::2].sum())
    rows = np.repeat(np.arange(R), np.diff(batch.rowptr))
    Lij = np.einsum("ek,ek->e", z[rows], z[batch.colidx])
    sp = np.maximum(Lij, 0) + np.log1p(np.exp(-np.abs(Lij)))
    terms = (pos_weight - 1.0) * sp - pos_weight * Lij
    ref_loss = float(terms.sum())
    assert abs(got_loss - ref_loss) <= 1e-6 * float(np.abs(terms).sum()), (got_loss, ref_loss)
    amb = int(np.sum(np.abs(Lij) < 1e-3))
    ref_tp = int(np.sum(Lij > 0))
    assert abs(got_tp - ref_tp) <= amb, (got_tp, ref_tp, amb)
