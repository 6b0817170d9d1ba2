"""snd_vae_amd.autograd (SURVEY §8b's torch.autograd.Function callers) against plain
PyTorch fp32 references of the same ops on the same GPU inputs: forward values and
every input gradient (upstream gradients random).  Tolerance: 1e-5 relative to the
tensor's max-abs (fp32 sums in a different order), 1e-4 for the CE sum over N^2 pairs."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from snd_vae_amd.config import tscale
from snd_vae_amd.data import synthetic_batch

pytestmark = pytest.mark.gpu
BNC = 1.0 / (1.0 + 1e-3) ** 0.5


@pytest.fixture(scope="module")
def case(lib_built):
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm device")
    cfg = tscale(96, 16, mean_degree=6.0)
    b = synthetic_batch(cfg, 2, seed=3)
    dev = torch.device("cuda", 0)
    A = torch.zeros(b.n_graphs * 96, b.n_graphs * 96, dtype=torch.float64)
    for g in range(b.n_graphs):
        A[g * 96:(g + 1) * 96, g * 96:(g + 1) * 96] = torch.from_numpy(b.dense_adj(g).astype(np.float64))
    return (torch.from_numpy(b.rowptr).to(dev), torch.from_numpy(b.colidx).to(dev), A.float().to(dev),
            b.n_graphs, 96, dev)


def _close(a, b, tol=1e-5):
    a, b = a.detach().double(), b.detach().double()
    assert float((a - b).abs().max()) <= tol * max(float(b.abs().max()), 1e-30)


def _leaf(*shape, dev, scale=1.0, gen=None):
    return (torch.randn(*shape, generator=gen) * scale).to(dev).requires_grad_(True)


def _check(fn_snd, fn_ref, inputs, upstream, tol=1e-5):
    out = fn_snd(*inputs)
    ref_in = [t.detach().clone().requires_grad_(True) for t in inputs]
    ref = fn_ref(*ref_in)
    _close(out, ref, tol)
    gs = torch.autograd.grad(out, inputs, upstream)
    gr = torch.autograd.grad(ref, ref_in, upstream)
    for a, b in zip(gs, gr):
        _close(a, b, tol)


def test_spmm_and_linear(case):
    from snd_vae_amd import autograd as AG
    rp, ci, A, B, n, dev = case
    gen = torch.Generator().manual_seed(0)
    h = _leaf(B * n, 24, dev=dev, gen=gen)
    _check(lambda x: AG.spmm(rp, ci, x), lambda x: A @ x, [h], torch.randn(B * n, 24, generator=gen).to(dev))
    x, w, bias = _leaf(B * n, 19, dev=dev, gen=gen), _leaf(19, 32, dev=dev, gen=gen), _leaf(32, dev=dev, gen=gen)
    _check(AG.linear, lambda a, b_, c: a @ b_ + c, [x, w, bias], torch.randn(B * n, 32, generator=gen).to(dev))


def test_graph_convolution_bn(case):
    from snd_vae_amd import autograd as AG
    rp, ci, A, B, n, dev = case
    gen = torch.Generator().manual_seed(1)
    x, w = _leaf(B * n, 19, dev=dev, gen=gen), _leaf(19, 16, dev=dev, scale=0.3, gen=gen)
    g, b = _leaf(16, dev=dev, gen=gen), _leaf(16, dev=dev, gen=gen)
    _check(lambda x_, w_, g_, b_: AG.graph_convolution(rp, ci, x_, w_, g_, b_),
           lambda x_, w_, g_, b_: F.leaky_relu(A @ (x_ @ w_), 0.2) * (g_ * BNC) + b_,
           [x, w, g, b], torch.randn(B * n, 16, generator=gen).to(dev))


def test_conv1d_same_bn_lrelu(case):
    from snd_vae_amd import autograd as AG
    _, _, _, B, n, dev = case
    gen = torch.Generator().manual_seed(2)
    x, w, bias = _leaf(B * n, 12, dev=dev, gen=gen), _leaf(5, 12, 20, dev=dev, scale=0.2, gen=gen), \
        _leaf(20, dev=dev, gen=gen)
    g, b = _leaf(20, dev=dev, gen=gen), _leaf(20, dev=dev, gen=gen)

    def ref(x_, w_, bias_, g_, b_):   # per graph: SAME padding never crosses graphs
        xt = x_.view(B, n, 12).transpose(1, 2)
        y = F.conv1d(xt, w_.permute(2, 1, 0), bias_, padding=2).transpose(1, 2).reshape(B * n, 20)
        return F.leaky_relu(y * (g_ * BNC) + b_, 0.2)

    _check(lambda *a: AG.conv1d_same(*a, n), ref, [x, w, bias, g, b], torch.randn(B * n, 20, generator=gen).to(dev))


def test_reparameterize(case):
    from snd_vae_amd import autograd as AG
    _, _, _, B, n, dev = case
    gen = torch.Generator().manual_seed(3)
    mu, ls = _leaf(B * n, 16, dev=dev, gen=gen), _leaf(B * n, 16, dev=dev, scale=0.3, gen=gen)
    eps = torch.randn(B * n, 16, generator=gen).to(dev)
    _check(lambda m_, s_: AG.reparameterize(m_, s_, eps), lambda m_, s_: m_ + eps * torch.exp(s_),
           [mu, ls], torch.randn(B * n, 16, generator=gen).to(dev))


def test_inner_product_ce(case):
    """CE sum over all B N^2 pairs (off-diagonal softplus(L) - A L, diagonal softplus(-1)
    without gradient, model.py:205-207) and the argmax-correct count, with dz."""
    from snd_vae_amd import autograd as AG
    rp, ci, A, B, n, dev = case
    gen = torch.Generator().manual_seed(4)
    z = _leaf(B * n, 16, dev=dev, scale=0.5, gen=gen)
    ce, stats = AG.inner_product_ce(z, rp, ci, B)
    zr = z.detach().double().clone().requires_grad_(True)
    tot, correct = 0.0, 0
    off = ~torch.eye(n, dtype=torch.bool, device=dev)
    for g in range(B):
        zg = zr[g * n:(g + 1) * n]
        L = zg @ zg.T
        Ag = A[g * n:(g + 1) * n, g * n:(g + 1) * n].double()
        tot = tot + ((F.softplus(L) - Ag * L)[off]).sum() + n * F.softplus(torch.tensor(-1.0, dtype=torch.float64))
        correct += int((((L > 0).double() == Ag) & off).sum()) + n
    _close(ce, tot, 1e-4)
    assert int(stats[1].item()) == correct
    gz, = torch.autograd.grad(ce, z)
    gr, = torch.autograd.grad(tot, zr)
    _close(gz, gr, 1e-4)
