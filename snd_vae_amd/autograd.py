"""torch.autograd.Function wrappers over the C ABI (SURVEY §8b "Caller").

The reference builds its layers as TF graph ops and lets TF autodiff produce the
backward pass.  These wrappers give the same composability on torch tensors: each
forward and backward is one or a few libsndvae launches on the current stream
(no CPU path; a missing library raises), so a caller can assemble a model from the
reference's layers and call ``loss.backward()``.  The fused training step
(``snd_train_step``) remains the throughput path; these serve models the plan does
not cover and tests that compose the layers with torch code.

    spmm(rowptr, colidx, h)                      A @ h           (layers.py:122)
    linear(x, w, b)                              x @ w + b       (layers.py:566-576)
    graph_convolution(rowptr, colidx, x, w, gamma, beta)
                                                 BN(lrelu(A (x w))) (layers.py:115-125 + model.py:107)
    conv1d_same(x, w, b, gamma, beta, n_per_graph)
                                                 lrelu(BN(conv1d(x) + b)) (model_joint.py:115-116)
    reparameterize(mu, logstd, eps)              mu + eps e^logstd (model.py:153-159)
    inner_product_ce(z, rowptr, colidx, n_graphs) sum of the 2-class CE over all pairs
                                                 (layers.py:407-409, model.py:205-207, optimizer.py:142-144)

The adjacency is symmetric (input_data.py:62-67 asserts it), so A^T dY = A dY.
All tensors are contiguous float32 on the device; the index arrays int32.
"""
from __future__ import annotations

import torch

from . import _lib

_P = _lib.ptr
_BNC = 1.0 / (1.0 + 1e-3) ** 0.5   # frozen Keras BN: gamma / sqrt(1 + eps)


def _f32(*ts):
    for t in ts:
        if t is not None and not (t.is_cuda and t.is_contiguous() and t.dtype == torch.float32):
            raise ValueError("snd_vae_amd.autograd: contiguous float32 device tensors expected")


def _gemm(ta, tb, m, n, k, a, lda, b, ldb, c, ldc, bias=None):
    _lib.check(_lib.lib().snd_gemm(int(ta), int(tb), m, n, k, _P(a), lda, _P(b), ldb, _P(c), ldc,
                                   _P(bias), 0, _lib.stream_ptr()), "snd_gemm")


def _colsum(g):
    """Sum over rows of g [m, n] -> [n] (1^T g on the GEMM)."""
    m, n = g.shape
    ones = torch.ones(m, 1, device=g.device)
    out = torch.empty(1, n, device=g.device)
    _gemm(1, 0, 1, n, m, ones, 1, g, n, out, n)
    return out.view(n)


def _spmm(rowptr, colidx, h):
    rows, width = h.shape
    out = torch.empty(rows, width, device=h.device)
    _lib.check(_lib.lib().snd_csr_spmm(
        _P(rowptr), _P(colidx), rows, _P(h), width, width, _P(out), width, 0, None, None, None, 0,
        None, 0, 0, None, None, None, 0, _lib.stream_ptr()), "snd_csr_spmm")
    return out


class _SpMM(torch.autograd.Function):
    @staticmethod
    def forward(ctx, rowptr, colidx, h):
        _f32(h)
        ctx.save_for_backward(rowptr, colidx)
        return _spmm(rowptr, colidx, h)

    @staticmethod
    def backward(ctx, g):
        rowptr, colidx = ctx.saved_tensors
        return None, None, _spmm(rowptr, colidx, g.contiguous())


def spmm(rowptr, colidx, h):
    """A @ h over the block-diagonal CSR (tf.matmul(adj, x), layers.py:122)."""
    return _SpMM.apply(rowptr, colidx, h)


class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        _f32(x, w, b)
        m, k = x.shape
        n = w.shape[1]
        out = torch.empty(m, n, device=x.device)
        _gemm(0, 0, m, n, k, x, k, w, n, out, n, b)
        ctx.save_for_backward(x, w)
        ctx.has_b = b is not None
        return out

    @staticmethod
    def backward(ctx, g):
        x, w = ctx.saved_tensors
        g = g.contiguous()
        m, k = x.shape
        n = w.shape[1]
        dx = torch.empty(m, k, device=x.device)
        dw = torch.empty(k, n, device=x.device)
        _gemm(0, 1, m, k, n, g, n, w, n, dx, k)          # dx = g w^T
        _gemm(1, 0, k, n, m, x, k, g, n, dw, n)          # dw = x^T g
        return dx, dw, (_colsum(g) if ctx.has_b else None)


def linear(x, w, b=None):
    """x @ w + b (linear, layers.py:566-576) on the MFMA GEMM, fp32."""
    return _Linear.apply(x, w, b)


def _bn_act_bwd(dx, y, gamma, beta, act, act_first):
    rows, c = y.shape
    dy = torch.empty_like(y)
    dg = torch.empty(c, device=y.device)
    db = torch.empty(c, device=y.device)
    _lib.check(_lib.lib().snd_bn_act_bwd(_P(dx), c, _P(y), c, rows, c, _P(gamma), _P(beta), act,
                                         int(act_first), _P(dy), c, _P(dg), _P(db), _lib.stream_ptr()),
               "snd_bn_act_bwd")
    return dy, dg, db


class _GraphConvolution(torch.autograd.Function):
    @staticmethod
    def forward(ctx, rowptr, colidx, x, w, gamma, beta):
        _f32(x, w, gamma, beta)
        rows, fin = x.shape
        width = w.shape[1]
        xw = torch.empty(rows, width, device=x.device)
        _gemm(0, 0, rows, width, fin, x, fin, w, width, xw, width)
        out = torch.empty(rows, width, device=x.device)
        pre = torch.empty(rows, width, device=x.device)
        _lib.check(_lib.lib().snd_csr_spmm(
            _P(rowptr), _P(colidx), rows, _P(xw), width, width, _P(out), width, 1, _P(gamma), _P(beta),
            _P(pre), width, None, 0, 0, None, None, None, 0, _lib.stream_ptr()), "snd_csr_spmm")
        ctx.save_for_backward(rowptr, colidx, x, w, gamma, beta, pre)
        return out

    @staticmethod
    def backward(ctx, g):
        rowptr, colidx, x, w, gamma, beta, pre = ctx.saved_tensors
        rows, fin = x.shape
        width = w.shape[1]
        dpre, dgamma, dbeta = _bn_act_bwd(g.contiguous(), pre, gamma, beta, 2, True)   # BN(lrelu(.))
        dxw = _spmm(rowptr, colidx, dpre)                                              # A^T = A
        dx = torch.empty(rows, fin, device=x.device)
        dw = torch.empty(fin, width, device=x.device)
        _gemm(0, 1, rows, fin, width, dxw, width, w, width, dx, fin)
        _gemm(1, 0, fin, width, rows, x, fin, dxw, width, dw, width)
        return None, None, dx, dw, dgamma, dbeta


def graph_convolution(rowptr, colidx, x, w, gamma, beta):
    """BN(lrelu(A (x w))): GraphConvolution (layers.py:115-125, keep_prob 1) followed by
    the frozen Keras BN of model.py:107 (gamma = 1, beta = 0 for the plain layer)."""
    return _GraphConvolution.apply(rowptr, colidx, x, w, gamma, beta)


class _Conv1dSame(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, gamma, beta, n_per_graph):
        _f32(x, w, b, gamma, beta)
        rows, cin = x.shape
        cout = w.shape[2]
        out = torch.empty(rows, cout, device=x.device)
        pre = torch.empty(rows, cout, device=x.device)
        _lib.check(_lib.lib().snd_conv1d_same_fwd(
            _P(x), cin, rows, n_per_graph, cin, _P(w), cout, _P(b), _P(gamma), _P(beta), _P(pre), cout,
            _P(out), cout, 0, _lib.stream_ptr()), "snd_conv1d_same_fwd")
        ctx.save_for_backward(x, w, gamma, beta, pre)
        ctx.npg = n_per_graph
        ctx.has_b = b is not None
        return out

    @staticmethod
    def backward(ctx, g):
        x, w, gamma, beta, pre = ctx.saved_tensors
        rows, cin = x.shape
        cout = w.shape[2]
        L = _lib.lib()
        dpre, dgamma, dbeta = _bn_act_bwd(g.contiguous(), pre, gamma, beta, 2, False)   # lrelu(BN(.))
        dx = torch.empty(rows, cin, device=x.device)
        _lib.check(L.snd_conv1d_same_bwd_data(_P(dpre), cout, rows, ctx.npg, cout, _P(w), cin, _P(dx), cin, 0,
                                              _lib.stream_ptr()), "snd_conv1d_same_bwd_data")
        nws = L.snd_conv1d_bwd_weight_workspace(rows, cin, cout)
        ws = torch.empty(max(nws, 16), dtype=torch.uint8, device=x.device)
        dw = torch.empty_like(w)
        _lib.check(L.snd_conv1d_same_bwd_weight(_P(x), cin, _P(dpre), cout, rows, ctx.npg, cin, cout, _P(dw),
                                                _P(ws), nws, 0, _lib.stream_ptr()), "snd_conv1d_same_bwd_weight")
        return dx, dw, (_colsum(dpre) if ctx.has_b else None), dgamma, dbeta, None


def conv1d_same(x, w, b, gamma, beta, n_per_graph):
    """lrelu(BN(conv1d(x, k=5, SAME) + b)) over each graph's node axis
    (tf.layers.conv1d + Keras BN + lrelu, model_joint.py:115-116,138-139); w is the
    TF kernel [5][cin][cout]."""
    return _Conv1dSame.apply(x, w, b, gamma, beta, n_per_graph)


class _Reparameterize(torch.autograd.Function):
    @staticmethod
    def forward(ctx, mu, logstd, eps):
        _f32(mu, logstd, eps)
        rows, lat = mu.shape
        ms = torch.cat([mu, logstd], 1).contiguous()
        z = torch.empty(rows, lat, device=mu.device)
        kl = torch.empty(_lib.lib().snd_reparam_kl_blocks(rows, lat), dtype=torch.float64, device=mu.device)
        _lib.check(_lib.lib().snd_reparam_kl(_P(ms), 2 * lat, rows, lat, _P(eps), 0, None, None, _P(z), _P(kl),
                                             _lib.stream_ptr()), "snd_reparam_kl")
        ctx.save_for_backward(ms, eps)
        return z

    @staticmethod
    def backward(ctx, g):
        ms, eps = ctx.saved_tensors
        rows, lat = eps.shape
        dms = torch.empty_like(ms)
        _lib.check(_lib.lib().snd_reparam_bwd(_P(ms), 2 * lat, rows, lat, _P(eps), _P(g.contiguous()), None, None,
                                              _P(dms), 2 * lat, _lib.stream_ptr()), "snd_reparam_bwd")
        return dms[:, :lat], dms[:, lat:], None


def reparameterize(mu, logstd, eps):
    """z = mu + eps * exp(logstd) (get_z, model.py:153-159) with an injected eps."""
    return _Reparameterize.apply(mu, logstd, eps)


class _InnerProductCE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, z, rowptr, colidx, n_graphs, pos_weight, norm):
        _f32(z)
        rows, d = z.shape
        n = rows // n_graphs
        L = _lib.lib()
        wsb = L.snd_zzt_ce_workspace(n_graphs, n, d, 0)
        ws = torch.empty(max(wsb, 16), dtype=torch.uint8, device=z.device)
        stats = torch.zeros(2, dtype=torch.float64, device=z.device)
        dz = torch.empty_like(z)
        _lib.check(L.snd_zzt_ce(_P(z), n_graphs, n, d, _P(rowptr), _P(colidx), pos_weight, norm, _P(stats),
                                _P(dz), _P(ws), wsb, 0, _lib.stream_ptr()), "snd_zzt_ce")
        ctx.save_for_backward(dz)
        ctx.mark_non_differentiable(stats)
        return stats[0].float(), stats

    @staticmethod
    def backward(ctx, g, _):
        (dz,) = ctx.saved_tensors
        return dz * g, None, None, None, None, None


def inner_product_ce(z, rowptr, colidx, n_graphs, pos_weight=1.0, norm=1.0):
    """Sum over all B*N*N pairs of the 2-class softmax CE of the inner-product decoder
    (InnerProductDecoder, layers.py:407-409; diagonal rule model.py:205-207; CE
    optimizer.py:142-144), fp32, fused with its gradient.  Returns (ce_sum, stats) with
    stats = [ce_sum, #correct] in float64 (the accuracy of main.py:334 is
    stats[1] / (B N^2)); divide ce_sum by B N^2 for the reference's mean."""
    return _InnerProductCE.apply(z, rowptr, colidx, n_graphs, float(pos_weight), float(norm))
