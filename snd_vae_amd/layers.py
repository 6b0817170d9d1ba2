"""Functional hot-path ops over torch device tensors, backed by libsndvae.so.

Named after the reference layer functions they replace (`layers.py`):
``GraphConvolution`` (:115-125), ``linear`` (:566-576), ``InnerProductDecoder``
(:400-410) fused with the CE of `optimizer.py:142-144`, ``conv1d`` SAME as
used by the decoders (`model_joint.py:115,138`).  The reference versions
create TF variables under a variable_scope; these take the weights
explicitly (the flat parameter buffer owns them, `params.py`).  Forward
only, except where the reference's loss gradient is fused (CE, MSE).
Every call is one or a few HIP launches on the current stream; there is no
CPU path.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import _lib
from .model import DTYPES

_P = _lib.ptr


def _dt(dtype):
    return DTYPES[dtype] if isinstance(dtype, str) else int(dtype)


def _need(t, name):
    if not (t.is_cuda and t.is_contiguous() and t.dtype == torch.float32):
        raise ValueError(f"{name}: expected a contiguous float32 device tensor")


def graph_convolution(rowptr, colidx, h, w, gamma=None, beta=None, concat_x=None,
                      enc_gamma=None, enc_beta=None, dtype="f32"):
    """GraphConvolution(adj, h, out) + BN + concat (model.py:107-112).

    Returns (out, preact[, out2]).  Without gamma/beta: plain lrelu(A (h w))
    is not separable from BN in the fused kernel, so gamma=1, beta=0 is used.
    """
    rows, fin = h.shape
    width = w.shape[1]
    xw = linear(h, w, None, dtype)
    if gamma is None:
        gamma = torch.ones(width, device=h.device)
        beta = torch.zeros(width, device=h.device)
    fx = 0 if concat_x is None else concat_x.shape[1]
    out = torch.empty(rows, width + fx, device=h.device)
    pre = torch.empty(rows, width, device=h.device)
    out2 = torch.empty_like(out) if enc_gamma is not None else None
    _lib.check(_lib.lib().snd_csr_spmm(
        _P(rowptr), _P(colidx), rows, _P(xw), width, width, _P(out), width + fx, 1,
        _P(gamma), _P(beta), _P(pre), width, _P(concat_x), fx, fx, _P(enc_gamma),
        _P(enc_beta), _P(out2), width + fx, _lib.stream_ptr()), "snd_csr_spmm")
    return (out, pre, out2) if out2 is not None else (out, pre)


def spmm(rowptr, colidx, h):
    """A @ h on the block-diagonal CSR (tf.matmul(adj, x), layers.py:122)."""
    _need(h, "spmm")
    rows, width = h.shape
    out = torch.empty_like(h)
    _lib.check(_lib.lib().snd_csr_spmm(
        _P(rowptr), _P(colidx), rows, _P(h), width, width, _P(out), width, 0, 0, 0, 0, 0,
        0, 0, 0, 0, 0, 0, 0, _lib.stream_ptr()), "snd_csr_spmm")
    return out


def spmm_bf16(rowptr, colidx, h, n_per_graph=0, n_graphs=0, row_order=None):
    """A @ h over bf16 rows, fp32 accumulation (the bf16 path's SpMM, layers.py:122).

    n_per_graph / n_graphs let the kernel keep each graph's row blocks on one XCD;
    row_order (int32 device tensor, data.locality_order) is the processing schedule."""
    if not (h.is_cuda and h.is_contiguous() and h.dtype == torch.bfloat16):
        raise ValueError("spmm_bf16: expected a contiguous bfloat16 device tensor")
    rows, width = h.shape
    out = torch.empty_like(h)
    _lib.check(_lib.lib().snd_csr_spmm_bf16(
        _P(rowptr), _P(colidx), rows, _P(h), width, width, _P(out), width, n_per_graph,
        n_graphs, _P(row_order), _lib.stream_ptr()), "snd_csr_spmm_bf16")
    return out


def spmm_bf16_tiled(rowptr, colidx, tiles, h, n_per_graph=0, n_graphs=0, row_order=None):
    """spmm_bf16 over row tiles (snd_csr_spmm_bf16_tiled): neighbour rows staged in LDS.

    tiles: model.DeviceTiles over the schedule row_order (data.row_tiles);
    bit-identical to spmm_bf16."""
    if not (h.is_cuda and h.is_contiguous() and h.dtype == torch.bfloat16):
        raise ValueError("spmm_bf16_tiled: expected a contiguous bfloat16 device tensor")
    rows, width = h.shape
    out = torch.empty_like(h)
    t = tiles.c_struct()
    _lib.check(_lib.lib().snd_csr_spmm_bf16_tiled(
        _P(rowptr), _P(colidx), rows, C.byref(t), _P(h), width, width, _P(out), width,
        n_per_graph, n_graphs, _P(row_order), _lib.stream_ptr()), "snd_csr_spmm_bf16_tiled")
    return out


class DeviceWindowPlan:
    """data.WindowPlan on the device (meta, slots, rows, order) for spmm_bf16_window."""

    def __init__(self, plan, device="cuda"):
        self.meta = torch.from_numpy(plan.meta).to(device)
        self.slots = torch.from_numpy(plan.slots.view(np.int16)).to(device)
        self.rows = torch.from_numpy(plan.rows).to(device)
        self.order = torch.from_numpy(plan.order).to(device)
        self.beta = plan.beta


def spmm_bf16_window(wplan, h, n_per_graph, n_graphs):
    """spmm_bf16 streamed through an LDS window (snd_csr_spmm_bf16_window; plan:
    data.window_plan): bit-identical to spmm_bf16 on every tested batch.
    wplan: DeviceWindowPlan."""
    if not (h.is_cuda and h.is_contiguous() and h.dtype == torch.bfloat16):
        raise ValueError("spmm_bf16_window: expected a contiguous bfloat16 device tensor")
    rows, width = h.shape
    out = torch.empty_like(h)
    L = _lib.lib()
    fn, name = L.snd_csr_spmm_bf16_window, "snd_csr_spmm_bf16_window"
    _lib.check(fn(_P(wplan.meta), _P(wplan.slots), _P(wplan.rows), _P(wplan.order), rows, n_per_graph, n_graphs,
                  wplan.beta, _P(h), width, width, _P(out), width, _lib.stream_ptr()), name)
    return out


def linear(x, w, b=None, dtype="f32", trans_w=False):
    """x @ w + b (layers.py:566-576) on MFMA (fp32 or bf16 operands, fp32 acc)."""
    _need(x, "linear x")
    m, k = x.shape
    n = w.shape[0] if trans_w else w.shape[1]
    out = torch.empty(m, n, device=x.device)
    _lib.check(_lib.lib().snd_gemm(0, int(trans_w), m, n, k, _P(x), k, _P(w), w.shape[1],
                                   _P(out), n, _P(b), _dt(dtype), _lib.stream_ptr()), "snd_gemm")
    return out


def conv1d_same(x, w, b, n_per_graph, gamma=None, beta=None, dtype="f32"):
    """conv1d(k=5, SAME) [+ BN + lrelu] over each graph's node axis.

    Returns out (and y_pre when BN is applied)."""
    _need(x, "conv1d x")
    rows, cin = x.shape
    cout = w.shape[2]
    out = torch.empty(rows, cout, device=x.device)
    pre = torch.empty(rows, cout, device=x.device) if gamma is not None else None
    _lib.check(_lib.lib().snd_conv1d_same_fwd(
        _P(x), cin, rows, n_per_graph, cin, _P(w), cout, _P(b), _P(gamma), _P(beta), _P(pre),
        cout, _P(out), cout, _dt(dtype), _lib.stream_ptr()), "snd_conv1d_same_fwd")
    return (out, pre) if gamma is not None else out


def conv1d_same_bwd(x, w, dy, n_per_graph, dtype="f32"):
    """(dx, dw) of conv1d SAME (TF autodiff of tf.layers.conv1d)."""
    rows, cin = x.shape
    cout = w.shape[2]
    dx = torch.empty(rows, cin, device=x.device)
    _lib.check(_lib.lib().snd_conv1d_same_bwd_data(
        _P(dy), cout, rows, n_per_graph, cout, _P(w), cin, _P(dx), cin, _dt(dtype),
        _lib.stream_ptr()), "snd_conv1d_same_bwd_data")
    ws_n = _lib.lib().snd_conv1d_bwd_weight_workspace(rows, cin, cout)
    ws = torch.empty(max(ws_n, 4), dtype=torch.uint8, device=x.device)
    dw = torch.empty_like(w)
    _lib.check(_lib.lib().snd_conv1d_same_bwd_weight(
        _P(x), cin, _P(dy), cout, rows, n_per_graph, cin, cout, _P(dw), _P(ws), ws_n,
        _dt(dtype), _lib.stream_ptr()), "snd_conv1d_same_bwd_weight")
    return dx, dw


def inner_product_ce(z, n_graphs, rowptr, colidx, pos_weight=1.0, norm=1.0, dtype="bf16"):
    """InnerProductDecoder + diagonal rule + softmax CE, fused (no logits in HBM).

    Returns (ce_sum, n_correct, dz) with dz = d(ce_sum)/dz."""
    _need(z, "inner_product_ce z")
    rows, d = z.shape
    n = rows // n_graphs
    L = _lib.lib()
    wsb = L.snd_zzt_ce_workspace(n_graphs, n, d, _dt(dtype))
    ws = torch.empty(wsb, dtype=torch.uint8, device=z.device)
    stats = torch.zeros(2, dtype=torch.float64, device=z.device)
    dz = torch.empty_like(z)
    _lib.check(L.snd_zzt_ce(_P(z), n_graphs, n, d, _P(rowptr), _P(colidx), pos_weight, norm,
                            _P(stats), _P(dz), _P(ws), wsb, _dt(dtype), _lib.stream_ptr()),
               "snd_zzt_ce")
    s = stats.cpu()
    return float(s[0]), float(s[1]), dz


def inner_product_ce_rows(z, row0, row1, rowptr, colidx, pos_weight=1.0, norm=1.0, dtype="bf16"):
    """The fused CE of one graph's rows [row0, row1) against all its columns
    (snd_zzt_ce_rows; the row-sharded zz^T of SURVEY §8e): z [n, d] is the WHOLE graph,
    rowptr the range's row pointers (a slice of the graph's CSR), colidx global ids.

    Returns (stats, dz_rows): stats a float64 device tensor [ce_sum, n_correct] over the
    range (left on the device for the caller's all-reduce); dz_rows [row1 - row0, d] is
    d(ce_sum over ALL pairs)/dz for those rows (L symmetric: no reduction needed)."""
    _need(z, "inner_product_ce_rows z")
    n, d = z.shape
    L = _lib.lib()
    wsb = L.snd_zzt_ce_rows_workspace(n, d, row0, row1, _dt(dtype))
    if wsb == 0:
        raise _lib.SNDError(f"snd_zzt_ce_rows_workspace: bad shape n={n} d={d} rows [{row0}, {row1})")
    ws = torch.empty(wsb, dtype=torch.uint8, device=z.device)
    stats = torch.zeros(2, dtype=torch.float64, device=z.device)
    dz = torch.empty(row1 - row0, d, dtype=torch.float32, device=z.device)
    _lib.check(L.snd_zzt_ce_rows(_P(z), n, d, row0, row1, _P(rowptr), _P(colidx), pos_weight, norm,
                                 _P(stats), _P(dz), _P(ws), wsb, _dt(dtype), _lib.stream_ptr()),
               "snd_zzt_ce_rows")
    return stats, dz


def dense_to_csr(adj):
    """Reference dense adj_truth [B,N,N] -> (rowptr, colidx) on the device."""
    b, n, _ = adj.shape
    L = _lib.lib()
    rowptr = torch.empty(b * n + 1, dtype=torch.int32, device=adj.device)
    nnz = torch.zeros(1, dtype=torch.int32, device=adj.device)
    ws = torch.empty(L.snd_dense_to_csr_workspace(b, n), dtype=torch.uint8, device=adj.device)
    _lib.check(L.snd_dense_to_csr(_P(adj), b, n, _P(rowptr), 0, 0, _P(nnz), _P(ws), ws.numel(),
                                  _lib.stream_ptr()), "snd_dense_to_csr")
    total = int(rowptr[-1].item())
    colidx = torch.empty(max(total, 1), dtype=torch.int32, device=adj.device)
    _lib.check(L.snd_dense_to_csr(_P(adj), b, n, _P(rowptr), _P(colidx), total, _P(nnz), _P(ws),
                                  ws.numel(), _lib.stream_ptr()), "snd_dense_to_csr")
    return rowptr, colidx[:total]
