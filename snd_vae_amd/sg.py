"""Spatial-graph encoder: ``SpatialGraphConvolution`` (`layers.py:143-198`) and the
model_joint encoder stack (`model_joint.py:72-85`) on libsndvae.so.

The reference builds B x N x N x N message tensors; the HIP layer
(`csrc/snd_sg.hip`) is the factorised equivalent, O(nnz (h0 + deg)) plus row
GEMMs, with a hand-derived backward.  Inputs per batch: the symmetric CSR of
``adj`` (the sampled spanning trees, `input_data.py:76-83`, or adj_truth) and
the dense ``rel`` [B, N, N] (`2D_rel.npy` / 600, `input_data.py:59`).

Per-layer parameters live in one flat fp32 buffer (layout in
include/snd_vae.h): Matrix1, bias1, Matrix2, bias2, Matrix3, bias3 with the
reference initialisers (N(0, 0.02) matrices, zero biases; `layers.py:163-174`)
and the layer's frozen Keras BN gamma / beta (`model_joint.py:78`).
"""
from __future__ import annotations

import ctypes as C
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _lib

_P = _lib.ptr


def sg_param_shapes(f: int, hidden: Sequence[int]):
    h0, h1, h2 = hidden
    return [("Matrix1", (3 * f + 3, h0)), ("bias1", (h0,)), ("Matrix2", (2 * f + 1 + h0, h1)),
            ("bias2", (h1,)), ("Matrix3", (f + h1, h2)), ("bias3", (h2,)),
            ("gamma", (h2,)), ("beta", (h2,))]


def sg_pack(f: int, hidden: Sequence[int], blocks: dict) -> np.ndarray:
    """Flat parameter vector of one layer from named blocks (missing BN -> 1 / 0)."""
    parts = []
    for name, shp in sg_param_shapes(f, hidden):
        v = blocks.get(name)
        if v is None:
            v = np.ones(shp) if name == "gamma" else np.zeros(shp)
        v = np.asarray(v, np.float64)
        if v.shape != shp:
            raise ValueError(f"{name}: shape {v.shape} != {shp}")
        parts.append(v.reshape(-1))
    flat = np.concatenate(parts)
    n = _lib.lib().snd_sg_param_count(f, *hidden)
    assert flat.size == n, (flat.size, n)
    return flat


def sg_unpack(f: int, hidden: Sequence[int], flat) -> dict:
    flat = np.asarray(flat)
    out, o = {}, 0
    for name, shp in sg_param_shapes(f, hidden):
        n = int(np.prod(shp))
        out[name] = flat[o:o + n].reshape(shp)
        o += n
    return out


def init_sg_layer(f: int, hidden: Sequence[int], rng: np.random.Generator, stddev=0.02) -> dict:
    """`layers.py:163-174`: random_normal(stddev) matrices, constant(0) biases."""
    out = {}
    for name, shp in sg_param_shapes(f, hidden):
        if name.startswith("Matrix"):
            out[name] = rng.normal(0.0, stddev, shp)
        elif name == "gamma":
            out[name] = np.ones(shp)
        else:
            out[name] = np.zeros(shp)
    return out


class SGGraph:
    """Device-side adjacency + rel scalars of one batch (snd_sg_prep)."""

    def __init__(self, rowptr, colidx, n_per_graph: int, rel: torch.Tensor):
        dev = rel.device
        self.rowptr = torch.as_tensor(np.asarray(rowptr), dtype=torch.int32).to(dev)
        self.colidx = torch.as_tensor(np.asarray(colidx), dtype=torch.int32).to(dev)
        if self.colidx.numel() == 0:
            self.colidx = torch.zeros(1, dtype=torch.int32, device=dev)
        nnz = max(1, int(np.asarray(colidx).size))
        R = self.rowptr.numel() - 1
        if rel.shape != (R // n_per_graph, n_per_graph, n_per_graph) or rel.dtype != torch.float32:
            raise ValueError(f"rel must be float32 [B, N, N], got {tuple(rel.shape)} {rel.dtype}")
        self.rel = rel.contiguous()
        self.edge_lr = torch.empty(nnz, device=dev)
        self.edge_q = torch.empty(nnz, device=dev)
        self.edge_rev = torch.empty(nnz, dtype=torch.int32, device=dev)
        self.node_deg = torch.empty(R, device=dev)
        self.node_e = torch.empty(R, device=dev)
        self.n_rows, self.n_per_graph = R, n_per_graph
        self.c = _lib.SGGraph(_P(self.rowptr), _P(self.colidx), R, n_per_graph, _P(self.edge_lr),
                              _P(self.edge_q), _P(self.edge_rev), _P(self.node_deg),
                              _P(self.node_e))
        bad = torch.zeros(1, dtype=torch.int32, device=dev)
        _lib.check(_lib.lib().snd_sg_prep(C.byref(self.c), _P(self.rel), _P(bad),
                                          _lib.stream_ptr()), "snd_sg_prep")
        if int(bad.item()):
            raise ValueError(f"adjacency is not symmetric ({int(bad.item())} edges without "
                             "a reverse edge); the spatial-graph encoder needs adj == adj^T")


class SpatialGraphConvolution:
    """One encoder layer: y = SGConv(adj, x, rel); out = lrelu(BN(y)) when bn_act."""

    def __init__(self, f: int, hidden: Sequence[int], params: torch.Tensor, bn_act: bool = True):
        self.f, self.hidden = f, tuple(int(h) for h in hidden)
        n = _lib.lib().snd_sg_param_count(f, *self.hidden)
        if params.numel() != n or params.dtype != torch.float32 or not params.is_cuda:
            raise ValueError(f"params must be a float32 device tensor of {n} elements")
        self.params = params
        self.bn_act = bool(bn_act)
        self._ws = None

    def _workspace(self, R, dev):
        nb = int(_lib.lib().snd_sg_workspace(R, self.f, *self.hidden))
        if self._ws is None or self._ws.numel() < nb:
            self._ws = torch.zeros(nb, dtype=torch.uint8, device=dev)
        return self._ws

    def forward(self, g: SGGraph, x: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        R = g.n_rows
        if x.shape != (R, self.f) or not x.is_contiguous():
            raise ValueError(f"x must be contiguous [{R}, {self.f}]")
        h2 = self.hidden[2]
        y = torch.empty(R, h2, device=x.device)
        out = torch.empty_like(y) if self.bn_act else y
        ws = self._workspace(R, x.device)
        _lib.check(_lib.lib().snd_sg_layer_fwd(
            C.byref(g.c), _P(x), self.f, self.f, *self.hidden, _P(self.params), int(self.bn_act),
            _P(y), _P(out), _P(ws), _lib.stream_ptr()), "snd_sg_layer_fwd")
        self._saved = (g, x, y)
        return out, y

    def backward(self, dout: torch.Tensor, want_dx: bool = True):
        """Gradients of the last forward: (grads flat [param_count], dx or None)."""
        g, x, y = self._saved
        grads = torch.empty_like(self.params)
        dx = torch.empty_like(x) if want_dx else None
        _lib.check(_lib.lib().snd_sg_layer_bwd(
            C.byref(g.c), _P(x), self.f, self.f, *self.hidden, _P(self.params), int(self.bn_act),
            _P(y), _P(dout.contiguous()), _P(dx), self.f, _P(grads), _P(self._ws),
            _lib.stream_ptr()), "snd_sg_layer_bwd")
        return grads, dx


class SGEncoder:
    """`model_joint.py:77-80`: s_g = lrelu(BN(SGConv(adj, s_g, rel))) for every layer
    (dropout keep 1).  sg_conv_hidden defaults to the reference [[20,20,20],[50,50,50]]."""

    def __init__(self, f_in: int, sg_conv_hidden: Sequence[Sequence[int]] = ((20, 20, 20), (50, 50, 50)),
                 seed: int = 0, device="cuda", blocks: Optional[List[dict]] = None):
        rng = np.random.default_rng(seed)
        self.layers: List[SpatialGraphConvolution] = []
        f = f_in
        for i, hid in enumerate(sg_conv_hidden):
            b = blocks[i] if blocks is not None else init_sg_layer(f, hid, rng)
            flat = torch.from_numpy(sg_pack(f, hid, b).astype(np.float32)).to(device)
            self.layers.append(SpatialGraphConvolution(f, hid, flat))
            f = hid[2]
        self.out_width = f

    def forward(self, g: SGGraph, x: torch.Tensor) -> torch.Tensor:
        s = x
        for layer in self.layers:
            s, _ = layer.forward(g, s)
        return s

    def backward(self, dout: torch.Tensor, want_dx: bool = False):
        grads = [None] * len(self.layers)
        d = dout
        for i in range(len(self.layers) - 1, -1, -1):
            grads[i], d = self.layers[i].backward(d, want_dx=(i > 0 or want_dx))
        return grads, d
