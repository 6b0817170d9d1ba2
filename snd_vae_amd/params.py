"""Parameter layout of the SND-VAE hot path (both decoder-input topologies).

The reference keeps one TF variable per layer in the variable store, keyed by
variable_scope (`layers.py:115-125`, `layers.py:566-576`, Keras BN and
``tf.layers.conv1d`` in `model.py`/`model_joint.py`).  On MI355X all trainable
state lives in ONE flat fp32 buffer (params, grads, Adam m and v share the
layout) so that the DP all-reduce is a single RCCL call and the TF1-Adam step
is one kernel.  Blocks are 64-float aligned.

Physical blocks fuse layers that read the same input:
* ``enc.Wms`` = [g_g2_lin/Matrix || g_g3_lin/Matrix]: mu and log-std heads in
  one GEMM (`model.py:114-115`).
* ``dec.K1`` = [s1_deconv || n0_deconv] along Cout: the spatial and node
  decoders' first conv1d both read J (`model_joint.py:112-115,129-138`).

``LOGICAL`` maps each reference variable name to (block, column slice).

Graph-latent (tref) layouts differ in two places: ``enc.Wh`` is the
[N*W, g_hidden] matrix of `model.py:113` (row index n*W + c, the row-major
tf.reshape of G), and the decoder projection ``dec.Wp`` [L, N*node_h] /
``dec.bp`` (`model_joint.py:97`, 'd_sg_lin1') follows the heads.
"""
from __future__ import annotations

from collections import OrderedDict
from dataclasses import dataclass
from typing import Dict, List, Tuple

import numpy as np

from .config import CONV_K, SNDConfig

ALIGN = 64


def sg_layer_shapes(f: int, hidden) -> "List[Tuple[str, Tuple[int, ...]]]":
    """One SpatialGraphConvolution layer's variables in the flat layer layout of
    snd_sg_param_count (include/snd_vae.h; layers.py:158-169, BN of model_joint.py:78)."""
    h0, h1, h2 = hidden
    return [("Matrix1", (3 * f + 3, h0)), ("bias1", (h0,)), ("Matrix2", (2 * f + 1 + h0, h1)),
            ("bias2", (h1,)), ("Matrix3", (f + h1, h2)), ("bias3", (h2,)), ("gamma", (h2,)),
            ("beta", (h2,))]


def sg_layer_inputs(cfg: SNDConfig) -> List[int]:
    """Input width of each spatial-graph layer."""
    return [cfg.f_in] + [h[2] for h in cfg.sg_conv_hidden[:-1]]


def block_shapes(cfg: SNDConfig) -> "OrderedDict[str, Tuple[int, ...]]":
    if cfg.topology not in ("tscale", "tref", "sgjoint"):
        raise ValueError(f"unknown topology {cfg.topology!r}")
    sg = cfg.topology == "sgjoint"
    tref = cfg.topology != "tscale"
    f, (h0, h1), gh, L, nh = (cfg.f_in, cfg.g_conv_hidden, cfg.g_hidden_size,
                              cfg.latent, cfg.node_h_size)
    if not tref and nh != L:
        raise ValueError("tscale requires node_h_size == latent (J = z)")
    n = cfg.n_nodes
    s1, s2, s3 = cfg.s_d_channel
    n1, n2 = cfg.n_d_channel
    k = CONV_K
    shapes = OrderedDict()
    if sg:
        if len(cfg.sg_conv_hidden) != 2:
            raise ValueError("sgjoint: two spatial-graph layers (the plan's encoder)")
        for i, (fi, hid) in enumerate(zip(sg_layer_inputs(cfg), cfg.sg_conv_hidden)):
            shapes[f"enc.sg{i}"] = (sum(int(np.prod(sh)) for _, sh in sg_layer_shapes(fi, hid)),)
    else:
        shapes["enc.W0"] = (f, h0)
        shapes["enc.bn0.gamma"] = (h0,)
        shapes["enc.bn0.beta"] = (h0,)
        shapes["enc.W1"] = (h0 + f, h1)
        shapes["enc.bn1.gamma"] = (h1,)
        shapes["enc.bn1.beta"] = (h1,)
        shapes["enc.bne.gamma"] = (h1 + f,)
        shapes["enc.bne.beta"] = (h1 + f,)
    W = cfg.enc_width
    shapes["enc.Wh"] = ((n * W) if tref else W, gh)
    shapes["enc.bh"] = (gh,)
    shapes["enc.Wms"] = (gh, 2 * L)
    shapes["enc.bms"] = (2 * L,)
    if tref:
        shapes["dec.Wp"] = (L, n * nh)
        shapes["dec.bp"] = (n * nh,)
    shapes["dec.K1"] = (k, nh, s1 + n1)
    shapes["dec.b1"] = (s1 + n1,)
    shapes["dec.bn1.gamma"] = (s1 + n1,)
    shapes["dec.bn1.beta"] = (s1 + n1,)
    shapes["dec.K2s"] = (k, s1, s2)
    shapes["dec.b2s"] = (s2,)
    shapes["dec.bn2s.gamma"] = (s2,)
    shapes["dec.bn2s.beta"] = (s2,)
    shapes["dec.K2n"] = (k, n1, n2)
    shapes["dec.b2n"] = (n2,)
    shapes["dec.bn2n.gamma"] = (n2,)
    shapes["dec.bn2n.beta"] = (n2,)
    shapes["dec.K3s"] = (k, s2, s3)
    shapes["dec.b3s"] = (s3,)
    shapes["dec.bn3s.gamma"] = (s3,)
    shapes["dec.bn3s.beta"] = (s3,)
    shapes["dec.Ws"] = (s3, cfg.spatial_dim)
    shapes["dec.bs"] = (cfg.spatial_dim,)
    shapes["dec.Wn"] = (n2, cfg.num_feature)
    shapes["dec.bn"] = (cfg.num_feature,)
    return shapes


def logical_names(cfg: SNDConfig) -> Dict[str, tuple]:
    """Reference variable name -> (physical block, slice on the last axis), or for a
    variable stored flattened inside a block (the spatial-graph layers) (block, flat
    slice, the variable's shape)."""
    L = cfg.latent
    s1 = cfg.s_d_channel[0]
    n1 = cfg.n_d_channel[0]
    full = slice(None)
    m = {
        "encoder/g_g0_conv/w": ("enc.W0", full),
        "encoder/g_bn_g0/gamma": ("enc.bn0.gamma", full),
        "encoder/g_bn_g0/beta": ("enc.bn0.beta", full),
        "encoder/g_g1_conv/w": ("enc.W1", full),
        "encoder/g_bn_g1/gamma": ("enc.bn1.gamma", full),
        "encoder/g_bn_g1/beta": ("enc.bn1.beta", full),
        "encoder/encoder_g/gamma": ("enc.bne.gamma", full),
        "encoder/encoder_g/beta": ("enc.bne.beta", full),
        "encoder/g_g1_lin/Matrix": ("enc.Wh", full),
        "encoder/g_g1_lin/bias": ("enc.bh", full),
        "encoder/g_g2_lin/Matrix": ("enc.Wms", slice(0, L)),
        "encoder/g_g2_lin/bias": ("enc.bms", slice(0, L)),
        "encoder/g_g3_lin/Matrix": ("enc.Wms", slice(L, 2 * L)),
        "encoder/g_g3_lin/bias": ("enc.bms", slice(L, 2 * L)),
        "decoder/d_sg_lin1/Matrix": ("dec.Wp", full),
        "decoder/d_sg_lin1/bias": ("dec.bp", full),
        "decoder/s1_deconv/kernel": ("dec.K1", slice(0, s1)),
        "decoder/s1_deconv/bias": ("dec.b1", slice(0, s1)),
        "decoder/d_bn_s0/gamma": ("dec.bn1.gamma", slice(0, s1)),
        "decoder/d_bn_s0/beta": ("dec.bn1.beta", slice(0, s1)),
        "decoder/n0_deconv/kernel": ("dec.K1", slice(s1, s1 + n1)),
        "decoder/n0_deconv/bias": ("dec.b1", slice(s1, s1 + n1)),
        "decoder/d_bn_n0/gamma": ("dec.bn1.gamma", slice(s1, s1 + n1)),
        "decoder/d_bn_n0/beta": ("dec.bn1.beta", slice(s1, s1 + n1)),
        "decoder/s2_deconv/kernel": ("dec.K2s", full),
        "decoder/s2_deconv/bias": ("dec.b2s", full),
        "decoder/d_bn_s1/gamma": ("dec.bn2s.gamma", full),
        "decoder/d_bn_s1/beta": ("dec.bn2s.beta", full),
        "decoder/n1_deconv/kernel": ("dec.K2n", full),
        "decoder/n1_deconv/bias": ("dec.b2n", full),
        "decoder/d_bn_n1/gamma": ("dec.bn2n.gamma", full),
        "decoder/d_bn_n1/beta": ("dec.bn2n.beta", full),
        "decoder/s3_deconv/kernel": ("dec.K3s", full),
        "decoder/s3_deconv/bias": ("dec.b3s", full),
        "decoder/d_bn_s2/gamma": ("dec.bn3s.gamma", full),
        "decoder/d_bn_s2/beta": ("dec.bn3s.beta", full),
        "decoder/d_s_lin2/Matrix": ("dec.Ws", full),
        "decoder/d_s_lin2/bias": ("dec.bs", full),
        "decoder/d_n_lin2/Matrix": ("dec.Wn", full),
        "decoder/d_n_lin2/bias": ("dec.bn", full),
    }
    if cfg.topology == "tscale":
        del m["decoder/d_sg_lin1/Matrix"], m["decoder/d_sg_lin1/bias"]
    if cfg.topology == "sgjoint":   # model_joint.py:72-85: g_sg<i>_conv, g_bn_sg<i>, g_sg1..3_lin
        for k in [k for k in m if k.startswith("encoder/")]:
            del m[k]
        for i, (fi, hid) in enumerate(zip(sg_layer_inputs(cfg), cfg.sg_conv_hidden)):
            o = 0
            for name, shp in sg_layer_shapes(fi, hid):
                size = int(np.prod(shp))
                ref = (f"encoder/g_bn_sg{i}/{name}" if name in ("gamma", "beta")
                       else f"encoder/g_sg{i}_conv/{name}")
                m[ref] = (f"enc.sg{i}", slice(o, o + size), shp)
                o += size
        m.update({"encoder/g_sg1_lin/Matrix": ("enc.Wh", full), "encoder/g_sg1_lin/bias": ("enc.bh", full),
                  "encoder/g_sg2_lin/Matrix": ("enc.Wms", slice(0, L)),
                  "encoder/g_sg2_lin/bias": ("enc.bms", slice(0, L)),
                  "encoder/g_sg3_lin/Matrix": ("enc.Wms", slice(L, 2 * L)),
                  "encoder/g_sg3_lin/bias": ("enc.bms", slice(L, 2 * L))})
    return m


@dataclass
class FlatLayout:
    shapes: "OrderedDict[str, Tuple[int, ...]]"
    offsets: Dict[str, int]
    total: int

    def numel(self, name: str) -> int:
        return int(np.prod(self.shapes[name]))

    def view(self, flat, name: str):
        o = self.offsets[name]
        return flat[o:o + self.numel(name)].reshape(self.shapes[name])

    def pack(self, blocks: Dict[str, np.ndarray], dtype=np.float32) -> np.ndarray:
        flat = np.zeros(self.total, dtype)
        for k in self.shapes:
            self.view(flat, k)[...] = blocks[k]
        return flat

    def unpack(self, flat) -> Dict[str, np.ndarray]:
        return {k: np.array(self.view(flat, k)) for k in self.shapes}


def flat_layout(cfg: SNDConfig) -> FlatLayout:
    shapes = block_shapes(cfg)
    offsets, off = {}, 0
    for k, s in shapes.items():
        offsets[k] = off
        off += -(-int(np.prod(s)) // ALIGN) * ALIGN
    return FlatLayout(shapes, offsets, off)


def _truncated_normal(rng, shape, std):
    """tf.truncated_normal_initializer: resample draws beyond 2 std."""
    x = rng.standard_normal(shape)
    bad = np.abs(x) > 2.0
    while bad.any():
        x[bad] = rng.standard_normal(int(bad.sum()))
        bad = np.abs(x) > 2.0
    return x * std


def _glorot_uniform(rng, shape):
    """tf.layers.conv1d default kernel init; fan over receptive field."""
    k, cin, cout = shape
    lim = np.sqrt(6.0 / (k * cin + k * cout))
    return rng.uniform(-lim, lim, shape)


def init_blocks(cfg: SNDConfig, seed: int = 0) -> Dict[str, np.ndarray]:
    """Reference initialisers (layers.py:119, 569-572; conv glorot; BN 1/0)."""
    rng = np.random.default_rng(seed)
    shapes = block_shapes(cfg)
    out: Dict[str, np.ndarray] = {}
    L = cfg.latent
    s1 = cfg.s_d_channel[0]
    for k, s in shapes.items():
        if k.startswith("enc.sg"):                        # layers.py:158-169 + Keras BN
            i = int(k[6:])
            fi, hid = sg_layer_inputs(cfg)[i], cfg.sg_conv_hidden[i]
            parts = []
            for name, shp in sg_layer_shapes(fi, hid):
                if name.startswith("Matrix"):
                    parts.append(rng.normal(0.0, 0.02, shp).reshape(-1))
                else:
                    parts.append((np.ones(shp) if name == "gamma" else np.zeros(shp)).reshape(-1))
            v = np.concatenate(parts)
        elif k in ("enc.W0", "enc.W1"):
            v = _truncated_normal(rng, s, 0.02)           # GraphConvolution w
        elif k in ("enc.Wh", "dec.Ws", "dec.Wn", "dec.Wp"):
            v = rng.normal(0.0, 0.02, s)                  # linear Matrix
        elif k == "enc.Wms":
            v = np.concatenate([rng.normal(0.0, 0.02, (s[0], L)),
                                rng.normal(0.0, 0.02, (s[0], L))], 1)
        elif k == "dec.K1":
            v = np.concatenate([_glorot_uniform(rng, (s[0], s[1], s1)),
                                _glorot_uniform(rng, (s[0], s[1], s[2] - s1))], 2)
        elif k.startswith("dec.K"):
            v = _glorot_uniform(rng, s)
        elif k.endswith(".gamma"):
            v = np.ones(s)
        else:
            v = np.zeros(s)                               # biases, BN beta
        out[k] = v.astype(np.float64)
    return out
