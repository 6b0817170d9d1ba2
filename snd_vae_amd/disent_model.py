"""The reference's disentangled SND-VAE, assembled.

``SGCNModelVAE`` of `model.py:19-222` with the `optimizer.py:123-203` costs: three
encoders, three latents, three decoders --

* graph encoder (`model.py:104-115`): two GraphConvolution layers on adj_truth and
  the node features (BN after lrelu, the features concatenated back), BN
  encoder_g, flat heads g_g1_lin -> [g_g2_lin | g_g3_lin];
* spatial encoder (`model.py:119-129`): three conv1d(k=5, SAME) + BN + relu over the
  coordinates, BN encoder_s, flat heads g_s1..3_lin;
* spatial-graph encoder (`model.py:134-151`): two SpatialGraphConvolution layers over
  the B * sampling_num spanning-tree copies (lrelu after BN), BN encoder_sg, flat heads
  per copy g_sg1..3_lin;
* decoder (`model.py:172-222`): J_sg = mean over the copies of d_sg_lin1(z_sg)
  (`model.py:177,180`), J_s = d_s_lin1(z_s), J_g = d_g_lin1(z_g); node features from
  [J_sg | J_g] (conv1d + BN, no activation, x2; BN decoder_node; sigmoid(d_n_lin2)),
  the adjacency from [J_sg | J_g] through the e2e structure decoder
  (`disent.structure_decoder`), coordinates from [J_sg | J_s] (conv1d + BN x3,
  sigmoid(d_s_lin2));
* cost (`optimizer.py:142-203`): adj CE + node MSE + spatial MSE + the model_type's
  latent regularisers (`disent.disentangled_cost`), overall_loss in the reference order.

Every forward and backward operation is a HIP kernel of libsndvae.so reached through
the C ABI (GEMM, CSR SpMM with the GraphConvolution epilogue, conv1d, frozen-BN +
activation, SpatialGraphConvolution, reparameterisation, e2e, regularisers, sigmoid
MSE heads, TF1 Adam); torch only allocates, views and copies device memory.  The
reference's scale is small (N = 25, B = 10, S = 10: `main.py:100,173-217`), so the
model is a host-ordered composition of launches, not a fused plan.
"""
from __future__ import annotations

from collections import OrderedDict
from dataclasses import dataclass
from typing import Dict, Optional, Tuple

import numpy as np
import torch

from . import _lib
from .config import CONV_K
from .data import SGBatch
from .disent import disentangled_cost, structure_decoder
from .layers import conv1d_same_bwd, graph_convolution, spmm
from .params import _glorot_uniform, _truncated_normal, sg_layer_shapes
from .sg import SGGraph, SpatialGraphConvolution

_P = _lib.ptr


@dataclass(frozen=True)
class DisentangledConfig:
    """FLAGS of the synthetic2 dataset (`main.py:173-217`) the model reads."""
    n_nodes: int = 25
    num_feature: int = 1
    spatial_dim: int = 2
    g_conv_hidden: Tuple[int, ...] = (10, 20)                    # main.py:189
    g_hidden: int = 100                                          # g_hidden_size
    g_latent: int = 100
    s_channel: Tuple[int, ...] = (10, 10, 20)                    # main.py:181
    s_hidden: int = 100
    s_latent: int = 100
    sg_conv_hidden: Tuple[Tuple[int, int, int], ...] = ((20, 20, 20), (50, 50, 50))
    sg_hidden: int = 100
    sg_latent: int = 100
    sampling_num: int = 10                                       # main.py:100
    node_h: int = 20                                             # main.py:209
    n_d_channel: Tuple[int, ...] = (50, 20)                      # [:graph_deconv_layers]
    e_d_hidden: Tuple[int, ...] = (50, 20)                       # [:graph_deconv_layers]
    s_d_channel: Tuple[int, ...] = (50, 20, 10)
    model_type: str = "disentangled"                             # main.py:515
    beta: float = 1.0
    gamma: float = 1.0
    capacity: float = 0.0                                        # disentangled_C: C of the step
    learning_rate: float = 0.0008
    adam_beta1: float = 0.9
    adam_beta2: float = 0.999
    adam_eps: float = 1e-8

    def replace(self, **kw) -> "DisentangledConfig":
        import dataclasses
        return dataclasses.replace(self, **kw)


def _bn(shapes, name, c):
    shapes[name + "/gamma"] = (c,)
    shapes[name + "/beta"] = (c,)


def block_shapes(cfg: DisentangledConfig) -> "OrderedDict[str, Tuple[int, ...]]":
    """Variables by reference name (the mu / log-std heads of a group are one
    [hidden, 2 L] block '<..>23_lin' = [<..>2_lin | <..>3_lin])."""
    N, F, nh = cfg.n_nodes, cfg.num_feature, cfg.node_h
    s = OrderedDict()
    f = F
    for i, h in enumerate(cfg.g_conv_hidden):                    # layers.py:117-119
        s[f"g_g{i}_conv/w"] = (f, h)
        _bn(s, f"g_bn_g{i}", h)
        f = h + F
    _bn(s, "encoder_g", f)
    s["g_g1_lin/Matrix"], s["g_g1_lin/bias"] = (N * f, cfg.g_hidden), (cfg.g_hidden,)
    s["g_g23_lin/Matrix"], s["g_g23_lin/bias"] = (cfg.g_hidden, 2 * cfg.g_latent), (2 * cfg.g_latent,)
    c = cfg.spatial_dim
    for i, co in enumerate(cfg.s_channel):
        s[f"g_s{i + 1}_conv/kernel"], s[f"g_s{i + 1}_conv/bias"] = (CONV_K, c, co), (co,)
        _bn(s, f"g_bn_s{i}", co)
        c = co
    _bn(s, "encoder_s", c)
    s["g_s1_lin/Matrix"], s["g_s1_lin/bias"] = (N * c, cfg.s_hidden), (cfg.s_hidden,)
    s["g_s23_lin/Matrix"], s["g_s23_lin/bias"] = (cfg.s_hidden, 2 * cfg.s_latent), (2 * cfg.s_latent,)
    f = F
    for i, hid in enumerate(cfg.sg_conv_hidden):                 # SG layer + its BN (snd_sg layout)
        s[f"g_sg{i}_conv"] = (sum(int(np.prod(sh)) for _, sh in sg_layer_shapes(f, hid)),)
        f = hid[2]
    _bn(s, "encoder_sg", f)
    s["g_sg1_lin/Matrix"], s["g_sg1_lin/bias"] = (N * f, cfg.sg_hidden), (cfg.sg_hidden,)
    s["g_sg23_lin/Matrix"], s["g_sg23_lin/bias"] = (cfg.sg_hidden, 2 * cfg.sg_latent), (2 * cfg.sg_latent,)
    for g, lat in (("sg", cfg.sg_latent), ("s", cfg.s_latent), ("g", cfg.g_latent)):
        s[f"d_{g}_lin1/Matrix"], s[f"d_{g}_lin1/bias"] = (lat, N * nh), (N * nh,)
    c = 2 * nh
    for i, co in enumerate(cfg.n_d_channel):
        s[f"n{i}_deconv/kernel"], s[f"n{i}_deconv/bias"] = (CONV_K, c, co), (co,)
        _bn(s, f"d_bn_n{i}", co)
        c = co
    _bn(s, "decoder_node", c)
    s["d_n_lin2/Matrix"], s["d_n_lin2/bias"] = (c, F), (F,)
    c = 4 * nh                                                   # the pair [z_i | z_j] of [J_sg | J_g]
    for i, co in enumerate(cfg.e_d_hidden):
        _bn(s, f"d_bn_e{i}", c)
        s[f"e{i}_deconv/w1"], s[f"e{i}_deconv/biases1"] = (N, c, co), (co,)
        c = co
    _bn(s, "decoder_adj", c)
    s["d_e_lin2/Matrix"], s["d_e_lin2/bias"] = (c, 2), (2,)
    c = 2 * nh
    for i, co in enumerate(cfg.s_d_channel):
        s[f"s{i + 1}_deconv/kernel"], s[f"s{i + 1}_deconv/bias"] = (CONV_K, c, co), (co,)
        _bn(s, f"d_bn_s{i}", co)
        c = co
    s["d_s_lin2/Matrix"], s["d_s_lin2/bias"] = (c, cfg.spatial_dim), (cfg.spatial_dim,)
    return s


def init_blocks(cfg: DisentangledConfig, seed: int = 0) -> Dict[str, np.ndarray]:
    """The reference initialisers: GraphConvolution w and e2e w1 truncated-normal(0.02)
    (layers.py:119,435), linear Matrix N(0, 0.02) (layers.py:570), SG matrices
    N(0, 0.02) (layers.py:158-169), conv1d glorot-uniform, biases 0, BN gamma 1 beta 0."""
    rng = np.random.default_rng(seed)
    out = {}
    f = cfg.num_feature
    sg_in = {}
    for i, hid in enumerate(cfg.sg_conv_hidden):
        sg_in[f"g_sg{i}_conv"] = (f, hid)
        f = hid[2]
    for k, shp in block_shapes(cfg).items():
        if k in sg_in:
            fi, hid = sg_in[k]
            parts = [rng.normal(0.0, 0.02, sh).reshape(-1) if n.startswith("Matrix")
                     else (np.ones(sh) if n == "gamma" else np.zeros(sh)).reshape(-1)
                     for n, sh in sg_layer_shapes(fi, hid)]
            v = np.concatenate(parts)
        elif k.endswith("_conv/w") or k.endswith("/w1"):
            v = _truncated_normal(rng, shp, 0.02)
        elif k.endswith("/Matrix"):
            v = rng.normal(0.0, 0.02, shp)
        elif k.endswith("/kernel"):
            v = _glorot_uniform(rng, shp)
        elif k.endswith("/gamma"):
            v = np.ones(shp)
        else:
            v = np.zeros(shp)
        out[k] = v.astype(np.float64)
    return out


# ------------------------------------------------------------------------------ op helpers
def _gemm(a, b, c, m, n, k, ta=False, tb=False, lda=None, ldb=None, ldc=None, bias=None):
    """c[m, n] = op(a) op(b) (+ bias) on MFMA (snd_gemm, fp32); views with explicit strides."""
    lda = lda if lda is not None else (m if ta else k)
    ldb = ldb if ldb is not None else (k if tb else n)
    ldc = ldc if ldc is not None else n
    _lib.check(_lib.lib().snd_gemm(int(ta), int(tb), m, n, k, _P(a), lda, _P(b), ldb, _P(c), ldc, _P(bias), 0,
                                   _lib.stream_ptr()), "snd_gemm")


def _bn_act(y, ldy, rows, c, g, b, act, act_first, x, ldx):
    _lib.check(_lib.lib().snd_bn_act_fwd(_P(y), ldy, rows, c, _P(g), _P(b), act, int(act_first), _P(x), ldx,
                                         _lib.stream_ptr()), "snd_bn_act_fwd")


def _bn_act_bwd(dx, lddx, y, ldy, rows, c, g, b, act, act_first, dy, lddy, dg, db):
    _lib.check(_lib.lib().snd_bn_act_bwd(_P(dx), lddx, _P(y), ldy, rows, c, _P(g), _P(b), act, int(act_first),
                                         _P(dy), lddy, _P(dg), _P(db), _lib.stream_ptr()), "snd_bn_act_bwd")


def _add(x, ldx, y, ldy, rows, cols, alpha=1.0):
    _lib.check(_lib.lib().snd_add_strided(rows, cols, alpha, _P(x), ldx, _P(y), ldy, _lib.stream_ptr()),
               "snd_add_strided")


def _conv(x, ldx, rows, npg, cin, w, cout, bias, out):
    _lib.check(_lib.lib().snd_conv1d_same_fwd(_P(x), ldx, rows, npg, cin, _P(w), cout, _P(bias), None, None,
                                              None, cout, _P(out), cout, 0, _lib.stream_ptr()),
               "snd_conv1d_same_fwd")


RELU, LRELU, IDENT = 1, 2, 0


class DisentangledSGCNModelVAE:
    """Parameters (one flat fp32 buffer), TF1 Adam state and the training step of the
    disentangled model for batches of ``n_graphs`` SGBatch graphs on one GPU."""

    def __init__(self, cfg: DisentangledConfig, n_graphs: int, blocks: Optional[Dict[str, np.ndarray]] = None,
                 seed: int = 0, device="cuda"):
        if not torch.cuda.is_available():
            raise _lib.SNDError("the disentangled model needs a ROCm GPU (no CPU fallback)")
        self.cfg, self.B, self.device = cfg, n_graphs, device
        self.shapes = block_shapes(cfg)
        self.offsets, off = {}, 0
        for k, shp in self.shapes.items():
            self.offsets[k] = off
            off += -(-int(np.prod(shp)) // 64) * 64
        self.param_count = off
        self.params = torch.zeros(off, device=device)
        self.grads = torch.zeros(off, device=device)
        self.m = torch.zeros(off, device=device)
        self.v = torch.zeros(off, device=device)
        self.step_counter = torch.zeros(1, dtype=torch.int32, device=device)
        self.load_blocks(blocks if blocks is not None else init_blocks(cfg, seed))
        S, B = cfg.sampling_num, n_graphs
        avg = np.zeros((B, B * S), np.float32)                   # zbar = avg @ z_sg (model.py:180)
        for b in range(B):
            avg[b, b * S:(b + 1) * S] = 1.0 / S
        self._avg = torch.from_numpy(avg).to(device)
        self._ones = torch.ones(max(B * S * cfg.n_nodes, 1), device=device)
        f = cfg.num_feature
        self.sg_layers = []
        for i, hid in enumerate(cfg.sg_conv_hidden):
            self.sg_layers.append(SpatialGraphConvolution(f, hid, self.w(f"g_sg{i}_conv")))
            f = hid[2]

    # ---- parameters
    def w(self, k):
        o = self.offsets[k]
        return self.params[o:o + int(np.prod(self.shapes[k]))].view(self.shapes[k])

    def g(self, k):
        o = self.offsets[k]
        return self.grads[o:o + int(np.prod(self.shapes[k]))].view(self.shapes[k])

    def load_blocks(self, blocks):
        flat = np.zeros(self.param_count, np.float32)
        for k, shp in self.shapes.items():
            o = self.offsets[k]
            flat[o:o + int(np.prod(shp))] = np.asarray(blocks[k], np.float32).reshape(-1)
        self.params.copy_(torch.from_numpy(flat))

    def blocks(self):
        flat = self.params.double().cpu().numpy()
        return {k: flat[self.offsets[k]:self.offsets[k] + int(np.prod(s))].reshape(s) for k, s in self.shapes.items()}

    def grad_blocks(self):
        flat = self.grads.double().cpu().numpy()
        return {k: flat[self.offsets[k]:self.offsets[k] + int(np.prod(s))].reshape(s) for k, s in self.shapes.items()}

    def _colsum(self, dy, rows, cols, out, ld=None):
        """out[cols] = sum over rows of dy (a 1 x rows by rows x cols GEMM: bias gradients)."""
        _gemm(self._ones, dy, out, 1, cols, rows, ta=True, lda=1, ldb=ld if ld is not None else cols)

    # ---- one training step
    def step(self, batch: "DeviceDisentBatch", eps: Dict[str, torch.Tensor]) -> Dict[str, float]:
        """Forward, hand-chained backward and the TF1-Adam update of one batch
        (main.py:331); eps: {'s': [B, Ls], 'g': [B, Lg], 'sg': [B*S, Lsg]} normals."""
        cfg, B = self.cfg, self.B
        N, F, nh, S = cfg.n_nodes, cfg.num_feature, cfg.node_h, cfg.sampling_num
        R, RS = B * N, B * S * N
        dev = self.device
        T = lambda *shape: torch.empty(*shape, device=dev)
        self.grads.zero_()
        # ================================ encoders ================================
        # graph encoder (model.py:104-115)
        x = batch.x
        gl = []
        hin, fin = x, F
        for i, h in enumerate(cfg.g_conv_hidden):
            last = i + 1 == len(cfg.g_conv_hidden)
            res = graph_convolution(batch.rowptr, batch.colidx, hin, self.w(f"g_g{i}_conv/w"),
                                    self.w(f"g_bn_g{i}/gamma"), self.w(f"g_bn_g{i}/beta"), concat_x=x,
                                    enc_gamma=self.w("encoder_g/gamma") if last else None,
                                    enc_beta=self.w("encoder_g/beta") if last else None)
            gl.append((hin, fin) + tuple(res))
            hin, fin = res[0], h + F
        G = gl[-1][4]                                                 # BN encoder_g output [R, W]
        Wg = fin
        heads = {}

        def head(name, feat, rows, K, hidden, lat):
            hh = T(rows, hidden)
            _gemm(feat, self.w(f"{name}1_lin/Matrix"), hh, rows, hidden, K, bias=self.w(f"{name}1_lin/bias"))
            ms = T(rows, 2 * lat)
            _gemm(hh, self.w(f"{name}23_lin/Matrix"), ms, rows, 2 * lat, hidden, bias=self.w(f"{name}23_lin/bias"))
            heads[name] = (feat, rows, K, hidden, lat, hh, ms)
            return ms
        ms_g = head("g_g", G, B, N * Wg, cfg.g_hidden, cfg.g_latent)
        # spatial encoder (model.py:119-129)
        sl = []
        hs, cin = batch.spatial, cfg.spatial_dim
        for i, co in enumerate(cfg.s_channel):
            y = T(R, co)
            _conv(hs, cin, R, N, cin, self.w(f"g_s{i + 1}_conv/kernel"), co, self.w(f"g_s{i + 1}_conv/bias"), y)
            u = T(R, co)
            _bn_act(y, co, R, co, self.w(f"g_bn_s{i}/gamma"), self.w(f"g_bn_s{i}/beta"), RELU, False, u, co)
            sl.append((hs, cin, y, u))
            hs, cin = u, co
        Vs = T(R, cin)
        _bn_act(hs, cin, R, cin, self.w("encoder_s/gamma"), self.w("encoder_s/beta"), IDENT, False, Vs, cin)
        Ws = cin
        ms_s = head("g_s", Vs, B, N * Ws, cfg.s_hidden, cfg.s_latent)
        # spatial-graph encoder (model.py:134-151) over the B*S copies
        sg_in = batch.x_sg
        for layer in self.sg_layers:
            sg_in, _ = layer.forward(batch.sg_graph, sg_in)
        Wsg = cfg.sg_conv_hidden[-1][2]
        sg_out = sg_in
        Vsg = T(RS, Wsg)
        _bn_act(sg_out, Wsg, RS, Wsg, self.w("encoder_sg/gamma"), self.w("encoder_sg/beta"), IDENT, False, Vsg, Wsg)
        ms_sg = head("g_sg", Vsg, B * S, N * Wsg, cfg.sg_hidden, cfg.sg_latent)
        # get_z (model.py:153-161)
        z = {}
        for name, ms, rows, lat in (("s", ms_s, B, cfg.s_latent), ("g", ms_g, B, cfg.g_latent),
                                    ("sg", ms_sg, B * S, cfg.sg_latent)):
            zz = T(rows, lat)
            kl = torch.zeros(max(1, _lib.lib().snd_reparam_kl_blocks(rows, lat)), dtype=torch.float64, device=dev)
            _lib.check(_lib.lib().snd_reparam_kl(_P(ms), 2 * lat, rows, lat, _P(eps[name]), 0, None, None, _P(zz),
                                                 _P(kl), _lib.stream_ptr()), "snd_reparam_kl")
            z[name] = zz
        # ================================ decoder =================================
        zbar = T(B, cfg.sg_latent)
        _gemm(self._avg, z["sg"], zbar, B, cfg.sg_latent, B * S)
        Jsg_g, Jsg_s = T(R, 2 * nh), T(R, 2 * nh)                     # [J_sg | J_g], [J_sg | J_s]
        J = {}
        for name, zz, lat in (("sg", zbar, cfg.sg_latent), ("s", z["s"], cfg.s_latent), ("g", z["g"], cfg.g_latent)):
            j = T(B, N * nh)
            _gemm(zz, self.w(f"d_{name}_lin1/Matrix"), j, B, N * nh, lat, bias=self.w(f"d_{name}_lin1/bias"))
            J[name] = j.view(R, nh)
        Jsg_g[:, :nh].copy_(J["sg"]); Jsg_g[:, nh:].copy_(J["g"])
        Jsg_s[:, :nh].copy_(J["sg"]); Jsg_s[:, nh:].copy_(J["s"])

        def conv_bn_chain(inp, prefix, bnp, chans, key):
            out, cin = [], 2 * nh
            h = inp
            for i, co in enumerate(chans):
                y = T(R, co)
                _conv(h, cin, R, N, cin, self.w(f"{prefix}{i + key}_deconv/kernel"), co,
                      self.w(f"{prefix}{i + key}_deconv/bias"), y)
                u = T(R, co)
                _bn_act(y, co, R, co, self.w(f"{bnp}{i}/gamma"), self.w(f"{bnp}{i}/beta"), IDENT, False, u, co)
                out.append((h, cin, y, u))
                h, cin = u, co
            return out, h, cin

        def sigmoid_head(u, cin, wname, target, cout):
            ws_n = _lib.lib().snd_sigmoid_mse_blocks(R)
            sse = torch.zeros(ws_n, dtype=torch.float64, device=dev)
            yhat, du = T(R, cout), T(R, cin)
            ws = torch.empty(ws_n * (cin * cout + cout), device=dev)
            _lib.check(_lib.lib().snd_sigmoid_mse(_P(u), cin, R, cin, _P(self.w(wname + "/Matrix")),
                                                  _P(self.w(wname + "/bias")), cout, _P(target), cout, _P(sse),
                                                  _P(yhat), _P(du), cin, _P(self.g(wname + "/Matrix")),
                                                  _P(self.g(wname + "/bias")), _P(ws), ws.numel() * 4,
                                                  _lib.stream_ptr()), "snd_sigmoid_mse")
            return float(sse.sum().item()) / (R * cout), du
        # node decoder (model.py:186-191): conv + BN (no activation) x2, BN decoder_node, sigmoid head
        nlay, nu, nc = conv_bn_chain(Jsg_g, "n", "d_bn_n", cfg.n_d_channel, 0)
        Vn = T(R, nc)
        _bn_act(nu, nc, R, nc, self.w("decoder_node/gamma"), self.w("decoder_node/beta"), IDENT, False, Vn, nc)
        node_cost, dVn = sigmoid_head(Vn, nc, "d_n_lin2", batch.x, F)
        # structure decoder (model.py:193-208) with its CE (optimizer.py:142-144)
        layers = [{"gamma": self.w(f"d_bn_e{i}/gamma"), "beta": self.w(f"d_bn_e{i}/beta"),
                   "w": self.w(f"e{i}_deconv/w1"), "b": self.w(f"e{i}_deconv/biases1")}
                  for i in range(len(cfg.e_d_hidden))]
        hd = {"gamma": self.w("decoder_adj/gamma"), "beta": self.w("decoder_adj/beta"),
              "w": self.w("d_e_lin2/Matrix"), "b": self.w("d_e_lin2/bias")}
        adj_cost, correct, dz_e, eg, hg = structure_decoder(Jsg_g.view(B, N, 2 * nh), batch.adj_dense, layers, hd)
        for i, gi in enumerate(eg):
            self.g(f"d_bn_e{i}/gamma").copy_(gi["gamma"]); self.g(f"d_bn_e{i}/beta").copy_(gi["beta"])
            self.g(f"e{i}_deconv/w1").copy_(gi["w"]); self.g(f"e{i}_deconv/biases1").copy_(gi["b"])
        self.g("decoder_adj/gamma").copy_(hg["gamma"]); self.g("decoder_adj/beta").copy_(hg["beta"])
        self.g("d_e_lin2/Matrix").copy_(hg["w"]); self.g("d_e_lin2/bias").copy_(hg["b"])
        # spatial decoder (model.py:212-219): conv + BN x3 on [J_sg | J_s], sigmoid head
        slay, su, sc = conv_bn_chain(Jsg_s, "s", "d_bn_s", cfg.s_d_channel, 1)
        spatial_cost, dsu = sigmoid_head(su, sc, "d_s_lin2", batch.spatial, cfg.spatial_dim)
        # latent regularisers and the cost (optimizer.py:159-203)
        cap = cfg.capacity
        groups = {"s": (ms_s[:, :cfg.s_latent].contiguous(), ms_s[:, cfg.s_latent:].contiguous(), z["s"]),
                  "g": (ms_g[:, :cfg.g_latent].contiguous(), ms_g[:, cfg.g_latent:].contiguous(), z["g"]),
                  "sg": (ms_sg[:, :cfg.sg_latent].contiguous(), ms_sg[:, cfg.sg_latent:].contiguous(), z["sg"])}
        mse = {"adj_cost": adj_cost, "node_cost": node_cost, "spatial_cost": spatial_cost}
        overall, reg_grads = disentangled_cost(cfg.model_type, groups, mse, cfg.beta, cfg.gamma, cap)
        # ================================ backward ================================
        def conv_bn_chain_bwd(lays, du, prefix, bnp, key):
            d = du
            for i in range(len(lays) - 1, -1, -1):
                h, cin, y, u = lays[i]
                co = y.shape[1]
                dy = T(R, co)
                _bn_act_bwd(d, co, y, co, R, co, self.w(f"{bnp}{i}/gamma"), self.w(f"{bnp}{i}/beta"), IDENT, False,
                            dy, co, self.g(f"{bnp}{i}/gamma"), self.g(f"{bnp}{i}/beta"))
                dx, dw = conv1d_same_bwd(h, self.w(f"{prefix}{i + key}_deconv/kernel"), dy, N)
                self.g(f"{prefix}{i + key}_deconv/kernel").copy_(dw)
                self._colsum(dy, R, co, self.g(f"{prefix}{i + key}_deconv/bias"))
                d = dx
            return d
        dn = T(R, nc)
        _bn_act_bwd(dVn, nc, nu, nc, R, nc, self.w("decoder_node/gamma"), self.w("decoder_node/beta"), IDENT, False,
                    dn, nc, self.g("decoder_node/gamma"), self.g("decoder_node/beta"))
        dJsg_g = conv_bn_chain_bwd(nlay, dn, "n", "d_bn_n", 0)                   # [R, 2 nh]
        _add(dz_e.view(R, 2 * nh), 2 * nh, dJsg_g, 2 * nh, R, 2 * nh)
        dJsg_s = conv_bn_chain_bwd(slay, dsu, "s", "d_bn_s", 1)
        dJ = {"sg": T(R, nh), "g": T(R, nh), "s": T(R, nh)}
        dJ["sg"].copy_(dJsg_g[:, :nh]); dJ["g"].copy_(dJsg_g[:, nh:]); dJ["s"].copy_(dJsg_s[:, nh:])
        _add(dJsg_s, 2 * nh, dJ["sg"], nh, R, nh)
        # projections (d_*_lin1) and the mean over the copies
        dz = {}
        for name, zz, lat in (("sg", zbar, cfg.sg_latent), ("s", z["s"], cfg.s_latent), ("g", z["g"], cfg.g_latent)):
            dflat = dJ[name].view(B, N * nh)
            _gemm(zz, dflat, self.g(f"d_{name}_lin1/Matrix"), lat, N * nh, B, ta=True)
            self._colsum(dflat, B, N * nh, self.g(f"d_{name}_lin1/bias"))
            d = T(B, lat)
            _gemm(dflat, self.w(f"d_{name}_lin1/Matrix"), d, B, lat, N * nh, tb=True)
            dz[name] = d
        dzsg = T(B * S, cfg.sg_latent)
        _gemm(self._avg, dz["sg"], dzsg, B * S, cfg.sg_latent, B, ta=True)
        dz["sg"] = dzsg
        # reparameterisation (reconstruction path + the regulariser gradients) and the heads
        dfeat = {}
        for name, key, lat in (("s", "g_s", cfg.s_latent), ("g", "g_g", cfg.g_latent), ("sg", "g_sg", cfg.sg_latent)):
            feat, rows, K, hidden, _, hh, ms = heads[key]
            dms = T(rows, 2 * lat)
            dmu_r, ds_r = reg_grads.get(name, (None, None))
            _lib.check(_lib.lib().snd_reparam_bwd(_P(ms), 2 * lat, rows, lat, _P(eps[name]), _P(dz[name]), _P(dmu_r),
                                                  _P(ds_r), _P(dms), 2 * lat, _lib.stream_ptr()), "snd_reparam_bwd")
            _gemm(hh, dms, self.g(f"{key}23_lin/Matrix"), hidden, 2 * lat, rows, ta=True)
            self._colsum(dms, rows, 2 * lat, self.g(f"{key}23_lin/bias"))
            dh = T(rows, hidden)
            _gemm(dms, self.w(f"{key}23_lin/Matrix"), dh, rows, hidden, 2 * lat, tb=True)
            _gemm(feat.view(rows, K), dh, self.g(f"{key}1_lin/Matrix"), K, hidden, rows, ta=True)
            self._colsum(dh, rows, hidden, self.g(f"{key}1_lin/bias"))
            df = T(rows, K)
            _gemm(dh, self.w(f"{key}1_lin/Matrix"), df, rows, K, hidden, tb=True)
            dfeat[name] = df
        # spatial-graph encoder backward
        dsg = T(RS, Wsg)
        _bn_act_bwd(dfeat["sg"].view(RS, Wsg), Wsg, sg_out, Wsg, RS, Wsg, self.w("encoder_sg/gamma"),
                    self.w("encoder_sg/beta"), IDENT, False, dsg, Wsg, self.g("encoder_sg/gamma"),
                    self.g("encoder_sg/beta"))
        d = dsg
        for i in range(len(self.sg_layers) - 1, -1, -1):
            gr, d = self.sg_layers[i].backward(d, want_dx=i > 0)
            self.g(f"g_sg{i}_conv").copy_(gr)
        # spatial encoder backward
        d = T(R, Ws)
        _bn_act_bwd(dfeat["s"].view(R, Ws), Ws, sl[-1][3], Ws, R, Ws, self.w("encoder_s/gamma"),
                    self.w("encoder_s/beta"), IDENT, False, d, Ws, self.g("encoder_s/gamma"), self.g("encoder_s/beta"))
        for i in range(len(sl) - 1, -1, -1):
            hs_i, cin, y, u = sl[i]
            co = y.shape[1]
            dy = T(R, co)
            _bn_act_bwd(d, co, y, co, R, co, self.w(f"g_bn_s{i}/gamma"), self.w(f"g_bn_s{i}/beta"), RELU, False,
                        dy, co, self.g(f"g_bn_s{i}/gamma"), self.g(f"g_bn_s{i}/beta"))
            dx, dw = conv1d_same_bwd(hs_i, self.w(f"g_s{i + 1}_conv/kernel"), dy, N)
            self.g(f"g_s{i + 1}_conv/kernel").copy_(dw)
            self._colsum(dy, R, co, self.g(f"g_s{i + 1}_conv/bias"))
            d = dx
        # graph encoder backward (G = BN_enc(H2), H2 = [BN_1(lrelu(P1)) | x], ...)
        dH = T(R, Wg)
        Hn = gl[-1][2]
        _bn_act_bwd(dfeat["g"].view(R, Wg), Wg, Hn, Wg, R, Wg, self.w("encoder_g/gamma"), self.w("encoder_g/beta"),
                    IDENT, False, dH, Wg, self.g("encoder_g/gamma"), self.g("encoder_g/beta"))
        for i in range(len(gl) - 1, -1, -1):
            hin_i, fin_i, Pi = gl[i][0], gl[i][1], gl[i][3]
            h = Pi.shape[1]
            dP = T(R, h)
            _bn_act_bwd(dH, dH.shape[1], Pi, h, R, h, self.w(f"g_bn_g{i}/gamma"), self.w(f"g_bn_g{i}/beta"), LRELU,
                        True, dP, h, self.g(f"g_bn_g{i}/gamma"), self.g(f"g_bn_g{i}/beta"))
            dXW = spmm(batch.rowptr, batch.colidx, dP)                          # A symmetric: A^T = A
            _gemm(hin_i, dXW, self.g(f"g_g{i}_conv/w"), fin_i, h, R, ta=True)
            if i > 0:
                dH = T(R, fin_i)
                _gemm(dXW, self.w(f"g_g{i}_conv/w"), dH, R, fin_i, h, tb=True)
        # TF1 Adam (optimizer.py:125,197); the step counter is the TF global step
        self.step_counter += 1
        _lib.check(_lib.lib().snd_adam_tf1(_P(self.params), _P(self.grads), _P(self.m), _P(self.v),
                                           self.param_count, cfg.learning_rate, cfg.adam_beta1, cfg.adam_beta2,
                                           cfg.adam_eps, 1.0, _P(self.step_counter), _lib.stream_ptr()),
                   "snd_adam_tf1")
        names = ("cost", "spatial_cost", "adj_cost", "node_cost") + \
            (("kl_g", "kl_s", "kl_sg") if len(overall) == 7 else ("kl_sg",))   # overall_loss order
        out = dict(zip(names, overall))
        out["correct"] = correct
        return out


class DeviceDisentBatch:
    """An SGBatch on the device for the disentangled model: adj_truth (CSR and dense for
    the e2e CE), node features and coordinates per graph, the copies' features, trees
    and rel (the feeds of main.py:253-264)."""

    def __init__(self, batch: SGBatch, device="cuda"):
        t = lambda a, dt=torch.float32: torch.from_numpy(np.ascontiguousarray(a)).to(device=device, dtype=dt)
        B, N = batch.n_graphs, batch.n_nodes
        self.rowptr = t(batch.rowptr, torch.int32)
        self.colidx = t(batch.colidx if batch.nnz else np.zeros(1, np.int32), torch.int32)
        self.x = t(batch.feature_truth)
        self.spatial = t(batch.spatial_truth)
        self.adj_dense = t(np.stack([batch.dense_adj(b) for b in range(B)]))
        self.x_sg = t(batch.features)
        self.rel = t(batch.rel)
        self.sg_graph = SGGraph(batch.tree_rowptr, batch.tree_colidx, N, self.rel)
