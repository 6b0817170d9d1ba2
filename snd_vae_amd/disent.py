"""Disentangled-model pieces over torch device tensors.

* ``e2e`` / ``e2e_bwd``: the structure decoder's edge-to-edge filter
  (`layers.py:431-450`; applied with k_h = N at `model.py:196`), fp32.
* ``latent_reg``: one latent group's regulariser (KL, the 'disentangled_C'
  capacity form, DIP, total correlation; `optimizer.py:7-58,159-190`) with its
  gradients, one launch.
* ``OptimizerDisentangled``-style combination ``disentangled_cost``: the
  model_type branches of `optimizer.py:159-203` over the groups (s, g, sg),
  returning ``overall_loss`` in the reference order and the per-group
  gradients.

The reference creates TF variables; these take the weights explicitly.  Every
call runs HIP kernels of libsndvae.so on the current stream (no CPU path).
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, Optional, Tuple

import torch

from . import _lib

_P = _lib.ptr

MODEL_TYPES = ("base", "disentangled", "disentangled_C", "NED-VAE-IP", "beta-TCVAE", "geoGCN", "posGCN")


def _f32(t, name):
    if not (t.is_cuda and t.is_contiguous() and t.dtype == torch.float32):
        raise ValueError(f"{name}: expected a contiguous float32 device tensor")
    return t


def e2e(x, w1, b1):
    """e2e(input_, output_dim, k_h) of `layers.py:431-450`: x [B, N, N, C], w1 [K, C, O]
    (the [1, K, C, O] kernel), b1 [O] -> [B, N, N, O]."""
    for t, n in ((x, "x"), (w1, "w1"), (b1, "b1")):
        _f32(t, f"e2e {n}")
    B, N, N2, Cc = x.shape
    K, Cw, O = w1.shape
    if N2 != N or Cw != Cc or b1.numel() != O:
        raise ValueError("e2e: shapes x [B,N,N,C], w1 [K,C,O], b1 [O]")
    out = torch.empty(B, N, N, O, device=x.device, dtype=torch.float32)
    _lib.check(_lib.lib().snd_e2e_fwd(_P(x), B, N, Cc, _P(w1), _P(b1), K, O, _P(out), _lib.stream_ptr()),
               "snd_e2e_fwd")
    return out


def e2e_bwd(x, w1, dout):
    """(dx, dw1, db1) of sum(e2e(x, w1, b1) * dout)."""
    for t, n in ((x, "x"), (w1, "w1"), (dout, "dout")):
        _f32(t, f"e2e_bwd {n}")
    B, N, _, Cc = x.shape
    K, _, O = w1.shape
    dx = torch.empty_like(x)
    dw1 = torch.empty_like(w1)
    db1 = torch.empty(O, device=x.device, dtype=torch.float32)
    _lib.check(_lib.lib().snd_e2e_bwd(_P(x), B, N, Cc, _P(w1), K, O, _P(dout), _P(dx), _P(dw1), _P(db1),
                                      _lib.stream_ptr()), "snd_e2e_bwd")
    return dx, dw1, db1


def latent_reg(mu, logstd, z=None, w_kl=1.0, cap_gamma=0.0, cap_c=0.0, w_dip=0.0, lambda_od=10.0,
               lambda_d=100.0, w_tc=0.0) -> Tuple[Dict[str, float], torch.Tensor, torch.Tensor]:
    """One group's term w_kl kl (or cap_gamma relu(kl - cap_c)) + w_dip DIP(mu) + w_tc TC(z);
    returns ({kl, term, dip, tc}, d term / d mu, d term / d logstd) -- the gradients include
    the path through z = mu + eps e^logstd (model.py:155-159)."""
    _f32(mu, "latent_reg mu")
    _f32(logstd, "latent_reg logstd")
    if z is not None:
        _f32(z, "latent_reg z")
    if w_tc and z is None:
        raise ValueError("latent_reg: the total-correlation term needs the sample z")
    B, L = mu.shape
    L_ = _lib.lib()
    w = _lib.LatentReg(w_kl, cap_gamma, cap_c, w_dip, lambda_od, lambda_d, w_tc)
    ws = None
    if w_dip or w_tc:
        ws = torch.empty(int(L_.snd_latent_reg_workspace(B, L)) // 4 + 1, device=mu.device, dtype=torch.float32)
    dmu, ds = torch.empty_like(mu), torch.empty_like(logstd)
    out = torch.empty(4, device=mu.device, dtype=torch.float64)
    _lib.check(L_.snd_latent_reg(_P(mu), _P(logstd), _P(z) if z is not None else None, B, L, C.byref(w),
                                 _P(dmu), _P(ds), _P(out), _P(ws) if ws is not None else None,
                                 _lib.stream_ptr()), "snd_latent_reg")
    v = out.cpu().tolist()
    return {"kl": v[0], "term": v[1], "dip": v[2], "tc": v[3]}, dmu, ds


def capacity(global_iter: int, c_max: float, c_step: int, c_stop_iter: int) -> float:
    """C of 'disentangled_C' (`optimizer.py:167`)."""
    return min(max(c_max * c_step / c_stop_iter * (global_iter // c_step), 0.0), c_max)


def group_weights(model_type: str, beta: float = 1.0, gamma: float = 1.0, c: float = 0.0):
    """Per-group regulariser weights of `optimizer.py:159-190` for the groups s, g, sg."""
    if model_type not in MODEL_TYPES:
        raise ValueError(f"unknown model_type {model_type!r} (main.py:72)")
    if model_type in ("disentangled", "geoGCN", "posGCN"):
        return {"s": {"w_kl": beta}, "g": {"w_kl": beta}, "sg": {"w_kl": beta}}
    if model_type == "disentangled_C":
        return {"s": {"w_kl": 1.0}, "g": {"w_kl": 1.0}, "sg": {"w_kl": 0.0, "cap_gamma": gamma, "cap_c": c}}
    if model_type == "NED-VAE-IP":
        return {k: {"w_kl": 1.0, "w_dip": beta, "lambda_od": 10.0, "lambda_d": 100.0} for k in ("s", "g", "sg")}
    if model_type == "beta-TCVAE":
        return {k: {"w_kl": beta, "w_tc": 10.0} for k in ("s", "g", "sg")}
    return {"sg": {"w_kl": beta}}


def disentangled_cost(model_type: str, groups: Dict[str, tuple], mse: Dict[str, float], beta: float = 1.0,
                      gamma: float = 1.0, c: float = 0.0):
    """The cost of `optimizer.py:146-203` given the reconstruction terms
    mse = {spatial_cost, adj_cost, node_cost} and groups = {'s' | 'g' | 'sg': (mu, logstd, z)}.
    Returns (overall_loss list in the reference order, {group: (dmu, dlogstd)})."""
    weights = group_weights(model_type, beta, gamma, c)
    reg, grads, kls = 0.0, {}, {}
    for name, w in weights.items():
        mu, s, z = groups[name]
        v, dmu, ds = latent_reg(mu, s, z, **w)
        reg += v["term"]
        kls[name] = v["kl"]
        grads[name] = (dmu, ds)
    cost = mse["adj_cost"] + mse["node_cost"] + mse["spatial_cost"] + reg
    if model_type == "base":
        return [cost, mse["spatial_cost"], mse["adj_cost"], mse["node_cost"], kls["sg"]], grads
    return [cost, mse["spatial_cost"], mse["adj_cost"], mse["node_cost"], kls["g"], kls["s"], kls["sg"]], grads


def _bn_relu(y, g, b):
    rows, c = y.numel() // y.shape[-1], y.shape[-1]
    x = torch.empty_like(y)
    _lib.check(_lib.lib().snd_bn_relu_fwd(_P(y), rows, c, _P(g), _P(b), _P(x), _lib.stream_ptr()), "snd_bn_relu_fwd")
    return x


def structure_decoder(z, adj, layers, head):
    """The e2e structure decoder of `model.py:193-208` with the CE of `optimizer.py:142-144`,
    forward and backward in one call.

    z [B, N, D] (z_sg_g), adj [B, N, N] 0/1 (adj_truth); layers: per e2e layer i a dict
    {gamma, beta (d_bn_e[i], over its input channels), w [N, Cin, Cout], b [Cout]};
    head: {gamma, beta (decoder_adj), w [Cin, 2], b [2]} (d_e_lin2).  Returns
    (adj_cost = mean CE over B N^2, correct = #(argmax == A) (main.py:334), dz,
    grads: a list of per-layer dicts and the head dict, same keys as the inputs)."""
    B, N, D = z.shape
    _f32(z, "structure_decoder z")
    _f32(adj, "structure_decoder adj")
    L_ = _lib.lib()
    sp = _lib.stream_ptr()
    # forward: x0 = relu(BN0(pair(z))), y_{i+1} = e2e(x_i), x_i = relu(BN_i(y_i))
    x = torch.empty(B, N, N, 2 * D, device=z.device, dtype=torch.float32)
    l0 = layers[0]
    _lib.check(L_.snd_e2e_pair_fwd(_P(z), B, N, D, _P(l0["gamma"]), _P(l0["beta"]), _P(x), sp), "snd_e2e_pair_fwd")
    xs, ys = [x], []
    for i, lay in enumerate(layers):
        y = e2e(xs[-1], lay["w"], lay["b"])
        ys.append(y)
        if i + 1 < len(layers):
            nxt = layers[i + 1]
            xs.append(_bn_relu(y, nxt["gamma"], nxt["beta"]))
    yl = ys[-1]
    c = yl.shape[-1]
    dy = torch.empty_like(yl)
    hg = {k: torch.empty_like(v) for k, v in head.items()}
    out = torch.empty(2, device=z.device, dtype=torch.float64)
    _lib.check(L_.snd_e2e_head_ce(_P(yl), _P(adj), B, N, c, _P(head["gamma"]), _P(head["beta"]), _P(head["w"]),
                                  _P(head["b"]), _P(dy), _P(hg["w"]), _P(hg["b"]), _P(hg["gamma"]), _P(hg["beta"]),
                                  _P(out), sp), "snd_e2e_head_ce")
    # backward
    grads = [dict() for _ in layers]
    for i in range(len(layers) - 1, -1, -1):
        dx, grads[i]["w"], grads[i]["b"] = e2e_bwd(xs[i], layers[i]["w"], dy)
        if i > 0:
            lay = layers[i]
            dy = torch.empty_like(ys[i - 1])
            grads[i]["gamma"] = torch.empty_like(lay["gamma"])
            grads[i]["beta"] = torch.empty_like(lay["beta"])
            rows, cc = ys[i - 1].numel() // ys[i - 1].shape[-1], ys[i - 1].shape[-1]
            _lib.check(L_.snd_bn_relu_bwd(_P(dx), _P(ys[i - 1]), rows, cc, _P(lay["gamma"]), _P(lay["beta"]), _P(dy),
                                          _P(grads[i]["gamma"]), _P(grads[i]["beta"]), sp), "snd_bn_relu_bwd")
        else:
            dz = torch.empty_like(z)
            grads[0]["gamma"] = torch.empty_like(l0["gamma"])
            grads[0]["beta"] = torch.empty_like(l0["beta"])
            ws = torch.empty(int(L_.snd_e2e_pair_bwd_workspace(B, N, D)) // 4 + 1, device=z.device,
                             dtype=torch.float32)
            _lib.check(L_.snd_e2e_pair_bwd(_P(dx), _P(z), B, N, D, _P(l0["gamma"]), _P(l0["beta"]), _P(dz),
                                           _P(grads[0]["gamma"]), _P(grads[0]["beta"]), _P(ws), sp),
                       "snd_e2e_pair_bwd")
    o = out.cpu().tolist()
    return o[0] / (B * N * N), o[1], dz, grads, hg
