"""ORACLE -- test infrastructure only.  Never imported by the product path.

Literal float64 restatement of ``SpatialGraphConvolution`` (`layers.py:143-198`)
and of the model_joint spatial-graph encoder (`model_joint.py:72-85`), written
with the reference's own dense B x N x N x N tensors (small N only), in numpy
for the forward pass and in torch-CPU autograd (float64) for gradients.

Parity status: TensorFlow is unavailable and the reference ships no fixtures,
so this is parity unpinned against TF itself; it is pinned by its line-by-line
correspondence, finite differences (tests/test_sg_oracle.py) and agreement of
the numpy and torch formulations.

layers.py:143-198 (rel_dim r = 1; Matrix1 has 3F + 2r + 1 rows):
    rel_ij[b,i,j,k] = rel[b,i,j]   rel_jk[...] = rel[b,j,k]   dis_ik[...] = rel[b,i,k]
    adj_3d[b,i,j,k] = adj[b,i,j] * adj[b,j,k]
    m3 = lrelu([x_i, x_j, x_k, rel_ij, rel_jk, dis_ik]) @ Matrix1 + bias1
    m3_sum[b,i,j] = sum_k m3[b,i,j,k] * adj_3d[b,i,j,k]
    m2 = lrelu([x_i, x_j, rel_ij, m3_sum]) @ Matrix2 + bias2
    m2_sum[b,i] = sum_j m2[b,i,j] * adj[b,i,j]
    out = lrelu([x, m2_sum]) @ Matrix3 + bias3
model_joint.py:77-85: s_g = lrelu(BN(SGConv(adj, s_g, rel))) per layer (dropout keep 1),
    then g_sg1_lin / g_sg2_lin / g_sg3_lin on the row-major flat s_g.
"""
from __future__ import annotations

import numpy as np

BN_C = 1.0 / np.sqrt(1.0 + 1e-3)
LEAK = 0.2


def lrelu(x):
    return np.maximum(x, LEAK * x)


def sgconv(adj, x, rel, p):
    """adj [B,N,N], x [B,N,F], rel [B,N,N] (rel_dim 1), p: M1,b1,M2,b2,M3,b3."""
    adj, x, rel = (np.asarray(a, np.float64) for a in (adj, x, rel))
    B, N, F = x.shape
    xi = np.broadcast_to(x[:, :, None, None, :], (B, N, N, N, F))
    xj = np.broadcast_to(x[:, None, :, None, :], (B, N, N, N, F))
    xk = np.broadcast_to(x[:, None, None, :, :], (B, N, N, N, F))
    rij = np.broadcast_to(rel[:, :, :, None, None], (B, N, N, N, 1))
    rjk = np.broadcast_to(rel[:, None, :, :, None], (B, N, N, N, 1))
    dik = np.broadcast_to(rel[:, :, None, :, None], (B, N, N, N, 1))
    adj3 = adj[:, :, :, None] * adj[:, None, :, :]
    m3 = np.concatenate([xi, xj, xk, rij, rjk, dik], -1)
    m3 = lrelu(m3) @ p["M1"] + p["b1"]                         # [B,N,N,N,h0]
    m3_sum = np.einsum("bijkh,bijk->bijh", m3, adj3)
    m2 = np.concatenate([x[:, :, None, :].repeat(N, 2), x[:, None, :, :].repeat(N, 1),
                         rel[..., None], m3_sum], -1)
    m2 = lrelu(m2) @ p["M2"] + p["b2"]                         # [B,N,N,h1]
    m2_sum = np.einsum("bijh,bij->bih", m2, adj)
    m1 = np.concatenate([x, m2_sum], -1)
    return lrelu(m1) @ p["M3"] + p["b3"]


def sg_encoder(adj, x, rel, layers, heads=None):
    """model_joint.py:77-85: per layer s_g = lrelu(BN(SGConv)); returns s_g (and the
    heads' [mu || s] when heads = (Wh, bh, Wms, bms) is given)."""
    s = np.asarray(x, np.float64)
    for p in layers:
        y = sgconv(adj, s, rel, p)
        s = lrelu(y * (p["gamma"] * BN_C) + p["beta"])
    if heads is None:
        return s
    Wh, bh, Wms, bms = heads
    h = s.reshape(s.shape[0], -1) @ Wh + bh
    return s, h @ Wms + bms


# --------------------------------------------------------------------------- torch autograd
def sgconv_torch(adj, x, rel, p):
    """Same graph in torch ops (autograd stands in for TF autodiff)."""
    import torch
    lr = lambda t: torch.maximum(t, LEAK * t)
    B, N, F = x.shape
    xi = x[:, :, None, None, :].expand(B, N, N, N, F)
    xj = x[:, None, :, None, :].expand(B, N, N, N, F)
    xk = x[:, None, None, :, :].expand(B, N, N, N, F)
    rij = rel[:, :, :, None, None].expand(B, N, N, N, 1)
    rjk = rel[:, None, :, :, None].expand(B, N, N, N, 1)
    dik = rel[:, :, None, :, None].expand(B, N, N, N, 1)
    adj3 = adj[:, :, :, None] * adj[:, None, :, :]
    m3 = lr(torch.cat([xi, xj, xk, rij, rjk, dik], -1)) @ p["M1"] + p["b1"]
    m3_sum = torch.einsum("bijkh,bijk->bijh", m3, adj3)
    m2 = torch.cat([x[:, :, None, :].expand(B, N, N, F), x[:, None, :, :].expand(B, N, N, F),
                    rel[..., None], m3_sum], -1)
    m2 = lr(m2) @ p["M2"] + p["b2"]
    m2_sum = torch.einsum("bijh,bij->bih", m2, adj)
    return lr(torch.cat([x, m2_sum], -1)) @ p["M3"] + p["b3"]


def sgconv_grads(adj, x, rel, p, dout):
    """Gradients of sum(out * dout) wrt x and every parameter (float64 autograd)."""
    import torch
    t = lambda a, g=False: torch.tensor(np.asarray(a, np.float64), requires_grad=g)
    tp = {k: t(v, True) for k, v in p.items() if k in ("M1", "b1", "M2", "b2", "M3", "b3")}
    tx = t(x, True)
    out = sgconv_torch(t(adj), tx, t(rel), tp)
    (out * t(dout)).sum().backward()
    g = {k: v.grad.numpy() for k, v in tp.items()}
    g["x"] = tx.grad.numpy()
    return out.detach().numpy(), g


def init_sg_layer(F, hidden, rng, stddev=0.02):
    """layers.py:163-174 initialisers: Matrix ~ N(0, stddev), bias = 0; BN gamma 1 beta 0."""
    h0, h1, h2 = hidden
    return {"M1": rng.normal(0, stddev, (3 * F + 3, h0)), "b1": np.zeros(h0),
            "M2": rng.normal(0, stddev, (2 * F + 1 + h0, h1)), "b2": np.zeros(h1),
            "M3": rng.normal(0, stddev, (F + h1, h2)), "b3": np.zeros(h2),
            "gamma": np.ones(h2), "beta": np.zeros(h2)}


# --------------------------------------------------------------------------- the SG-joint model
def unpack_layer(flat, F, hidden):
    """A layer's flat parameter vector (include/snd_vae.h layout: Matrix1, bias1, Matrix2,
    bias2, Matrix3, bias3, BN gamma, BN beta) -> dict of views (numpy or torch)."""
    h0, h1, h2 = hidden
    shapes = [("M1", (3 * F + 3, h0)), ("b1", (h0,)), ("M2", (2 * F + 1 + h0, h1)), ("b2", (h1,)),
              ("M3", (F + h1, h2)), ("b3", (h2,)), ("gamma", (h2,)), ("beta", (h2,))]
    out, o = {}, 0
    for name, shp in shapes:
        n = int(np.prod(shp))
        out[name] = flat[o:o + n].reshape(shp)
        o += n
    assert o == flat.shape[0], (o, flat.shape)
    return out


def sgjoint_loss_torch(p, trees, X, rel, adj, Xf, S, eps, cfg):
    """The SND-VAE spatial-graph model, literally, in float64 torch ops (autograd for
    the gradients):
      model_joint.py:77-80   s_g = lrelu(BN(SGConv(trees, s_g, rel))) per layer, on the
                             B*S spanning-tree copies (copy b*S + s: graph b's tree s,
                             features and rel; main.py:254-262 feeds, aligned per graph)
      model.py:146-151       h = flat(s_g) Wh + bh, [mu | s] per copy; z = mu + eps e^s
      model.py:177,180       J = mean_s reshape(z Wp + bp, [B, S, N, node_h])
      model_joint.py:112-145 decoders; optimizer.py:142-157,192-194 losses (KL over B*S*L)
    p: torch params by block name (enc.sg0 / enc.sg1 flat); trees [B*S,N,N];
    X [B*S,N,F]; rel [B*S,N,N]; adj / Xf / S per graph [B,N,.]; eps [B*S, L]."""
    import torch

    from oracle import ref_torch as T
    B, n, _ = adj.shape
    Sn, L = cfg.sampling_num, cfg.latent
    s_g = X
    F = X.shape[-1]
    for i, hid in enumerate(cfg.sg_conv_hidden):
        lp = unpack_layer(p[f"enc.sg{i}"], F, hid)
        y = sgconv_torch(trees, s_g, rel, lp)
        s_g = T.lrelu(T.bn(y, lp["gamma"], lp["beta"]))
        F = hid[2]
    h = torch.reshape(s_g, [B * Sn, -1]) @ p["enc.Wh"] + p["enc.bh"]
    ms = h @ p["enc.Wms"] + p["enc.bms"]
    mu, s = ms[..., :L], ms[..., L:]
    z = mu + eps * torch.exp(s)
    J = torch.reshape(z @ p["dec.Wp"] + p["dec.bp"], [B, Sn, n, cfg.node_h_size]).mean(1)
    return T.decoder_losses(p, J, adj, Xf, S, mu, s, cfg)


def sgjoint_forward_backward(blocks, trees, X, rel, adj, Xf, S, eps, cfg):
    """(losses dict, grads dict by block) of one step, float64."""
    import torch
    p = {k: torch.tensor(np.asarray(v, np.float64), requires_grad=True) for k, v in blocks.items()}
    t = lambda a: torch.tensor(np.asarray(a, np.float64))
    cost, parts = sgjoint_loss_torch(p, t(trees), t(X), t(rel), t(adj), t(Xf), t(S), t(eps), cfg)
    cost.backward()
    losses = {k: float(v.detach()) for k, v in parts.items()}
    return losses, {k: v.grad.numpy() for k, v in p.items()}
