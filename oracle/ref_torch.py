"""ORACLE -- test infrastructure only.  Never imported by the product path.

The reference TF1 graph written out literally in torch-CPU ops, with autograd
standing in for TF autodiff (`optimizer.py:197`).  It keeps the reference's
own (dense, materialising) formulation on purpose:

* ``tf.matmul(adj, X @ w)`` with the dense [B,N,N] adjacency (`layers.py:120-123`)
* logits materialised as [B,N,N,2] with the numpy ``diag`` constant
  (`model.py:185,205-207`), softmax-CE against ``concat([1-A, A])``
  (`optimizer.py:142-144`)
* ``tf.layers.conv1d`` SAME as F.conv1d(padding=2) (`model_joint.py:115,138`)
* TF1 Adam (`optimizer.py:125,197`)

Used two ways: float64, to cross-check the hand-derived backward of
``ref_numpy``; float32 on the host cores, as ``bench.py``'s ``cpu_baseline``
("reference-formula CPU path", kind "port": TensorFlow is unavailable).
"""
from __future__ import annotations

from typing import Dict

import numpy as np
import torch
import torch.nn.functional as F

BN_C = 1.0 / np.sqrt(1.0 + 1e-3)


def lrelu(x):
    return torch.maximum(x, 0.2 * x)


def bn(x, g, b):
    return x * (g * BN_C) + b


def conv1d_same(x, w, b):
    """x [B,N,Cin], w [5,Cin,Cout] (TF layout) -> [B,N,Cout]."""
    y = F.conv1d(x.transpose(1, 2), w.permute(2, 1, 0), b, padding=2)
    return y.transpose(1, 2)


def build_params(blocks: Dict[str, np.ndarray], dtype):
    return {k: torch.tensor(np.asarray(v), dtype=dtype, requires_grad=True)
            for k, v in blocks.items()}


def loss_fn(p, adj, X, Xf, S, eps, cfg):
    """adj [B,N,N]; X [B,N,f]; Xf [B,N,nf]; S [B,N,2]; eps [B,N,L] (tref: [B,L])."""
    B, n, _ = adj.shape
    L = cfg.latent
    s1 = cfg.s_d_channel[0]
    g = X
    for i, (w, bg, bb) in enumerate([("enc.W0", "enc.bn0.gamma", "enc.bn0.beta"),
                                     ("enc.W1", "enc.bn1.gamma", "enc.bn1.beta")]):
        conv = torch.matmul(adj, torch.matmul(g, p[w]))
        g = bn(lrelu(conv), p[bg], p[bb])
        g = torch.cat([g, X], -1)
    g = bn(g, p["enc.bne.gamma"], p["enc.bne.beta"])
    if cfg.topology == "tref":   # model.py:113-115, model_joint.py:87-97
        h = torch.reshape(g, [B, -1]) @ p["enc.Wh"] + p["enc.bh"]
        ms = h @ p["enc.Wms"] + p["enc.bms"]
        mu, s = ms[..., :L], ms[..., L:]
        z = mu + eps.reshape(B, L) * torch.exp(s)
        J = torch.reshape(z @ p["dec.Wp"] + p["dec.bp"], [B, n, cfg.node_h_size])
    else:
        h = g @ p["enc.Wh"] + p["enc.bh"]
        ms = h @ p["enc.Wms"] + p["enc.bms"]
        mu, s = ms[..., :L], ms[..., L:]
        z = mu + eps * torch.exp(s)
        J = z
    return decoder_losses(p, J, adj, Xf, S, mu, s, cfg)


def decoder_losses(p, J, adj, Xf, S, mu, s, cfg):
    """The decoders and the ELBO from J [B,N,node_h] (model_joint.py:112-145,
    model.py:205-208, optimizer.py:142-157,192-194); mu / s: the latent's mean and
    log-std over which the KL mean runs."""
    B, n, _ = adj.shape
    s1 = cfg.s_d_channel[0]
    X = J
    logit = torch.matmul(J, J.transpose(1, 2))
    diag = torch.ones(n, n, dtype=X.dtype) - torch.eye(n, dtype=X.dtype)
    l0 = diag * 0.0 * logit + (1 - diag)                  # model.py:206
    l1 = diag * logit                                      # model.py:205
    logits = torch.stack([l0, l1], -1)
    labels = torch.stack([1 - adj, adj], -1)               # optimizer.py:142
    ce = -(labels * torch.log_softmax(logits, -1)).sum(-1)
    adj_cost = ce.mean()
    generated_adj = torch.argmax(torch.softmax(logits, -1), -1)
    acc = (generated_adj == adj.long()).double().mean()

    u = lrelu(bn(conv1d_same(J, p["dec.K1"], p["dec.b1"]),
                 p["dec.bn1.gamma"], p["dec.bn1.beta"]))
    us, un = u[..., :s1], u[..., s1:]
    us = lrelu(bn(conv1d_same(us, p["dec.K2s"], p["dec.b2s"]),
                  p["dec.bn2s.gamma"], p["dec.bn2s.beta"]))
    us = lrelu(bn(conv1d_same(us, p["dec.K3s"], p["dec.b3s"]),
                  p["dec.bn3s.gamma"], p["dec.bn3s.beta"]))
    shat = torch.sigmoid(us @ p["dec.Ws"] + p["dec.bs"])
    un = lrelu(bn(conv1d_same(un, p["dec.K2n"], p["dec.b2n"]),
                  p["dec.bn2n.gamma"], p["dec.bn2n.beta"]))
    xhat = torch.sigmoid(un @ p["dec.Wn"] + p["dec.bn"])
    node_cost = ((Xf - xhat) ** 2).mean()
    spatial_cost = ((S - shat) ** 2).mean()
    kl = -0.5 * (1 + 2 * s - mu ** 2 - torch.exp(s) ** 2).mean()
    cost = adj_cost + node_cost + spatial_cost + cfg.beta * kl
    return cost, dict(cost=cost, adj_cost=adj_cost, node_cost=node_cost,
                      spatial_cost=spatial_cost, kl=kl, acc=acc)


class TF1Adam:
    """tf.train.AdamOptimizer(lr) semantics (epsilon outside the sqrt-corrected v)."""

    def __init__(self, params, lr, b1=0.9, b2=0.999, eps=1e-8):
        self.p, self.lr, self.b1, self.b2, self.eps = params, lr, b1, b2, eps
        self.m = {k: torch.zeros_like(v) for k, v in params.items()}
        self.v = {k: torch.zeros_like(v) for k, v in params.items()}
        self.t = 0

    @torch.no_grad()
    def step(self):
        self.t += 1
        lr_t = self.lr * np.sqrt(1 - self.b2 ** self.t) / (1 - self.b1 ** self.t)
        for k, x in self.p.items():
            gk = x.grad
            self.m[k].mul_(self.b1).add_(gk, alpha=1 - self.b1)
            self.v[k].mul_(self.b2).addcmul_(gk, gk, value=1 - self.b2)
            x.sub_(lr_t * self.m[k] / (self.v[k].sqrt() + self.eps))
            x.grad = None


def to_tensors(batch_arrays, cfg, dtype):
    """(adj list, X, Xf, S, eps) flat arrays -> batched torch tensors."""
    adj, X, Xf, S, eps = batch_arrays
    n = cfg.n_nodes
    B = X.shape[0] // n
    t = lambda a: torch.tensor(np.asarray(a), dtype=dtype).reshape(B, n, -1)
    e = torch.tensor(np.asarray(eps), dtype=dtype)
    e = e.reshape(B, -1) if cfg.topology == "tref" else e.reshape(B, n, -1)
    return (torch.tensor(np.stack(adj), dtype=dtype), t(X), t(Xf), t(S), e)
