"""ORACLE -- test infrastructure only.  Never imported by the product path.

Float64 NumPy restatement of the SND-VAE training step as the reference's
TensorFlow 1.x graph computes it, with the backward pass derived by hand (the
reference uses TF autodiff, `optimizer.py:197`).  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may use it.

Parity status: TensorFlow is not installed here and the reference ships no
tests, fixtures or logged values, so this restatement is **parity unpinned**
against TF itself.  It is pinned instead by analytic
known-answer constants, finite differences, and an independent torch-CPU
autograd formulation of the same reference graph (``ref_torch.py``).

Formulas and the reference lines they restate:

  lrelu(x) = max(x, 0.2 x)                                    layers.py:112-113
  GraphConvolution: lrelu(A @ (H @ W)), A raw binary adjacency layers.py:115-125
  BN (Keras, inference mode, moving mean 0 / var 1, eps 1e-3):
      y = gamma * x / sqrt(1.001) + beta                      model.py:41,107,112
  concat [g || node_feature]                                  model.py:109
  linear: x @ Matrix + bias                                   layers.py:566-576
  tref heads: h = flat(G) Wh + bh per graph (row-major reshape) model.py:113-115
  z = mu + eps * exp(logstd)                                  model.py:153-161
  tref projection: J = reshape(z Wp + bp, [B, N, node_h])     model_joint.py:97
  L = J @ J^T; logits (0, L) off-diagonal, (1, 0) on the
      diagonal; argmax first-index tie break                  layers.py:407-409,
                                                              model.py:185,205-208
  adj_cost = mean softmax-CE(labels [1-A, A])                 optimizer.py:142-144
  conv1d k=5 SAME stride 1 (cross-correlation, pad 2|2),
      BN, lrelu, dropout(keep=1)                              model_joint.py:112-145
  node/spatial cost = mean squared difference                 optimizer.py:149,153
  kl = -0.5 mean(1 + 2 s - mu^2 - exp(s)^2)                   optimizer.py:193
  cost = adj + node + spatial + beta * kl                     optimizer.py:157,194
  TF1 Adam                                                    optimizer.py:125,197

Derivative convention for max(x, 0.2x): TF's Maximum gradient routes to the
first input where x >= 0.2x, i.e. lrelu'(x) = 1 for x >= 0 else 0.2.

Parameter dict keys are the physical block names of ``snd_vae_amd/params.py``
(e.g. ``enc.Wms`` = [g_g2_lin/Matrix || g_g3_lin/Matrix]).
"""
from __future__ import annotations

from typing import Dict

import numpy as np

BN_C = 1.0 / np.sqrt(1.0 + 1e-3)
SOFTPLUS_M1 = float(np.logaddexp(0.0, -1.0))   # diag CE: logsumexp(1,0) - 1
K = 5


def lrelu(x):
    return np.maximum(x, 0.2 * x)


def lrelu_grad(x):
    return np.where(x >= 0, 1.0, 0.2)


def sigmoid(x):
    return 0.5 * (1.0 + np.tanh(0.5 * x))


def softplus(x):
    return np.logaddexp(0.0, x)


# ----------------------------------------------------------------- conv1d
def conv1d_same(x, w, b):
    """tf.layers.conv1d(k=5, SAME, stride 1): out[n] = b + sum_t x[n+t-2] @ w[t]."""
    n = x.shape[0]
    xp = np.pad(x, ((2, 2), (0, 0)))
    out = np.broadcast_to(b, (n, w.shape[2])).astype(np.float64).copy()
    for t in range(K):
        out += xp[t:t + n] @ w[t]
    return out


def conv1d_same_bwd(x, w, dy):
    n = x.shape[0]
    xp = np.pad(x, ((2, 2), (0, 0)))
    dyp = np.pad(dy, ((2, 2), (0, 0)))
    dx = np.zeros_like(x, dtype=np.float64)
    dw = np.zeros_like(w, dtype=np.float64)
    for t in range(K):
        dx += dyp[4 - t:4 - t + n] @ w[t].T
        dw[t] = xp[t:t + n].T @ dy
    return dx, dw, dy.sum(0)


def per_graph_conv(x, w, b, n):
    return np.concatenate([conv1d_same(x[i:i + n], w, b) for i in range(0, len(x), n)])


def per_graph_conv_bwd(x, w, dy, n):
    dxs, dw, db = [], np.zeros_like(w, dtype=np.float64), 0.0
    for i in range(0, len(x), n):
        a, b_, c = conv1d_same_bwd(x[i:i + n], w, dy[i:i + n])
        dxs.append(a)
        dw += b_
        db = db + c
    return np.concatenate(dxs), dw, db


# ----------------------------------------------------------------- adjacency
def spmm(adj, h, n):
    """Block-diagonal A @ H with a list of per-graph adjacencies (dense arrays or
    scipy sparse matrices: the same product, O(nnz h) for the latter)."""
    return np.concatenate([np.asarray(adj[b] @ h[b * n:(b + 1) * n]) for b in range(len(adj))])


def _dense_rows(A, lo, hi):
    if hasattr(A, "tocsr"):
        return A[lo:hi].toarray().astype(np.float64)
    return A[lo:hi]


def adj_ce(J, adj, n, pos_weight=1.0, norm=1.0, row_chunk=None, amb_tol=None):
    """Sum over graphs of the 2-class CE with the diagonal rule, plus dJ.

    Returns (ce_sum, dJ_of_sum, n_correct).  ce_sum / (B N^2) is adj_cost.
    The per-pair gradient g is symmetric (L and A are), so dJ = (g + g^T) J =
    2 g J; ``row_chunk`` rows of L at a time bound the memory (N = 16384: a
    dense L is 2 GB in float64), and ``adj`` may hold scipy sparse matrices.
    ``amb_tol``: also return the number of off-diagonal pairs with |L| < amb_tol
    (pairs whose argmax may flip under rounding) as a fourth value.
    """
    ce, correct, amb = 0.0, 0, 0
    dJ = np.zeros_like(J)
    rc = n if row_chunk is None else row_chunk
    for b, A in enumerate(adj):
        Jb = J[b * n:(b + 1) * n]
        for lo in range(0, n, rc):
            hi = min(n, lo + rc)
            L = Jb[lo:hi] @ Jb.T
            Ab = _dense_rows(A, lo, hi)
            off = np.ones(L.shape, dtype=bool)
            off[np.arange(hi - lo), np.arange(lo, hi)] = False
            sp = softplus(L)
            # pos_weight * A * softplus(-L) + (1 - A) * softplus(L); == sp - A L at pw=1
            term = (pos_weight * Ab * (sp - L) + (1.0 - Ab) * sp) * norm
            ce += term[off].sum() + (hi - lo) * SOFTPLUS_M1 * norm
            g = norm * (sigmoid(L) * (1.0 + Ab * (pos_weight - 1.0)) - Ab * pos_weight)
            g[~off] = 0.0
            dJ[b * n + lo:b * n + hi] = 2.0 * (g @ Jb)
            pred = (L > 0) & off                  # argmax(softmax(0, L)), tie -> 0
            correct += int((pred == (Ab > 0)).sum())
            if amb_tol is not None:
                amb += int(((np.abs(L) < amb_tol) & off).sum())
    if amb_tol is not None:
        return ce, dJ, correct, amb
    return ce, dJ, correct


def adj_ce_rows(J, A, n, r0, r1, pos_weight=1.0, norm=1.0, row_chunk=1024):
    """adj_ce of ONE graph restricted to its rows [r0, r1) (the row-sharded zz^T of
    SURVEY §8e): (ce over the range's rows x n pairs, dJ rows [r1 - r0, d] of the
    whole sum's gradient, #correct over the range).  Over a partition of [0, n) the
    ce and correct sum to adj_ce's and the dJ rows concatenate to its dJ."""
    ce, correct = 0.0, 0
    dJ = np.zeros((r1 - r0, J.shape[1]))
    for lo in range(r0, r1, row_chunk):
        hi = min(r1, lo + row_chunk)
        L = J[lo:hi] @ J.T
        Ab = _dense_rows(A, lo, hi)
        off = np.ones(L.shape, dtype=bool)
        off[np.arange(hi - lo), np.arange(lo, hi)] = False
        sp = softplus(L)
        term = (pos_weight * Ab * (sp - L) + (1.0 - Ab) * sp) * norm
        ce += term[off].sum() + (hi - lo) * SOFTPLUS_M1 * norm
        g = norm * (sigmoid(L) * (1.0 + Ab * (pos_weight - 1.0)) - Ab * pos_weight)
        g[~off] = 0.0
        dJ[lo - r0:hi - r0] = 2.0 * (g @ J)
        correct += int((((L > 0) & off) == (Ab > 0)).sum())
    return ce, dJ, correct


# ----------------------------------------------------------------- model
def forward_backward(p: Dict[str, np.ndarray], adj, X, Xf, S, eps, cfg,
                     want_grads=True, row_chunk=None, amb_tol=None, lrelu_override=None):
    """One training step's forward + hand-derived backward.

    adj: list of B [N,N] 0/1 adjacencies (dense arrays, or scipy sparse for
    large N with ``row_chunk``, see adj_ce); X [B*N, f_in]; Xf [B*N, nf];
    S [B*N, 2]; eps [B*N, L] (tscale) or [B, L] (tref, model_joint.py:89).
    Returns (losses dict, grads dict, cache); with ``amb_tol`` the losses hold
    ``ambiguous`` = #{off-diagonal |L| < amb_tol}.

    ``lrelu_override``: {pre-activation name: array of lrelu' values (1.0 / 0.2) or NaN}
    for the names "P0", "P1" (encoder, before BN) and "T1", "T2s", "T3s", "T2n" (decoder,
    BN output): the non-NaN entries replace the derivative at those elements.  A test uses
    it to evaluate the backward pass with a finite-precision evaluation's own derivative
    choice at pre-activations that are zero to within its rounding (where lrelu' is
    discontinuous and either side is a correct evaluation); cache holds every
    pre-activation under these names.
    """
    n = cfg.n_nodes
    R = X.shape[0]
    B = R // n
    L = cfg.latent
    h0, h1 = cfg.g_conv_hidden
    s1 = cfg.s_d_channel[0]
    f64 = lambda a: np.asarray(a, np.float64)
    X, Xf, S, eps = f64(X), f64(Xf), f64(S), f64(eps)
    adj = [a if hasattr(a, "tocsr") else f64(a) for a in adj]
    c = BN_C

    # ---- encoder (model.py:104-115)
    XW0 = X @ p["enc.W0"]
    P0 = spmm(adj, XW0, n)
    A0 = lrelu(P0)
    B0 = A0 * (p["enc.bn0.gamma"] * c) + p["enc.bn0.beta"]
    H1 = np.concatenate([B0, X], 1)
    XW1 = H1 @ p["enc.W1"]
    P1 = spmm(adj, XW1, n)
    A1 = lrelu(P1)
    B1 = A1 * (p["enc.bn1.gamma"] * c) + p["enc.bn1.beta"]
    H2 = np.concatenate([B1, X], 1)
    G = H2 * (p["enc.bne.gamma"] * c) + p["enc.bne.beta"]
    tref = cfg.topology == "tref"
    # heads (model.py:113-115): per node row (tscale) or on flat(G) per graph (tref,
    # tf.reshape(g, [B, -1]) is row-major: flat index n*W + c)
    Gin = G.reshape(B, -1) if tref else G
    h = Gin @ p["enc.Wh"] + p["enc.bh"]
    ms = h @ p["enc.Wms"] + p["enc.bms"]
    mu, s = ms[:, :L], ms[:, L:]
    es = np.exp(s)
    z = mu + eps * es                             # eps [B, L] (tref) / [B*N, L]
    if tref:   # J = reshape(linear(z, N*node_h, 'd_sg_lin1'), [B, N, node_h]) model_joint.py:97
        J = (z @ p["dec.Wp"] + p["dec.bp"]).reshape(B * n, cfg.node_h_size)
    else:
        J = z

    # ---- structure decoder + CE (layers.py:407-409, optimizer.py:144)
    ce_out = adj_ce(J, adj, n, cfg.pos_weight, cfg.norm, row_chunk=row_chunk, amb_tol=amb_tol)
    ce_sum, dJ_adj_sum, correct = ce_out[:3]
    adj_cost = ce_sum / (B * n * n)
    acc = correct / (B * n * n)

    # ---- spatial / node decoders (model_joint.py:112-145)
    Y1 = per_graph_conv(J, p["dec.K1"], p["dec.b1"], n)
    T1 = Y1 * (p["dec.bn1.gamma"] * c) + p["dec.bn1.beta"]
    U1 = lrelu(T1)
    U1s, U1n = U1[:, :s1], U1[:, s1:]
    Y2s = per_graph_conv(U1s, p["dec.K2s"], p["dec.b2s"], n)
    T2s = Y2s * (p["dec.bn2s.gamma"] * c) + p["dec.bn2s.beta"]
    U2s = lrelu(T2s)
    Y3s = per_graph_conv(U2s, p["dec.K3s"], p["dec.b3s"], n)
    T3s = Y3s * (p["dec.bn3s.gamma"] * c) + p["dec.bn3s.beta"]
    U3s = lrelu(T3s)
    Shat = sigmoid(U3s @ p["dec.Ws"] + p["dec.bs"])
    Y2n = per_graph_conv(U1n, p["dec.K2n"], p["dec.b2n"], n)
    T2n = Y2n * (p["dec.bn2n.gamma"] * c) + p["dec.bn2n.beta"]
    U2n = lrelu(T2n)
    Xhat = sigmoid(U2n @ p["dec.Wn"] + p["dec.bn"])

    spatial_cost = np.mean((Shat - S) ** 2)
    node_cost = np.mean((Xhat - Xf) ** 2)
    kl = -0.5 * np.mean(1.0 + 2.0 * s - mu ** 2 - es ** 2)
    cost = adj_cost + node_cost + spatial_cost + cfg.beta * kl
    losses = dict(cost=cost, spatial_cost=spatial_cost, adj_cost=adj_cost,
                  node_cost=node_cost, kl=kl, acc=acc, correct=correct)
    if amb_tol is not None:
        losses["ambiguous"] = ce_out[3]
    cache = dict(J=J, mu=mu, s=s, z=z, G=G, h=h, Shat=Shat, Xhat=Xhat,
                 P0=P0, P1=P1, H1=H1, H2=H2, Y1=Y1, U1=U1, U2s=U2s, U3s=U3s,
                 U2n=U2n, T1=T1, T2s=T2s, T3s=T3s, T2n=T2n, Y2s=Y2s, Y3s=Y3s, Y2n=Y2n)
    if not want_grads:
        return losses, None, cache

    g: Dict[str, np.ndarray] = {}
    # ---- heads + MSE (optimizer.py:149,153)
    dZs = 2.0 * (Shat - S) / Shat.size * Shat * (1.0 - Shat)
    g["dec.Ws"] = U3s.T @ dZs
    g["dec.bs"] = dZs.sum(0)
    dU3s = dZs @ p["dec.Ws"].T
    dZn = 2.0 * (Xhat - Xf) / Xhat.size * Xhat * (1.0 - Xhat)
    g["dec.Wn"] = U2n.T @ dZn
    g["dec.bn"] = dZn.sum(0)
    dU2n = dZn @ p["dec.Wn"].T

    def dlrelu(name, T):
        d = lrelu_grad(T)
        if lrelu_override is not None and name in lrelu_override:
            o = lrelu_override[name]
            d = np.where(np.isnan(o), d, o)
        return d

    def dec_layer(dU, T, Y, Xin, pre, wname, bname, tname):
        dT = dU * dlrelu(tname, T)
        g[pre + ".gamma"] = (dT * Y).sum(0) * c
        g[pre + ".beta"] = dT.sum(0)
        dY = dT * (p[pre + ".gamma"] * c)
        dX, dW, db = per_graph_conv_bwd(Xin, p[wname], dY, n)
        g[wname] = dW
        g[bname] = db
        return dX

    dU2s = dec_layer(dU3s, T3s, Y3s, U2s, "dec.bn3s", "dec.K3s", "dec.b3s", "T3s")
    dU1s = dec_layer(dU2s, T2s, Y2s, U1s, "dec.bn2s", "dec.K2s", "dec.b2s", "T2s")
    dU1n = dec_layer(dU2n, T2n, Y2n, U1n, "dec.bn2n", "dec.K2n", "dec.b2n", "T2n")
    dU1 = np.concatenate([dU1s, dU1n], 1)
    dJ_dec = dec_layer(dU1, T1, Y1, J, "dec.bn1", "dec.K1", "dec.b1", "T1")

    # ---- reparameterisation + KL (model.py:159, optimizer.py:193)
    dJ = dJ_dec + dJ_adj_sum / (B * n * n)
    if tref:   # d_sg_lin1 backward
        dJf = dJ.reshape(B, -1)
        g["dec.Wp"] = z.T @ dJf
        g["dec.bp"] = dJf.sum(0)
        dz = dJf @ p["dec.Wp"].T
    else:
        dz = dJ
    M = mu.size
    dmu = dz + cfg.beta * mu / M
    ds = dz * eps * es + cfg.beta * (es ** 2 - 1.0) / M
    dms = np.concatenate([dmu, ds], 1)
    g["enc.Wms"] = h.T @ dms
    g["enc.bms"] = dms.sum(0)
    dh = dms @ p["enc.Wms"].T
    g["enc.Wh"] = Gin.T @ dh
    g["enc.bh"] = dh.sum(0)
    dG = (dh @ p["enc.Wh"].T).reshape(G.shape)
    g["enc.bne.gamma"] = (dG * H2).sum(0) * c
    g["enc.bne.beta"] = dG.sum(0)
    dH2 = dG * (p["enc.bne.gamma"] * c)
    dB1 = dH2[:, :h1]
    g["enc.bn1.gamma"] = (dB1 * A1).sum(0) * c
    g["enc.bn1.beta"] = dB1.sum(0)
    dP1 = dB1 * (p["enc.bn1.gamma"] * c) * dlrelu("P1", P1)
    dXW1 = spmm(adj, dP1, n)                     # A symmetric
    g["enc.W1"] = H1.T @ dXW1
    dH1 = dXW1 @ p["enc.W1"].T
    dB0 = dH1[:, :h0]
    g["enc.bn0.gamma"] = (dB0 * A0).sum(0) * c
    g["enc.bn0.beta"] = dB0.sum(0)
    dP0 = dB0 * (p["enc.bn0.gamma"] * c) * dlrelu("P0", P0)
    dXW0 = spmm(adj, dP0, n)
    g["enc.W0"] = X.T @ dXW0
    cache["dJ"] = dJ
    return losses, g, cache


# ----------------------------------------------------------------- TF1 Adam

def generated_adj(J, n):
    """model.py:205-208: argmax of softmax over (0, L_ij) off-diagonal, (1, 0) on it.

    Returns (uint8 [B, N, N] predictions, float64 [B, N, N] logits L)."""
    B = len(J) // n
    Lg = np.stack([J[b * n:(b + 1) * n] @ J[b * n:(b + 1) * n].T for b in range(B)])
    pred = (Lg > 0).astype(np.uint8)               # ties (L == 0) -> index 0
    for b in range(B):
        np.fill_diagonal(pred[b], 0)               # diag logits (1, 0) -> index 0
    return pred, Lg


def decode(p: Dict[str, np.ndarray], z, cfg):
    """Decoder forward from a latent z (model.py:163-169 get_random_z + decoder;
    model_joint.py:97,112-145): returns J, generated_spatial, generated_node_feat."""
    n = cfg.n_nodes
    c = BN_C
    s1 = cfg.s_d_channel[0]
    z = np.asarray(z, np.float64)
    if cfg.topology == "tref":
        B = z.shape[0]
        J = (z @ p["dec.Wp"] + p["dec.bp"]).reshape(B * n, cfg.node_h_size)
    else:
        J = z
    U1 = lrelu(per_graph_conv(J, p["dec.K1"], p["dec.b1"], n) * (p["dec.bn1.gamma"] * c)
               + p["dec.bn1.beta"])
    U2s = lrelu(per_graph_conv(U1[:, :s1], p["dec.K2s"], p["dec.b2s"], n)
                * (p["dec.bn2s.gamma"] * c) + p["dec.bn2s.beta"])
    U3s = lrelu(per_graph_conv(U2s, p["dec.K3s"], p["dec.b3s"], n)
                * (p["dec.bn3s.gamma"] * c) + p["dec.bn3s.beta"])
    Shat = sigmoid(U3s @ p["dec.Ws"] + p["dec.bs"])
    U2n = lrelu(per_graph_conv(U1[:, s1:], p["dec.K2n"], p["dec.b2n"], n)
                * (p["dec.bn2n.gamma"] * c) + p["dec.bn2n.beta"])
    Xhat = sigmoid(U2n @ p["dec.Wn"] + p["dec.bn"])
    return J, Shat, Xhat


def adam_tf1(p, g, m, v, t, lr, b1=0.9, b2=0.999, eps=1e-8):
    """tf.train.AdamOptimizer.apply_gradients step t (1-based), in place."""
    lr_t = lr * np.sqrt(1.0 - b2 ** t) / (1.0 - b1 ** t)
    for k in p:
        m[k] = b1 * m[k] + (1.0 - b1) * g[k]
        v[k] = b2 * v[k] + (1.0 - b2) * g[k] ** 2
        p[k] = p[k] - lr_t * m[k] / (np.sqrt(v[k]) + eps)
    return p, m, v


def train_steps(p, adj, X, Xf, S, eps_list, cfg, steps):
    """`steps` reference train steps (main.py:315-331) with injected eps."""
    p = {k: np.array(v, np.float64) for k, v in p.items()}
    m = {k: np.zeros_like(v) for k, v in p.items()}
    v = {k: np.zeros_like(x) for k, x in p.items()}
    hist = []
    for t in range(1, steps + 1):
        losses, grads, _ = forward_backward(p, adj, X, Xf, S, eps_list[t - 1], cfg)
        hist.append((losses, grads))
        adam_tf1(p, grads, m, v, t, cfg.learning_rate, cfg.adam_beta1,
                 cfg.adam_beta2, cfg.adam_eps)
    return p, m, v, hist
