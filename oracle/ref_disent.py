"""ORACLE -- test infrastructure only.  Never imported by the product path.

Literal float64 restatement of the disentangled model's pieces that SURVEY.md
§8f rank 4 widens to:

* the ``e2e`` edge-to-edge filter of the structure decoder (`layers.py:431-450`):
      conv1 = conv2d(x, w1 [1, k_h, C, O], SAME) + b1      (a row filter over j)
      conv2 = conv2d(x, transpose(w1, [1,0,2,3]), SAME) + b1 (the same taps over i)
      e2e   = conv1 + conv2
  with k_h = N (`model.py:196`), TF SAME padding for stride 1: (k-1)//2 before,
  the rest after;
* the latent regularisers of `optimizer.py:159-190`: the per-group KL
  (`optimizer.py:160-162`), the capacity form gamma * relu(kl_sg - C) of
  'disentangled_C' (`:167-171`), DIP (`optimizer.py:7-21`) and the total-correlation
  estimate (`optimizer.py:23-58`, logvar = log(e^s e^s) = 2 s).

numpy for values, torch-CPU float64 autograd for gradients (the stand-in for TF's
autodiff).  Parity status: TensorFlow is unavailable and the reference ships no
fixtures, so this is parity unpinned against TF itself; it is pinned by its
line-by-line correspondence, finite differences and numpy == torch agreement
(tests/test_disent_oracle.py).
"""
from __future__ import annotations

import numpy as np

LOG_2PI = float(np.log(2.0 * np.pi))


# ---------------------------------------------------------------- e2e (layers.py:431-450)
def _pads(k):
    before = (k - 1) // 2
    return before, k - 1 - before


def e2e(x, w1, b1):
    """x [B,N,N,C] (NHWC), w1 [K,C,O] (the [1,K,C,O] kernel), b1 [O] -> [B,N,N,O]."""
    x, w1, b1 = (np.asarray(a, np.float64) for a in (x, w1, b1))
    B, N, _, C = x.shape
    K = w1.shape[0]
    pb, pa = _pads(K)
    xw = np.pad(x, ((0, 0), (0, 0), (pb, pa), (0, 0)))       # conv1: kernel [1, K] slides over j
    xh = np.pad(x, ((0, 0), (pb, pa), (0, 0), (0, 0)))       # conv2: kernel [K, 1] slides over i
    out = np.zeros((B, N, N, w1.shape[2]))
    for t in range(K):
        out += np.einsum("bijc,co->bijo", xw[:, :, t:t + N, :], w1[t])
        out += np.einsum("bijc,co->bijo", xh[:, t:t + N, :, :], w1[t])
    return out + 2.0 * b1


def e2e_torch(x, w1, b1):
    """The same filter in torch-CPU float64 ops (conv2d on NCHW), for autograd."""
    import torch
    import torch.nn.functional as F
    K = w1.shape[0]
    pb, pa = _pads(K)
    xc = x.permute(0, 3, 1, 2)                                # NCHW
    wk = w1.permute(2, 1, 0)                                  # [O, C, K]
    c1 = F.conv2d(F.pad(xc, (pb, pa, 0, 0)), wk[:, :, None, :])
    c2 = F.conv2d(F.pad(xc, (0, 0, pb, pa)), wk[:, :, :, None])
    return (c1 + c2).permute(0, 2, 3, 1) + 2.0 * b1


def e2e_grads(x, w1, b1, dout):
    """(dx, dw1, db1) of sum(e2e(x) * dout) by torch autograd (float64)."""
    import torch
    xt = torch.tensor(np.asarray(x, np.float64), requires_grad=True)
    wt = torch.tensor(np.asarray(w1, np.float64), requires_grad=True)
    bt = torch.tensor(np.asarray(b1, np.float64), requires_grad=True)
    (e2e_torch(xt, wt, bt) * torch.tensor(np.asarray(dout, np.float64))).sum().backward()
    return xt.grad.numpy(), wt.grad.numpy(), bt.grad.numpy()


# ---------------------------------------------------------------- latent regularisers
def kl(mu, s):
    """-0.5 * mean(1 + 2 s - mu^2 - exp(s)^2)  (optimizer.py:160)."""
    mu, s = np.asarray(mu, np.float64), np.asarray(s, np.float64)
    return float(-0.5 * np.mean(1.0 + 2.0 * s - mu ** 2 - np.exp(s) ** 2))


def dip(mu, lambda_od, lambda_d):
    """DIP-VAE regulariser of the encoder means (optimizer.py:7-21)."""
    mu = np.asarray(mu, np.float64)
    m = mu.mean(0)
    cov = (mu[:, None, :] * mu[:, :, None]).mean(0) - m[None, :] * m[:, None]
    d = np.diag(cov)
    off = cov - np.diag(d)
    return float(lambda_od * np.sum(off ** 2) + lambda_d * np.sum((d - 1.0) ** 2))


def _lse(a, axis):
    mx = a.max(axis=axis, keepdims=True)
    return (mx + np.log(np.exp(a - mx).sum(axis=axis, keepdims=True))).squeeze(axis)


def total_correlation(z, mu, s):
    """Minibatch total-correlation estimate (optimizer.py:23-58), logvar = 2 s."""
    z, mu, s = (np.asarray(a, np.float64) for a in (z, mu, s))
    logvar = np.log(np.exp(s) * np.exp(s))
    tmp = z[:, None, :] - mu[None, :, :]                      # [j, i, l]
    lqp = -0.5 * (tmp * tmp * np.exp(-logvar[None]) + logvar[None] + LOG_2PI)
    log_qz_product = _lse(lqp, 1).sum(1)
    log_qz = _lse(lqp.sum(2), 1)
    return float(np.mean(log_qz - log_qz_product))


def capacity(global_iter, c_max, c_step, c_stop_iter):
    """C of 'disentangled_C' (optimizer.py:167)."""
    return float(np.clip(c_max * c_step / c_stop_iter * (global_iter // c_step), 0.0, c_max))


def group_reg(mu, s, z, w_kl=1.0, cap_gamma=0.0, cap_c=0.0, w_dip=0.0, lambda_od=10.0, lambda_d=100.0,
              w_tc=0.0):
    """One latent group's term of the cost: w_kl * kl (or cap_gamma * relu(kl - cap_c) when
    cap_gamma > 0) + w_dip * DIP(mu) + w_tc * TC(z, mu, s), and its value parts."""
    k = kl(mu, s)
    kterm = cap_gamma * max(k - cap_c, 0.0) if cap_gamma > 0 else w_kl * k
    dv = dip(mu, lambda_od, lambda_d) if w_dip else 0.0
    tv = total_correlation(z, mu, s) if w_tc else 0.0
    return {"kl": k, "term": kterm + w_dip * dv + w_tc * tv, "dip": dv, "tc": tv}


def group_reg_torch(mu, s, eps, **kw):
    """The same term in torch float64 with z = mu + eps * exp(s) (model.py:155-159),
    returning (value, dmu, ds): the gradients through z are chained as TF's autodiff does."""
    import torch
    mt = torch.tensor(np.asarray(mu, np.float64), requires_grad=True)
    st = torch.tensor(np.asarray(s, np.float64), requires_grad=True)
    z = mt + torch.tensor(np.asarray(eps, np.float64)) * torch.exp(st)
    w_kl, cap_gamma, cap_c = kw.get("w_kl", 1.0), kw.get("cap_gamma", 0.0), kw.get("cap_c", 0.0)
    w_dip, lod, ld, w_tc = kw.get("w_dip", 0.0), kw.get("lambda_od", 10.0), kw.get("lambda_d", 100.0), kw.get("w_tc", 0.0)
    k = -0.5 * torch.mean(1 + 2 * st - mt ** 2 - torch.exp(st) ** 2)
    val = cap_gamma * torch.relu(k - cap_c) if cap_gamma > 0 else w_kl * k
    if w_dip:
        m = mt.mean(0)
        cov = (mt[:, None, :] * mt[:, :, None]).mean(0) - m[None, :] * m[:, None]
        d = torch.diagonal(cov)
        val = val + w_dip * (lod * torch.sum((cov - torch.diag(d)) ** 2) + ld * torch.sum((d - 1) ** 2))
    if w_tc:
        logvar = torch.log(torch.exp(st) * torch.exp(st))
        tmp = z[:, None, :] - mt[None, :, :]
        lqp = -0.5 * (tmp * tmp * torch.exp(-logvar[None]) + logvar[None] + LOG_2PI)
        tc = torch.mean(torch.logsumexp(lqp.sum(2), 1) - torch.logsumexp(lqp, 1).sum(1))
        val = val + w_tc * tc
    val.backward()
    return float(val.detach()), mt.grad.numpy(), st.grad.numpy()


def model_type_groups(model_type, beta=1.0, gamma=1.0, c=0.0):
    """Per-group weights of optimizer.py:159-190 for the groups (s, g, sg)."""
    if model_type in ("disentangled", "geoGCN", "posGCN"):
        return {"s": {"w_kl": beta}, "g": {"w_kl": beta}, "sg": {"w_kl": beta}}
    if model_type == "disentangled_C":
        return {"s": {"w_kl": 1.0}, "g": {"w_kl": 1.0}, "sg": {"w_kl": 0.0, "cap_gamma": gamma, "cap_c": c}}
    if model_type == "NED-VAE-IP":
        d = {"w_kl": 1.0, "w_dip": beta, "lambda_od": 10.0, "lambda_d": 100.0}
        return {"s": dict(d), "g": dict(d), "sg": dict(d)}
    if model_type == "beta-TCVAE":
        return {"s": {"w_kl": beta, "w_tc": 10.0}, "g": {"w_kl": beta, "w_tc": 10.0},
                "sg": {"w_kl": beta, "w_tc": 10.0}}
    return {"sg": {"w_kl": beta}}                               # 'base' (optimizer.py:186-188)


# ---------------------------------------------------------------- e2e structure decoder
BN_C = 1.0 / np.sqrt(1.0 + 1e-3)


def structure_decoder_torch(z, adj, layers, head):
    """model.py:193-208 + optimizer.py:142-144 literally, torch float64 (autograd-ready):
    pairwise concat [z_i | z_j], per layer e2e(relu(BN(h))), relu(BN(h)) @ W + b, the
    diagonal set to (1, 0), mean softmax-CE against [1 - A, A]; returns (ce, correct)."""
    import torch
    B, N, D = z.shape
    h = torch.cat([z[:, :, None, :].expand(B, N, N, D), z[:, None, :, :].expand(B, N, N, D)], -1)
    for lay in layers:
        h = e2e_torch(torch.relu(lay["gamma"] * h * BN_C + lay["beta"]), lay["w"], lay["b"])
    logits = torch.relu(head["gamma"] * h * BN_C + head["beta"]) @ head["w"] + head["b"]
    diag = 1.0 - torch.eye(N, dtype=logits.dtype)[None]
    p1 = diag * logits[..., 1]
    p0 = diag * logits[..., 0] + (1.0 - diag)
    prob = torch.stack([p0, p1], -1)
    a = torch.as_tensor(adj, dtype=logits.dtype)
    labels = torch.stack([1.0 - a, a], -1)
    ce = torch.mean(torch.logsumexp(prob, -1) - (labels * prob).sum(-1))
    correct = float(((p1 > p0).to(a.dtype) == a).sum())
    return ce, correct


def structure_decoder_grads(z, adj, layers, head):
    """(ce, correct, dz, layer grads, head grads) by torch autograd, float64."""
    import torch
    t = lambda a: torch.tensor(np.asarray(a, np.float64), requires_grad=True)
    zt = t(z)
    lt = [{k: t(v) for k, v in lay.items()} for lay in layers]
    ht = {k: t(v) for k, v in head.items()}
    ce, correct = structure_decoder_torch(zt, adj, lt, ht)
    ce.backward()
    g = lambda d: {k: v.grad.numpy() for k, v in d.items()}
    return float(ce.detach()), correct, zt.grad.numpy(), [g(l) for l in lt], g(ht)
