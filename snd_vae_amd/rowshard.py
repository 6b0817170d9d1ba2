"""Row-sharded training step of ONE large graph over several ranks (SURVEY §8e "beyond
DP"; C5: N = 16384, d = 128 -- a graph whose step cannot be split by graphs).

Every rank owns a contiguous, 128-row-aligned range of the graph's rows
(``parallel.row_ranges``) and computes the node-latent SND-VAE step (`model.py:104-161`,
`model_joint.py:112-145`, `optimizer.py:142-197`) for those rows; the weights are
replicated and their gradients all-reduced, exactly as the data-parallel step does.
What crosses ranks, per step:

* encoder, GraphConvolution 1: its input H1 = [BN0(lrelu(A X W0)) || X] is all-gathered
  (every rank multiplies the whole H1 by W1 and takes its rows of A @ (H1 W1)); layer 0
  needs only X, which every rank holds.  Backward: dH1 = (A[:, own] dP1) W1^T has rows on
  every rank -- reduce-scattered to the owners.  The rows of A are the rank's slice of
  the CSR (global column ids); A[:, own] = A[own, :]^T (A symmetric) is a CSR over all
  N rows with the rank's columns (``RowShardPlan.cols``).
* structure decoder: z is all-gathered; the rank's rows of the fused CE against all N
  columns (``snd_zzt_ce_rows``) give d(total CE)/dz for its own rows with no reduction
  (L symmetric), and its share of the CE sum and correct count.
* conv1d decoders (k = 5 SAME along the node axis, 3 layers): the rank recomputes them on
  the window [r0 - 6, r1 + 6) of the gathered z (2 halo rows per layer and side; graph
  ends keep TF's zero padding) and keeps its own rows.  Backward: the window's dJ is
  scattered into a zero [N, d] tensor and reduce-scattered to the owners.
* the loss terms: sums over own rows, all-reduced; every mean uses the whole graph's
  count (node_cost over N nf, adj_cost over N^2, KL over N L).

The arithmetic is a list of calls on an ``ops`` object (the HIP C ABI on the device:
``HipOps``; the CPU tests plug in a float64 torch restatement) and the collectives go
through a ``comm`` object (``TorchComm``: torch.distributed over RCCL, or gloo with the
device tensors staged through host memory).  The fused single-device step
(``snd_train_step``) stays the throughput path; this step is fp32 and composes ABI
launches from the host, one per layer (``disent_model.py`` does the same).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, Tuple

import numpy as np
import torch

from .config import SNDConfig
from .parallel import row_ranges

HALO = 6            # 3 conv1d layers x 2 rows (k = 5 SAME)


@dataclass
class RowCSR:
    """A CSR whose output rows are n_out (rowptr rebased to 0) over an input matrix of any
    row count (colidx indexes its rows)."""
    rowptr: torch.Tensor
    colidx: torch.Tensor
    n_out: int


class RowShardPlan:
    """Host-side layout of one rank's share of one graph (built once per graph).

    rowptr / colidx: the graph's CSR (numpy, symmetric, no diagonal)."""

    def __init__(self, rowptr: np.ndarray, colidx: np.ndarray, n: int, rank: int, world: int,
                 device, block: int = 128, index_dtype=torch.int32):
        import scipy.sparse as sp
        self.n, self.rank, self.world = n, rank, world
        self.ranges = row_ranges(n, world, block)
        self.r0, self.r1 = self.ranges[rank]
        if any(b <= a for a, b in self.ranges):
            raise ValueError(f"row sharding: {world} ranks over {n} rows in {block}-row blocks leaves "
                             f"a rank without rows ({self.ranges}); use at most {-(-n // block)} ranks")
        rowptr = np.asarray(rowptr, np.int64)
        colidx = np.asarray(colidx, np.int64)
        A = sp.csr_matrix((np.ones(len(colidx)), colidx, rowptr), shape=(n, n))
        own = A[self.r0:self.r1].tocsr()
        cols = A[:, self.r0:self.r1].tocsr()          # = own^T (A symmetric), all n rows
        cols.sort_indices()
        mk = lambda a: torch.as_tensor(np.asarray(a), dtype=index_dtype, device=device)
        self.rows = RowCSR(mk(own.indptr), mk(own.indices), self.r1 - self.r0)
        self.cols = RowCSR(mk(cols.indptr), mk(cols.indices), n)
        # snd_zzt_ce_rows: the range's slice of the GRAPH's row pointers (not rebased)
        self.ce_rowptr = mk(rowptr[self.r0:self.r1 + 1])
        self.ce_colidx = mk(colidx if len(colidx) else np.zeros(1, np.int64))
        self.w0 = max(0, self.r0 - HALO)
        self.w1 = min(n, self.r1 + HALO)
        self.scipy_rows = own                         # for CPU restatements (tests)


def _cat(a, b):
    return torch.cat([a, b], 1).contiguous()


def forward_backward(p: Dict[str, torch.Tensor], plan: RowShardPlan, X_full, Xf_own, S_own, eps_own,
                     cfg: SNDConfig, ops, comm) -> Tuple[Dict[str, float], Dict[str, torch.Tensor]]:
    """One row-sharded step's forward + backward (node latent).  p: the replicated
    parameters (2D/1D tensors, the params.py block names); X_full [N, f_in]; Xf_own /
    S_own / eps_own: the rank's rows.  Returns (losses, grads): the losses of the WHOLE
    graph (all-reduced) and the WHOLE gradient (all-reduced) on every rank."""
    n, r0, r1, w0, w1 = plan.n, plan.r0, plan.r1, plan.w0, plan.w1
    L = cfg.latent
    h0, h1 = cfg.g_conv_hidden
    s1 = cfg.s_d_channel[0]
    g: Dict[str, torch.Tensor] = {}

    # ---- encoder (model.py:104-115)
    XW0 = ops.mm(X_full, p["enc.W0"])                                   # [N, h0] (X on every rank)
    P0 = ops.spmm(plan.rows, XW0)                                       # own rows of A X W0
    B0 = ops.bn_act(P0, p["enc.bn0.gamma"], p["enc.bn0.beta"], 2, True)  # BN(lrelu(.))
    X_own = X_full[r0:r1].contiguous()
    H1 = _cat(B0, X_own)
    H1_full = comm.all_gather_rows(H1, plan.ranges)
    XW1 = ops.mm(H1_full, p["enc.W1"])
    P1 = ops.spmm(plan.rows, XW1)
    B1 = ops.bn_act(P1, p["enc.bn1.gamma"], p["enc.bn1.beta"], 2, True)
    H2 = _cat(B1, X_own)
    G = ops.bn_act(H2, p["enc.bne.gamma"], p["enc.bne.beta"], 0, False)
    h = ops.linear(G, p["enc.Wh"], p["enc.bh"])
    ms = ops.linear(h, p["enc.Wms"], p["enc.bms"])
    mu, s = ms[:, :L].contiguous(), ms[:, L:].contiguous()
    z, kl_part = ops.reparam(mu, s, eps_own)

    # ---- structure decoder + CE over the rank's rows (layers.py:407-409, optimizer.py:144)
    z_full = comm.all_gather_rows(z, plan.ranges)
    ce_sum, correct, dz_adj = ops.adj_ce_rows(z_full, plan, cfg.pos_weight, cfg.norm)

    # ---- conv1d decoders on the window, own rows kept (model_joint.py:112-145)
    J = z_full[w0:w1].contiguous()
    o0, o1 = r0 - w0, r1 - w0                         # own rows inside the window
    Y1, U1 = ops.conv_bn_lrelu(J, p["dec.K1"], p["dec.b1"], p["dec.bn1.gamma"], p["dec.bn1.beta"])
    U1s, U1n = U1[:, :s1].contiguous(), U1[:, s1:].contiguous()
    Y2s, U2s = ops.conv_bn_lrelu(U1s, p["dec.K2s"], p["dec.b2s"], p["dec.bn2s.gamma"], p["dec.bn2s.beta"])
    Y3s, U3s = ops.conv_bn_lrelu(U2s, p["dec.K3s"], p["dec.b3s"], p["dec.bn3s.gamma"], p["dec.bn3s.beta"])
    Y2n, U2n = ops.conv_bn_lrelu(U1n, p["dec.K2n"], p["dec.b2n"], p["dec.bn2n.gamma"], p["dec.bn2n.beta"])
    nf, sd = cfg.num_feature, cfg.spatial_dim
    sse_s, dU3s_own, g["dec.Ws"], g["dec.bs"] = ops.sigmoid_mse(U3s[o0:o1].contiguous(), p["dec.Ws"],
                                                                p["dec.bs"], S_own, n * sd)
    sse_n, dU2n_own, g["dec.Wn"], g["dec.bn"] = ops.sigmoid_mse(U2n[o0:o1].contiguous(), p["dec.Wn"],
                                                                p["dec.bn"], Xf_own, n * nf)

    # ---- loss terms of the whole graph
    stats = torch.tensor([ce_sum, float(correct), sse_s, sse_n, kl_part], dtype=torch.float64)
    stats = comm.all_reduce_host(stats)
    adj_cost = stats[0].item() / (n * n)
    spatial_cost = stats[2].item() / (n * sd)
    node_cost = stats[3].item() / (n * nf)
    kl = -0.5 * stats[4].item() / (n * L)
    losses = dict(cost=adj_cost + node_cost + spatial_cost + cfg.beta * kl, adj_cost=adj_cost,
                  spatial_cost=spatial_cost, node_cost=node_cost, kl=kl,
                  correct=stats[1].item(), acc=stats[1].item() / (n * n))

    # ---- decoder backward on the window (gradients only from the own rows)
    def own_rows(d_own, width):
        full = torch.zeros(w1 - w0, width, dtype=d_own.dtype, device=d_own.device)
        full[o0:o1] = d_own
        return full

    def dec_layer(dU, Y, Xin, pre, wname, bname):
        dY, g[pre + ".gamma"], g[pre + ".beta"] = ops.bn_act_bwd(dU, Y, p[pre + ".gamma"], p[pre + ".beta"], 2, False)
        dX, g[wname] = ops.conv_bwd(Xin, p[wname], dY)
        g[bname] = ops.colsum(dY)
        return dX

    dU2s = dec_layer(own_rows(dU3s_own, U3s.shape[1]), Y3s, U2s, "dec.bn3s", "dec.K3s", "dec.b3s")
    dU1s = dec_layer(dU2s, Y2s, U1s, "dec.bn2s", "dec.K2s", "dec.b2s")
    dU1n = dec_layer(own_rows(dU2n_own, U2n.shape[1]), Y2n, U1n, "dec.bn2n", "dec.K2n", "dec.b2n")
    dJ_win = dec_layer(_cat(dU1s, dU1n), Y1, J, "dec.bn1", "dec.K1", "dec.b1")
    dJ_full = torch.zeros(n, L, dtype=dJ_win.dtype, device=dJ_win.device)
    dJ_full[w0:w1] = dJ_win
    dJ_dec = comm.reduce_scatter_rows(dJ_full, plan.ranges)

    # ---- reparameterisation + KL backward (model.py:159, optimizer.py:193)
    dz = (dJ_dec + dz_adj / (n * n)).contiguous()
    dmu, ds = ops.reparam_bwd(mu, s, eps_own, dz, cfg.beta / (n * L))
    dms = _cat(dmu, ds)
    g["enc.Wms"] = ops.mm_tn(h, dms)
    g["enc.bms"] = ops.colsum(dms)
    dh = ops.mm_nt(dms, p["enc.Wms"])
    g["enc.Wh"] = ops.mm_tn(G, dh)
    g["enc.bh"] = ops.colsum(dh)
    dG = ops.mm_nt(dh, p["enc.Wh"])
    dH2, g["enc.bne.gamma"], g["enc.bne.beta"] = ops.bn_act_bwd(dG, H2, p["enc.bne.gamma"], p["enc.bne.beta"], 0, False)
    dP1, g["enc.bn1.gamma"], g["enc.bn1.beta"] = ops.bn_act_bwd(dH2[:, :h1].contiguous(), P1, p["enc.bn1.gamma"],
                                                                p["enc.bn1.beta"], 2, True)
    dXW1 = ops.spmm(plan.cols, dP1)                  # A[:, own] dP1: every row of the graph
    g["enc.W1"] = ops.mm_tn(H1_full, dXW1)
    dH1 = comm.reduce_scatter_rows(ops.mm_nt(dXW1, p["enc.W1"]), plan.ranges)
    dP0, g["enc.bn0.gamma"], g["enc.bn0.beta"] = ops.bn_act_bwd(dH1[:, :h0].contiguous(), P0, p["enc.bn0.gamma"],
                                                                p["enc.bn0.beta"], 2, True)
    dXW0 = ops.spmm(plan.cols, dP0)
    g["enc.W0"] = ops.mm_tn(X_full, dXW0)
    # the replicated weights: one all-reduce of every block's partial gradient
    g = comm.all_reduce_blocks(g)
    return losses, g


# ---------------------------------------------------------------- collectives
class TorchComm:
    """The step's collectives over torch.distributed.  staged=True moves device tensors
    through host memory (gloo between processes that share one GPU: the single-box
    rehearsal); otherwise the tensors go to the backend as they are (RCCL, or gloo on
    CPU tensors).  group None with world 1: identity."""

    def __init__(self, group=None, staged: bool = False, device=None):
        import torch.distributed as dist
        self.dist, self.group, self.staged = dist, group, staged
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        # where host-side scalars go for the collective: RCCL takes device tensors only,
        # so a non-staged RCCL group without an explicit device uses the current GPU
        if staged:
            self.scalar_device = torch.device("cpu")
        elif device is not None:
            self.scalar_device = torch.device(device)
        elif dist.is_initialized() and dist.get_backend(group) in ("nccl", "rccl"):
            self.scalar_device = torch.device("cuda", torch.cuda.current_device())
        else:
            self.scalar_device = torch.device("cpu")

    def _io(self, t):
        return t.cpu() if self.staged else t

    def _back(self, t, like):
        return t.to(like.device) if self.staged else t

    def all_gather_rows(self, x_own, ranges):
        if self.world == 1:
            return x_own
        from .parallel import allgather_rows
        return self._back(allgather_rows(self._io(x_own).contiguous(), ranges, self.group), x_own)

    def reduce_scatter_rows(self, x_full, ranges):
        """Sum over ranks of x_full [N, ...], this rank's rows (one reduce-scatter)."""
        if self.world == 1:
            return x_full
        from .parallel import reducescatter_rows
        return self._back(reducescatter_rows(self._io(x_full).contiguous(), ranges, self.group), x_full)

    def all_reduce_host(self, t):
        if self.world > 1:
            d = t.to(self.scalar_device)
            self.dist.all_reduce(d, group=self.group)
            t = d.cpu()
        return t

    def all_reduce_blocks(self, g):
        if self.world == 1:
            return g
        keys = sorted(g)
        flat = torch.cat([g[k].reshape(-1) for k in keys])
        flat = self._io(flat)
        self.dist.all_reduce(flat, group=self.group)
        out, o = {}, 0
        for k in keys:
            m = g[k].numel()
            out[k] = self._back(flat[o:o + m].reshape(g[k].shape), g[k])
            o += m
        return out


# ---------------------------------------------------------------- HIP ops
class HipOps:
    """The step's arithmetic on the C ABI (fp32; every call one or two launches on the
    current stream).  Elementwise glue (slices, concatenation, the KL gradient's two
    vectors) stays in torch."""

    def __init__(self):
        from . import _lib
        self._lib = _lib
        self.L = _lib.lib()
        self.P = _lib.ptr

    def _s(self):
        return self._lib.stream_ptr()

    def _gemm(self, ta, tb, m, n, k, a, lda, b, ldb, c, ldc, bias=None):
        self._lib.check(self.L.snd_gemm(int(ta), int(tb), m, n, k, self.P(a), lda, self.P(b), ldb, self.P(c), ldc,
                                        self.P(bias), 0, self._s()), "snd_gemm")

    def mm(self, a, b, bias=None):
        m, k = a.shape
        n = b.shape[1]
        out = torch.empty(m, n, device=a.device)
        self._gemm(0, 0, m, n, k, a.contiguous(), k, b.contiguous(), n, out, n, bias)
        return out

    def linear(self, x, w, b):
        return self.mm(x, w, b)

    def mm_tn(self, a, b):          # a^T b
        m, k = a.shape
        n = b.shape[1]
        out = torch.empty(k, n, device=a.device)
        self._gemm(1, 0, k, n, m, a.contiguous(), k, b.contiguous(), n, out, n)
        return out

    def mm_nt(self, a, b):          # a b^T
        m, n = a.shape
        k = b.shape[0]
        out = torch.empty(m, k, device=a.device)
        self._gemm(0, 1, m, k, n, a.contiguous(), n, b.contiguous(), n, out, k)
        return out

    def colsum(self, a):
        m, n = a.shape
        ones = torch.ones(m, 1, device=a.device)
        out = torch.empty(1, n, device=a.device)
        self._gemm(1, 0, 1, n, m, ones, 1, a.contiguous(), n, out, n)
        return out.view(n)

    def spmm(self, csr: RowCSR, h):
        width = h.shape[1]
        out = torch.empty(csr.n_out, width, device=h.device)
        self._lib.check(self.L.snd_csr_spmm(
            self.P(csr.rowptr), self.P(csr.colidx), csr.n_out, self.P(h.contiguous()), width, width, self.P(out),
            width, 0, None, None, None, 0, None, 0, 0, None, None, None, 0, self._s()), "snd_csr_spmm")
        return out

    def bn_act(self, y, gamma, beta, act, act_first):
        rows, c = y.shape
        x = torch.empty_like(y)
        self._lib.check(self.L.snd_bn_act_fwd(self.P(y), c, rows, c, self.P(gamma), self.P(beta), act,
                                              int(act_first), self.P(x), c, self._s()), "snd_bn_act_fwd")
        return x

    def bn_act_bwd(self, dx, y, gamma, beta, act, act_first):
        rows, c = y.shape
        dy = torch.empty_like(y)
        dg = torch.empty(c, device=y.device)
        db = torch.empty(c, device=y.device)
        self._lib.check(self.L.snd_bn_act_bwd(self.P(dx.contiguous()), c, self.P(y), c, rows, c, self.P(gamma),
                                              self.P(beta), act, int(act_first), self.P(dy), c, self.P(dg),
                                              self.P(db), self._s()), "snd_bn_act_bwd")
        return dy, dg, db

    def conv_bn_lrelu(self, x, w, b, gamma, beta):
        rows, cin = x.shape
        cout = w.shape[2]
        y = torch.empty(rows, cout, device=x.device)
        u = torch.empty(rows, cout, device=x.device)
        self._lib.check(self.L.snd_conv1d_same_fwd(self.P(x), cin, rows, rows, cin, self.P(w), cout, self.P(b),
                                                   self.P(gamma), self.P(beta), self.P(y), cout, self.P(u), cout, 0,
                                                   self._s()), "snd_conv1d_same_fwd")
        return y, u

    def conv_bwd(self, x, w, dy):
        rows, cin = x.shape
        cout = w.shape[2]
        dx = torch.empty(rows, cin, device=x.device)
        self._lib.check(self.L.snd_conv1d_same_bwd_data(self.P(dy), cout, rows, rows, cout, self.P(w), cin,
                                                        self.P(dx), cin, 0, self._s()), "snd_conv1d_same_bwd_data")
        nws = self.L.snd_conv1d_bwd_weight_workspace(rows, cin, cout)
        ws = torch.empty(max(nws, 16), dtype=torch.uint8, device=x.device)
        dw = torch.empty_like(w)
        self._lib.check(self.L.snd_conv1d_same_bwd_weight(self.P(x), cin, self.P(dy), cout, rows, rows, cin, cout,
                                                          self.P(dw), self.P(ws), nws, 0, self._s()),
                        "snd_conv1d_same_bwd_weight")
        return dx, dw

    def sigmoid_mse(self, u, w, b, target, count):
        """(sse over the rows, du, dw, db) with the mean over `count` elements (the whole
        graph's): the kernel's own denominator is rows * cout, rescaled here."""
        rows, cin = u.shape
        cout = w.shape[1]
        nb = self.L.snd_sigmoid_mse_blocks(rows)
        sse = torch.zeros(nb, dtype=torch.float64, device=u.device)
        yhat = torch.empty(rows, cout, device=u.device)
        du = torch.empty(rows, cin, device=u.device)
        dw = torch.zeros_like(w)
        db = torch.zeros_like(b)
        ws = torch.empty(max(1, nb * (cin * cout + cout)), device=u.device)
        self._lib.check(self.L.snd_sigmoid_mse(self.P(u), cin, rows, cin, self.P(w), self.P(b), cout,
                                               self.P(target.contiguous()), cout, self.P(sse), self.P(yhat),
                                               self.P(du), cin, self.P(dw), self.P(db), self.P(ws),
                                               ws.numel() * 4, self._s()), "snd_sigmoid_mse")
        sc = (rows * cout) / float(count)
        return float(sse.sum().item()), du * sc, dw * sc, db * sc

    def reparam(self, mu, s, eps):
        """z = mu + eps e^s and sum(1 + 2s - mu^2 - e^{2s}) over the rows (snd_reparam_kl)."""
        rows, lat = mu.shape
        ms = _cat(mu, s)
        z = torch.empty(rows, lat, device=mu.device)
        kl = torch.zeros(self.L.snd_reparam_kl_blocks(rows, lat), dtype=torch.float64, device=mu.device)
        self._lib.check(self.L.snd_reparam_kl(self.P(ms), 2 * lat, rows, lat, self.P(eps.contiguous()), 0, None,
                                              None, self.P(z), self.P(kl), self._s()), "snd_reparam_kl")
        return z, float(kl.sum().item())

    def reparam_bwd(self, mu, s, eps, dz, kl_coef):
        """(dmu, ds) of z = mu + eps e^s plus kl_coef * d/d(mu, s) of -0.5 sum(1 + 2s - mu^2 - e^{2s})."""
        rows, lat = mu.shape
        ms = _cat(mu, s)
        add_mu = (kl_coef * mu).contiguous()
        add_s = (kl_coef * torch.expm1(2.0 * s)).contiguous()
        dms = torch.empty(rows, 2 * lat, device=mu.device)
        self._lib.check(self.L.snd_reparam_bwd(self.P(ms), 2 * lat, rows, lat, self.P(eps.contiguous()),
                                               self.P(dz), self.P(add_mu), self.P(add_s), self.P(dms), 2 * lat,
                                               self._s()), "snd_reparam_bwd")
        return dms[:, :lat], dms[:, lat:]

    def adj_ce_rows(self, z_full, plan: RowShardPlan, pos_weight, norm):
        """The range's CE sum and correct count, and d(total CE)/dz for its rows (fp32)."""
        n, d = z_full.shape
        wsb = self.L.snd_zzt_ce_rows_workspace(n, d, plan.r0, plan.r1, 0)
        ws = torch.empty(max(wsb, 16), dtype=torch.uint8, device=z_full.device)
        stats = torch.zeros(2, dtype=torch.float64, device=z_full.device)
        dz = torch.empty(plan.r1 - plan.r0, d, device=z_full.device)
        self._lib.check(self.L.snd_zzt_ce_rows(self.P(z_full.contiguous()), n, d, plan.r0, plan.r1,
                                               self.P(plan.ce_rowptr), self.P(plan.ce_colidx), float(pos_weight),
                                               float(norm), self.P(stats), self.P(dz), self.P(ws), wsb, 0,
                                               self._s()), "snd_zzt_ce_rows")
        st = stats.cpu()
        return float(st[0]), float(st[1]), dz


class RowShardedVAE:
    """Parameters (replicated, one flat fp32 buffer in params.py order), TF1 Adam over it
    (snd_adam_tf1), and the row-sharded step."""

    def __init__(self, cfg: SNDConfig, plan: RowShardPlan, comm, blocks=None, seed: int = 0, device=None):
        from .params import flat_layout, init_blocks
        if cfg.topology != "tscale":
            raise ValueError("row sharding covers the node-latent model (one graph, C5)")
        self.cfg, self.plan, self.comm = cfg, plan, comm
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        self.layout = flat_layout(cfg)
        blocks = blocks if blocks is not None else init_blocks(cfg, seed)
        host = self.layout.pack({k: np.asarray(v, np.float32) for k, v in blocks.items()})
        self.params = torch.from_numpy(np.ascontiguousarray(host)).to(self.device)
        self.grads = torch.zeros_like(self.params)
        self.m = torch.zeros_like(self.params)
        self.v = torch.zeros_like(self.params)
        self.step_counter = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.ops = HipOps()

    def views(self, flat):
        return {k: flat[o:o + int(np.prod(sh))].view(*sh) for k, (o, sh) in
                ((k, (self.layout.offsets[k], self.layout.shapes[k])) for k in self.layout.shapes)}

    def step(self, X_full, Xf_own, S_own, eps_own):
        from . import _lib
        losses, g = forward_backward(self.views(self.params), self.plan, X_full, Xf_own, S_own, eps_own,
                                     self.cfg, self.ops, self.comm)
        gv = self.views(self.grads)
        for k, t in g.items():
            gv[k].copy_(t.reshape(gv[k].shape))
        self.step_counter += 1
        c = self.cfg
        _lib.check(_lib.lib().snd_adam_tf1(_lib.ptr(self.params), _lib.ptr(self.grads), _lib.ptr(self.m),
                                           _lib.ptr(self.v), self.layout.total, c.learning_rate, c.adam_beta1,
                                           c.adam_beta2, c.adam_eps, 1.0, _lib.ptr(self.step_counter),
                                           _lib.stream_ptr()), "snd_adam_tf1")
        return losses

    def blocks(self):
        return {k: v.detach().double().cpu().numpy() for k, v in self.views(self.params).items()}
