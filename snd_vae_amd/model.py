"""SGCNModelVAE on MI355X: parameters, plan and device batch.

Host-side mirror of the reference model classes for the hot path
(`model.py:19-161` encoder/get_z, `model_joint.py:94-182` decoders) in both
decoder-input topologies (node latent ``tscale``; graph latent ``tref`` with
the 'd_sg_lin1' projection of `model_joint.py:97`).  The reference builds a TF graph whose variables live in
the TF store; here a ``snd_plan`` (libsndvae.so) fixes the shapes of one
device batch and all trainable state is one flat fp32 device buffer
(`params.py`).  Forward + backward run as one native launch sequence
(``snd_train_step``); this class owns memory, not compute.

Attributes named as in the reference (read back after a step):
``z_mean_sg``/``z_std_sg`` (`model_joint.py:84-85`), ``z_sg``
(`model_joint.py:89`), ``generated_spatial`` (`model_joint.py:121`),
``generated_node_feat`` (`model_joint.py:144`).
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, Optional

import numpy as np
import torch

from . import _lib
from .config import SNDConfig
from .data import GraphBatch, SGBatch, locality_order, row_tiles, window_plan
from .params import flat_layout, init_blocks

DTYPES = {"f32": 0, "fp32": 0, "bf16": 1}
TAIL = 64  # floats after the parameters in the gradient buffer (loss terms for the all-reduce)
WINDOW_MAX_BETA = 352  # the window SpMM's ring bound (spmm_win_max_beta)


def c_config(cfg: SNDConfig, dtype: str) -> _lib.Config:
    s1, s2, s3 = cfg.s_d_channel
    n1, n2 = cfg.n_d_channel
    sg = cfg.topology == "sgjoint"
    sgh = [int(v) for h in cfg.sg_conv_hidden for v in h] if sg else [0] * 6
    if sg and len(sgh) != 6:
        raise ValueError("sgjoint: sg_conv_hidden must hold two layers of three widths")
    return _lib.Config(cfg.n_nodes, cfg.f_in, cfg.num_feature, cfg.spatial_dim,
                       cfg.g_conv_hidden[0], cfg.g_conv_hidden[1], cfg.g_hidden_size,
                       cfg.latent, s1, s2, s3, n1, n2, cfg.beta, cfg.pos_weight, cfg.norm,
                       DTYPES[dtype], _lib.TOPOLOGY[cfg.topology], cfg.node_h_size,
                       cfg.sampling_num if sg else 0, (C.c_int * 6)(*sgh))


class DeviceTiles:
    """data.RowTiles resident in HBM (snd_row_tiles_t)."""

    def __init__(self, rt, device="cuda"):
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)
        self.rows, self.trp, self.ucol = t(rt.rows), t(rt.trp), t(rt.ucol)
        self.lcol = t(rt.lcol.view(np.int16))
        self.tile_rows, self.ustride = rt.tile_rows, rt.ustride

    def c_struct(self) -> _lib.RowTiles:
        p = _lib.ptr
        return _lib.RowTiles(p(self.rows), p(self.trp), p(self.lcol), p(self.ucol), self.tile_rows,
                             self.ustride)


class DeviceBatch:
    """A GraphBatch resident in HBM (the feed dict of `main.py:327-329`)."""

    def __init__(self, batch: GraphBatch, device="cuda", locality: bool = True, tile_rows: int = 64,
                 window: bool = True):
        """locality: upload the per-graph RCM row schedule of the gather kernels
        (data.locality_order); results do not depend on it.  tile_rows > 0 (with
        locality) also uploads the SpMM row tiles over that schedule
        (data.row_tiles, data.default_tile_rows); bit-identical results.  window
        (with locality): the window SpMM's plan over the schedule (data.window_plan),
        used by the step's width-64 backward SpMM when its beta fits the ring."""
        t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a)).to(device=device, dtype=dt)
        self.sg = isinstance(batch, SGBatch)
        if self.sg:   # spatial-graph encoder: its trees and rel; the gather schedules do not apply
            locality = False
            tr = batch.tree_rowptr.astype(np.int64)
            rows = np.repeat(np.arange(len(tr) - 1), np.diff(tr))
            key = rows * len(tr) + batch.tree_colidx
            if not np.array_equal(np.sort(key), np.sort(batch.tree_colidx.astype(np.int64) * len(tr) + rows)):
                raise ValueError("spanning trees must be symmetric (input_data.py:31-37)")
            self.tree_rowptr = t(batch.tree_rowptr, torch.int32)
            self.tree_colidx = t(batch.tree_colidx if batch.tree_colidx.size else np.zeros(1), torch.int32)
            self.rel = t(batch.rel, torch.float32)
        self.n_graphs = batch.n_graphs
        self.n_nodes = batch.n_nodes
        self.nnz = batch.nnz
        self.rowptr = t(batch.rowptr, torch.int32)
        self.colidx = t(batch.colidx, torch.int32) if batch.nnz else torch.zeros(1, dtype=torch.int32, device=device)
        self.features = t(batch.features, torch.float32)
        self.feature_truth = t(batch.feature_truth, torch.float32)
        self.spatial_truth = t(batch.spatial_truth, torch.float32)
        order = locality_order(batch) if locality and batch.nnz else None
        self.row_order = t(order, torch.int32) if order is not None else None
        self.tiles = None
        if order is not None and tile_rows > 0:
            self.tiles = DeviceTiles(row_tiles(batch, order, tile_rows), device)
        self.window = None
        if order is not None and window:
            try:
                wp = window_plan(batch, order)
            except ValueError:        # a degree past the plan's 6-bit field: no window plan
                wp = None
            if wp is not None and (wp.beta + 7) // 8 * 8 <= WINDOW_MAX_BETA:
                t8 = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)
                self.window = (t8(wp.meta), t8(wp.slots.view(np.int16)), t8(wp.rows), t8(wp.order), wp.beta)
        self.host = batch

    def c_struct(self) -> _lib.Batch:
        p = _lib.ptr
        tl = self.tiles.c_struct() if self.tiles else _lib.RowTiles()
        w = self.window
        wp = _lib.WindowPlan(p(w[0]), p(w[1]), p(w[2]), p(w[3]), w[4]) if w else _lib.WindowPlan(None, None, None, None, -1)
        sg = (p(self.tree_rowptr), p(self.tree_colidx), p(self.rel)) if self.sg else (None, None, None)
        return _lib.Batch(p(self.rowptr), p(self.colidx), p(self.features),
                          p(self.feature_truth), p(self.spatial_truth), p(self.row_order), tl, wp, *sg)


class SGCNModelVAE:
    """Plan + flat parameters of the SND-VAE on one GPU (either topology)."""

    def __init__(self, cfg: SNDConfig, n_graphs: int, dtype: str = "bf16",
                 device="cuda", seed: int = 0, blocks: Optional[Dict[str, np.ndarray]] = None):
        if not torch.cuda.is_available():
            raise _lib.SNDError("SGCNModelVAE needs a ROCm GPU (no CPU fallback)")
        L = _lib.lib()
        self.cfg, self.n_graphs, self.dtype, self.device = cfg, n_graphs, dtype, device
        self._cfg_c = c_config(cfg, dtype)
        h = C.c_void_p()
        _lib.check(L.snd_plan_create(C.byref(self._cfg_c), n_graphs, C.byref(h)), "snd_plan_create")
        self.plan = h
        self.param_count = int(L.snd_plan_param_count(h))
        self.layout = flat_layout(cfg)
        self._check_layout()
        self.params = torch.zeros(self.param_count + TAIL, dtype=torch.float32, device=device)
        ws = int(L.snd_plan_workspace_bytes(h))
        self.workspace = torch.zeros(ws, dtype=torch.uint8, device=device)
        self.load_blocks(blocks if blocks is not None else init_blocks(cfg, seed))

    def _check_layout(self):
        L = _lib.lib()
        nb = L.snd_plan_num_blocks(self.plan)
        names = list(self.layout.shapes)
        if nb != len(names) or self.layout.total != self.param_count:
            raise _lib.SNDError("flat layout mismatch between params.py and libsndvae")
        for i in range(nb):
            nm, off, n = C.c_char_p(), C.c_longlong(), C.c_longlong()
            _lib.check(L.snd_plan_param_block(self.plan, i, C.byref(nm), C.byref(off), C.byref(n)))
            k = names[i]
            if (nm.value.decode() != k or off.value != self.layout.offsets[k]
                    or n.value != self.layout.numel(k)):
                raise _lib.SNDError(f"param block {i} mismatch: {nm.value} vs {k}")

    def __del__(self):
        try:
            if getattr(self, "plan", None):
                _lib.lib().snd_plan_destroy(self.plan)
                self.plan = None
        except Exception:
            pass

    # ---- parameters
    def load_blocks(self, blocks: Dict[str, np.ndarray]):
        flat = self.layout.pack(blocks, np.float32)
        self.params[:self.param_count].copy_(torch.from_numpy(flat))

    def blocks(self) -> Dict[str, np.ndarray]:
        return self.layout.unpack(self.params[:self.param_count].double().cpu().numpy())

    def set_option(self, name: str, value: int) -> bool:
        """A plan option (snd_plan_set_option): True when it is in effect for this plan.
        "conc_decoder": the fused decoder on a side stream beside zz^T (small batches)."""
        r = _lib.lib().snd_plan_set_option(self.plan, name.encode(), int(value))
        if r < 0:
            _lib.check(r, "snd_plan_set_option")
        return r == 1

    # ---- workspace views (intermediates of the last step)
    def buffer(self, name: str, dtype=torch.float32, shape=None) -> torch.Tensor:
        off, n = C.c_longlong(), C.c_longlong()
        _lib.check(_lib.lib().snd_plan_buffer(self.plan, name.encode(), C.byref(off), C.byref(n)),
                   "snd_plan_buffer")
        es = torch.tensor([], dtype=dtype).element_size()
        t = self.workspace[off.value:off.value + n.value * es].view(dtype)
        return t.view(*shape) if shape is not None else t

    def _rows(self, name, width, per_graph=False):
        rows = self.head_rows if per_graph else self.n_graphs * self.cfg.n_nodes
        return self.buffer(name)[:rows * width].view(rows, width)

    @property
    def _graph_latent(self):
        return self.cfg.topology != "tscale"

    @property
    def head_rows(self) -> int:
        """Rows of mu / log-std / z: B*N (node latent), B (graph latent), B*S (sgjoint:
        one latent per spanning-tree copy, model.py:148-151)."""
        c = self.cfg
        if c.topology == "tscale":
            return self.n_graphs * c.n_nodes
        return self.n_graphs * (c.sampling_num if c.topology == "sgjoint" else 1)

    @property
    def z_mean_sg(self):
        """[B, L] (graph latent), [B*S, L] (sgjoint) or [B*N, L] (node latent), model_joint.py:84."""
        return self._rows("MS", 2 * self.cfg.latent, self._graph_latent)[:, :self.cfg.latent]

    @property
    def z_std_sg(self):
        return self._rows("MS", 2 * self.cfg.latent, self._graph_latent)[:, self.cfg.latent:]

    @property
    def z_sg(self):
        """z (model_joint.py:89)."""
        if self._graph_latent:
            return self._rows("ZL", self.cfg.latent, True)
        return self._rows("Z", self.cfg.latent)

    @property
    def joint_h(self):
        """Decoder input J [B*N, node_h] (model_joint.py:97; == z for the node latent)."""
        return self._rows("Z", self.cfg.node_h_size)

    @property
    def generated_spatial(self):
        return self._rows("SHAT", self.cfg.spatial_dim)

    @property
    def generated_node_feat(self):
        return self._rows("XHAT", self.cfg.num_feature)

    # ---- evaluation / sampling (snd_generate)
    def generate(self, batch: Optional[DeviceBatch] = None, mode: str = "mean",
                 z: Optional[torch.Tensor] = None, eps: Optional[torch.Tensor] = None,
                 seed: int = 0, step: int = 0, want_adj: bool = True, stream=None) -> dict:
        """Forward-only decode (`main.py:358-469`, `model.py:163-169`).

        mode: "mean" (z = z_mean, reconstruction), "sample" (z = mu + eps e^s as
        in training), "prior" (z ~ N(0, 1), get_random_z) or "given" (``z``).
        ``eps``: injected normals [RH, L]; None draws them on the device from
        Philox at (seed, step).  Returns generated_adj (uint8 [B, N, N]),
        generated_spatial [B*N, 2], generated_node_feat [B*N, F], z, and
        z_mean / z_std for the encoding modes (all fresh tensors).
        """
        L = _lib.lib()
        m = _lib.GEN_MODES[mode]
        if mode in ("mean", "sample") and batch is None:
            raise ValueError(f"mode {mode!r} encodes a batch")
        src = z if mode == "given" else eps
        if mode == "given" and z is None:
            raise ValueError("mode 'given' needs z")
        if src is not None:
            rh = self.n_graphs if self._graph_latent else self.n_graphs * self.cfg.n_nodes
            src = src.to(device=self.device, dtype=torch.float32).contiguous()
            if tuple(src.shape) != (rh, self.cfg.latent):
                raise ValueError(f"z/eps must be [{rh}, {self.cfg.latent}], got {tuple(src.shape)}")
        n = self.cfg.n_nodes
        adj = (torch.empty(self.n_graphs, n, n, dtype=torch.uint8, device=self.device)
               if want_adj else None)
        step_t = torch.full((1,), step, dtype=torch.int32, device=self.device)
        bc = batch.c_struct() if batch is not None else None
        _lib.check(L.snd_generate(self.plan, C.byref(bc) if bc is not None else None,
                                  _lib.ptr(self.params), _lib.ptr(self.workspace), m,
                                  _lib.ptr(src), seed, _lib.ptr(step_t), _lib.ptr(adj),
                                  _lib.stream_ptr(stream)), "snd_generate")
        out = {"generated_adj": adj,
               "generated_spatial": self.generated_spatial.clone(),
               "generated_node_feat": self.generated_node_feat.clone(),
               "z": self.z_sg.clone()}
        if mode in ("mean", "sample"):
            out["z_mean"] = self.z_mean_sg.clone()
            out["z_std"] = self.z_std_sg.clone()
        return out


def adj_accuracy(gen_adj: torch.Tensor, batch: DeviceBatch) -> float:
    """`main.py:334`: mean over B*N*N of (generated_adj == adj_truth), from the CSR."""
    B, n = batch.n_graphs, batch.n_nodes
    total = B * n * n
    ones = int(gen_adj.sum(dtype=torch.int64).item())
    if batch.nnz == 0:
        return (total - ones) / total
    rows = torch.repeat_interleave(torch.arange(B * n, device=gen_adj.device),
                                   torch.diff(batch.rowptr.long()))
    flat = rows * n + batch.colidx[:batch.nnz].long() % n
    hits = int(gen_adj.view(-1)[flat].sum(dtype=torch.int64).item())
    return (total - batch.nnz - ones + 2 * hits) / total
