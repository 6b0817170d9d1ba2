"""Spatial-graph batches: synthetic random-geometric graphs and CSR ingest.

Reference behaviour mirrored here:

* The reference feeds a dense ``adj_truth`` [B, N, N] float32 placeholder
  (`main.py:257`), built by ``load_data_syn`` from scipy sparse matrices with
  the diagonal zeroed and symmetry asserted (`input_data.py:62-67`).
* Index order is row-major, the order of ``np.where`` (`input_data.py:72`) and
  of ``sparse_to_tuple`` (`preprocessing.py:7-13`).

The MI355X path never materialises the dense N x N adjacency: a batch of B
graphs is one block-diagonal CSR (int32 ``rowptr`` [B*N+1], ``colidx`` [nnz],
columns sorted within each row, column ids global = b*N + j).  Node data is
row-major [B*N, width] float32.

The reference datasets are not shipped, so benchmarks and tests use seeded
random-geometric graphs: positions U[0,1)^2, radius
r = sqrt(kbar / (pi N)), edges from ``cKDTree.query_pairs``.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np
from typing import NamedTuple

from .config import SNDConfig


@dataclass
class GraphBatch:
    """Host-side batch of B spatial graphs with N nodes each.

    ``rowptr``/``colidx`` form the block-diagonal CSR.  ``features`` is the
    encoder input X = [x_feat || S] when ``cfg.encoder_coords`` (decision iii)
    or x_feat alone; ``feature_truth`` and ``spatial_truth`` are the decoder
    targets (`main.py:258-259`).
    """
    n_graphs: int
    n_nodes: int
    rowptr: np.ndarray          # int32 [B*N + 1]
    colidx: np.ndarray          # int32 [nnz]
    features: np.ndarray        # float32 [B*N, f_in]
    feature_truth: np.ndarray   # float32 [B*N, num_feature]
    spatial_truth: np.ndarray   # float32 [B*N, spatial_dim]

    @property
    def nnz(self) -> int:
        return int(self.colidx.shape[0])

    def graph_nnz(self) -> np.ndarray:
        n = self.n_nodes
        rp = self.rowptr.astype(np.int64)
        return rp[n::n] - rp[:-1:n]

    def sparse_adj(self, b: int):
        """scipy CSR [N, N] adjacency of graph b (local column ids; any N)."""
        import scipy.sparse as sp
        n = self.n_nodes
        lo = b * n
        rp = self.rowptr[lo:lo + n + 1].astype(np.int64) - int(self.rowptr[lo])
        cols = self.colidx[int(self.rowptr[lo]):int(self.rowptr[lo + n])].astype(np.int64) - lo
        return sp.csr_matrix((np.ones(len(cols)), cols, rp), shape=(n, n))

    def dense_adj(self, b: int) -> np.ndarray:
        """Dense [N, N] adjacency of graph b (small N only; tests)."""
        n = self.n_nodes
        a = np.zeros((n, n), np.float32)
        lo = b * n
        for i in range(n):
            s, e = self.rowptr[lo + i], self.rowptr[lo + i + 1]
            a[i, self.colidx[s:e] - lo] = 1.0
        return a


@dataclass
class SGBatch(GraphBatch):
    """A batch for the spatial-graph encoder (config topology 'sgjoint').

    The GraphBatch fields hold the B graphs' adj_truth CSR and decoder targets, and
    ``features`` the encoder input of every spanning-tree copy: [B*S*N, num_feature],
    copy c = b*S + s holding graph b's node features.  ``tree_rowptr`` /
    ``tree_colidx``: the copies' spanning trees as one symmetric block-diagonal CSR
    over B*S*N rows (input_data.py:76-83); ``rel`` [B*S, N, N] float32 the copies'
    pairwise distances (2D_rel.npy / 600, input_data.py:59).  The reference feeds
    features and rel tiled sample-major (np.tile, main.py:307-309) against graph-major
    trees; the copies here keep each graph's own data."""
    sampling_num: int = 1
    tree_rowptr: np.ndarray = None
    tree_colidx: np.ndarray = None
    rel: np.ndarray = None


def pairwise_rel(pos: np.ndarray) -> np.ndarray:
    """cal_rel_dist (input_data.py:145-151): Euclidean distances between nodes."""
    d = pos[:, None, :] - pos[None, :, :]
    return np.sqrt((d * d).sum(-1))


def make_sg_batch(base: GraphBatch, trees: Sequence[Sequence[np.ndarray]], rel: np.ndarray,
                  num_feature: int) -> SGBatch:
    """SGBatch from a GraphBatch (targets, adj_truth), per graph S spanning-tree edge
    arrays [2, 2k] (input_data.spanning_tree_edges) and rel [B, N, N]."""
    B, n = base.n_graphs, base.n_nodes
    S = len(trees[0])
    if any(len(t) != S for t in trees) or rel.shape != (B, n, n):
        raise ValueError("make_sg_batch: every graph needs S trees and rel [B, N, N]")
    parts = []
    for b in range(B):
        for e in trees[b]:
            parts.append(csr_from_pairs(n, np.asarray(e, np.int64).T))
    trp, tci = stack_csr(parts, n)
    x = base.feature_truth.reshape(B, n, -1)[:, :, :num_feature]
    xc = np.repeat(x, S, axis=0).reshape(B * S * n, -1)
    relc = np.repeat(np.asarray(rel, np.float32), S, axis=0)
    return SGBatch(B, n, base.rowptr, base.colidx, np.ascontiguousarray(xc, np.float32),
                   base.feature_truth, base.spatial_truth, S, trp, tci, np.ascontiguousarray(relc))


def sgjoint_batch(cfg: SNDConfig, n_graphs: int, seed: Optional[int] = None) -> SGBatch:
    """B seeded RGG graphs with cfg.sampling_num scipy-MST spanning trees each under
    U[1,2) edge weights (input_data.py:18-38, np.random.RandomState(seed)) and rel
    from the node positions."""
    from .input_data import spanning_tree_edges
    seed = cfg.seed if seed is None else seed
    base = synthetic_batch(cfg, n_graphs, seed=seed)
    n = cfg.n_nodes
    rs = np.random.RandomState(seed)
    trees, rel = [], []
    for b in range(n_graphs):
        lo = b * n
        rp = base.rowptr[lo:lo + n + 1].astype(np.int64) - int(base.rowptr[lo])
        cols = base.colidx[int(base.rowptr[lo]):int(base.rowptr[lo + n])].astype(np.int64) - lo
        raw = np.stack([np.repeat(np.arange(n), np.diff(rp)), cols], 1)
        trees.append([spanning_tree_edges(raw, n, rs) for _ in range(cfg.sampling_num)])
        rel.append(pairwise_rel(base.spatial_truth[lo:lo + n].astype(np.float64)))
    return make_sg_batch(base, trees, np.stack(rel).astype(np.float32), cfg.num_feature)


def rgg_edges(n: int, kbar: float, rng: np.random.Generator):
    """Random geometric graph: returns (positions [n,2], i<j pair array)."""
    from scipy.spatial import cKDTree
    pos = rng.random((n, 2))
    r = np.sqrt(kbar / (np.pi * n))
    pairs = cKDTree(pos).query_pairs(r, output_type="ndarray")
    return pos, pairs


def csr_from_pairs(n: int, pairs: np.ndarray, offset: int = 0):
    """Symmetric CSR (sorted columns, no diagonal) from undirected pairs.

    Same entry order as ``np.where(dense)`` (`input_data.py:72`).
    """
    pairs = np.asarray(pairs, dtype=np.int64).reshape(-1, 2)
    keep = pairs[:, 0] != pairs[:, 1]               # diag zeroed (input_data.py:65)
    pairs = pairs[keep]
    rows = np.concatenate([pairs[:, 0], pairs[:, 1]])
    cols = np.concatenate([pairs[:, 1], pairs[:, 0]])
    key = np.unique(rows * n + cols)                 # row-major order, dedup
    rows, cols = key // n, key % n
    counts = np.bincount(rows, minlength=n)
    rowptr = np.zeros(n + 1, np.int64)
    np.cumsum(counts, out=rowptr[1:])
    return rowptr, (cols + offset)


def csr_from_dense(adj: np.ndarray):
    """CSR of one dense [N, N] 0/1 matrix in np.where order (host reference)."""
    adj = np.asarray(adj)
    if adj.shape[0] != adj.shape[1]:
        raise ValueError("adjacency must be square")
    if not np.array_equal(adj, adj.T):
        raise ValueError("adjacency must be symmetric (input_data.py:67)")
    a = adj.copy()
    np.fill_diagonal(a, 0)
    rows, cols = np.where(a)
    counts = np.bincount(rows, minlength=a.shape[0])
    rowptr = np.zeros(a.shape[0] + 1, np.int64)
    np.cumsum(counts, out=rowptr[1:])
    return rowptr, cols


def stack_csr(parts: Sequence, n: int):
    """Block-diagonal concatenation of per-graph (rowptr, local cols)."""
    rowptrs, cols = [], []
    base = 0
    for b, (rp, c) in enumerate(parts):
        rp = np.asarray(rp, np.int64)
        rowptrs.append(rp[:-1] + base)
        cols.append(np.asarray(c, np.int64) + b * n)
        base += int(rp[-1])
    rowptr = np.concatenate(rowptrs + [np.array([base], np.int64)])
    colidx = np.concatenate(cols) if cols else np.zeros(0, np.int64)
    if base >= 2 ** 31:
        raise ValueError("nnz exceeds int32 CSR range")
    return rowptr.astype(np.int32), colidx.astype(np.int32)


def synthetic_batch(cfg: SNDConfig, n_graphs: int, seed: Optional[int] = None,
                    kbar: Optional[float] = None) -> GraphBatch:
    """B seeded RGG graphs (graph b uses default_rng(seed + b))."""
    seed = cfg.seed if seed is None else seed
    kbar = cfg.mean_degree if kbar is None else kbar
    n = cfg.n_nodes
    parts: List = []
    feats, xs, ss = [], [], []
    for b in range(n_graphs):
        rng = np.random.default_rng(seed + b)
        pos, pairs = rgg_edges(n, kbar, rng)
        x = rng.random((n, cfg.num_feature))            # like node / 120 in [0,1)
        parts.append(csr_from_pairs(n, pairs))
        s = pos[:, :cfg.spatial_dim]                     # like geometry / 600
        xs.append(x)
        ss.append(s)
        feats.append(np.concatenate([x, s], 1) if cfg.encoder_coords else x)
    rowptr, colidx = stack_csr(parts, n)
    return GraphBatch(n_graphs, n, rowptr, colidx,
                      np.ascontiguousarray(np.concatenate(feats), np.float32),
                      np.ascontiguousarray(np.concatenate(xs), np.float32),
                      np.ascontiguousarray(np.concatenate(ss), np.float32))


def batch_from_dense(cfg: SNDConfig, adj: np.ndarray, feature: np.ndarray,
                     spatial: np.ndarray) -> GraphBatch:
    """Ingest the reference feed format (`main.py:253-264`) into a GraphBatch.

    adj [B,N,N] (dense adj_truth), feature [B,N,num_feature], spatial [B,N,2].
    """
    adj = np.asarray(adj)
    b, n, _ = adj.shape
    rowptr, colidx = stack_csr([csr_from_dense(adj[i]) for i in range(b)], n)
    x = np.asarray(feature, np.float32).reshape(b * n, -1)
    s = np.asarray(spatial, np.float32).reshape(b * n, -1)
    f = np.concatenate([x, s], 1) if cfg.encoder_coords else x
    return GraphBatch(b, n, rowptr, colidx, np.ascontiguousarray(f, np.float32),
                      np.ascontiguousarray(x), np.ascontiguousarray(s))


def locality_order(batch: GraphBatch) -> np.ndarray:
    """Processing order of the rows for the gather kernels (int32 [B*N]).

    Per graph, the reverse Cuthill-McKee permutation of its adjacency: rows that
    are consecutive in this order are graph neighbours, so the neighbour rows a
    workgroup gathers overlap and hit in L1 (32 consecutive rows of a seed-0
    N=4096 RGG share each gathered row ~4x, against ~1.06x in generator order).
    It is a schedule, not a relabelling: outputs stay at their original rows and
    the node order the conv1d decoders see (decision iv) is untouched.
    """
    import scipy.sparse as sp
    from scipy.sparse.csgraph import reverse_cuthill_mckee
    n, B = batch.n_nodes, batch.n_graphs
    out = np.empty(B * n, np.int32)
    rp = batch.rowptr.astype(np.int64)
    for b in range(B):
        lo = b * n
        s, e = rp[lo], rp[lo + n]
        a = sp.csr_matrix((np.ones(e - s, np.int8), batch.colidx[s:e] - lo, rp[lo:lo + n + 1] - s),
                          shape=(n, n))
        out[lo:lo + n] = reverse_cuthill_mckee(a, symmetric_mode=True).astype(np.int32) + lo
    return out


def default_tile_rows(width: int) -> int:
    """Rows per SpMM tile: 64.  The tile's neighbour set of an RCM-ordered RGG
    (<= ~310 rows at N = 4096 and 16384) then fits the 319-row fp32 LDS image
    (80 KB at width 64, two workgroups per CU; 160 KB at width 128)."""
    return 64


@dataclass
class RowTiles:
    """Host image of snd_row_tiles_t (see include/snd_vae.h)."""
    rows: np.ndarray     # int32 [R]      tile slot -> row (by degree inside a tile)
    trp: np.ndarray      # int32 [R+1]    slot-order row pointers into lcol
    lcol: np.ndarray     # uint16 [nnz]   local neighbour ids, slot order
    ucol: np.ndarray     # int32 [T*ustride] tile sets, padded with -1
    tile_rows: int
    ustride: int


def row_tiles(batch: GraphBatch, order: Optional[np.ndarray], tile_rows: int) -> RowTiles:
    """Row tiles of the bf16 SpMM over the schedule ``order`` (None = natural).

    Built on the host by the library's snd_spmm_tile_plan (plain C++, no GPU)
    once per batch."""
    import ctypes

    from . import _lib
    L = _lib.lib()
    R = batch.n_graphs * batch.n_nodes
    rp = np.ascontiguousarray(batch.rowptr, np.int32)
    ci = np.ascontiguousarray(batch.colidx, np.int32)
    od = None if order is None else np.ascontiguousarray(order, np.int32)
    P = lambda a: None if a is None else a.ctypes.data
    ust = ctypes.c_int(0)
    n = L.snd_spmm_tile_plan(P(rp), P(ci), R, P(od), tile_rows, None, None, None, None, ctypes.byref(ust))
    if n < 0:
        raise _lib.SNDError(f"snd_spmm_tile_plan failed ({n}): {_lib.last_error()}")
    rows = np.zeros(max(R, 1), np.int32)
    trp = np.zeros(R + 1, np.int32)
    lcol = np.zeros(max(len(ci), 1), np.uint16)
    ucol = np.zeros(max(n, 1), np.int32)
    n2 = L.snd_spmm_tile_plan(P(rp), P(ci), R, P(od), tile_rows, P(rows), P(trp), P(lcol), P(ucol),
                              ctypes.byref(ust))
    if n2 != n:
        raise _lib.SNDError(f"snd_spmm_tile_plan failed ({n2}): {_lib.last_error()}")
    return RowTiles(rows, trp, lcol, ucol, tile_rows, int(ust.value))


class WindowPlan(NamedTuple):
    """Sliding-window SpMM plan (snd_csr_spmm_bf16_window), one per batch."""
    meta: np.ndarray     # int32 [R]: (start8 << 6) | degree, rows by degree inside each 128-position block
    slots: np.ndarray    # uint16 [8 * sum(ceil8(degree))]: ring slot (position % 1096) per neighbour
    rows: np.ndarray     # int32 [R]: the row of each meta entry
    order: np.ndarray    # int32 [R]: the row at each position (the schedule)
    beta: int            # largest |position(neighbour) - position(row)|
    max_degree: int


def window_plan(batch: GraphBatch, order: np.ndarray, ring: int = 1096) -> WindowPlan:
    """Position-ordered neighbour lists for the window SpMM.

    Position q (per graph, in the schedule ``order``, e.g. locality_order) holds
    row order[q]; its neighbours (colidx order, so the kernel's fp32 sums are the
    register kernel's) are stored as ring slots (neighbour position mod ``ring``)
    in a list padded to 8 entries.  beta bounds |position distance| over all
    edges; the kernel needs ceil8(beta) <= 352 (snd_csr_spmm_bf16_window).
    meta / rows list each aligned block of 128 positions (one kernel step) by
    degree, descending (ties by position): a wavefront's 8 rows then have
    similar lengths, and the SIMD's four wavefronts together about the mean.
    """
    n, B = batch.n_nodes, batch.n_graphs
    R = n * B
    order = np.ascontiguousarray(order, np.int64)
    rp = batch.rowptr.astype(np.int64)
    ci = batch.colidx.astype(np.int64)
    pos = np.empty(R, np.int64)
    pos[order] = np.arange(R) % n                 # graph-local position of every row
    deg = np.diff(rp)[order]                      # degree of the row at each position
    if deg.size and deg.max() > 63:
        raise ValueError("window_plan: degree > 63 does not fit the metadata word")
    # per aligned 128-position block of each graph: degree descending, ties by position
    q = np.arange(R)
    blk = (q // n) * ((n + 127) // 128) + (q % n) // 128
    srt = np.lexsort((q, -deg, blk))
    # a wavefront sums the 8 rows of one sorted group together up to their largest
    # degree: every list is padded (with the ring's zero row, slot ``ring``) to its
    # group's largest degree (at most the 32 entries the kernel stages), in 8s
    rank = np.empty(R, np.int64)
    bs = blk[srt]
    first = np.searchsorted(bs, bs, side="left")          # sorted index of the block's first row
    rank[srt] = np.arange(R) - first                       # rank of a position inside its block
    gfirst = np.empty(R, np.int64)
    gfirst[srt] = first + (rank[srt] // 8) * 8             # sorted index of its group's first row
    gmax = deg[srt][gfirst] if R else deg
    pad = (np.maximum(deg, np.minimum(gmax, 32)) + 7) // 8 * 8
    start = np.zeros(R + 1, np.int64)
    np.cumsum(pad, out=start[1:])
    if start[-1] // 8 >= (1 << 25):
        raise ValueError("window_plan: slot lists exceed the 25-bit offset")
    nnz = int(deg.sum())
    # + 24: the kernel DMAs 32 entries of every row's list (8 rows x 4 lanes x 16 B), so
    # the last list (8 entries) is followed by 24 padding entries inside the array
    slots = np.full(max(int(start[-1]), 8) + 24, ring, np.uint16)
    beta = 0
    if nnz:
        excl = np.cumsum(deg) - deg               # exclusive prefix of degrees
        run = np.arange(nnz) - np.repeat(excl, deg)   # index within the row's list
        src = np.repeat(rp[order], deg) + run     # colidx entries in position order
        npos = pos[ci[src]]
        qpos = np.repeat(np.arange(R) % n, deg)
        beta = int(np.abs(npos - qpos).max())
        slots[np.repeat(start[:-1], deg) + run] = (npos % ring).astype(np.uint16)
    meta = ((start[:-1] // 8) << 6 | deg).astype(np.int32)
    return WindowPlan(meta[srt], slots, order[srt].astype(np.int32), order.astype(np.int32), beta,
                      int(deg.max()) if deg.size else 0)


def shard(batch: GraphBatch, rank: int, world: int) -> GraphBatch:
    """Contiguous equal shard of the global batch for DP rank ``rank``.

    SURVEY.md §8e: B/world graphs per rank; every loss term is a per-graph
    mean, so the global gradient is the mean of the rank gradients.
    """
    if batch.n_graphs % world:
        raise ValueError("global batch must divide evenly over ranks")
    per = batch.n_graphs // world
    n = batch.n_nodes
    lo, hi = rank * per * n, (rank + 1) * per * n
    rp = batch.rowptr[lo:hi + 1].astype(np.int64)
    cols = batch.colidx[rp[0]:rp[-1]].astype(np.int64) - lo
    return GraphBatch(per, n, (rp - rp[0]).astype(np.int32), cols.astype(np.int32),
                      batch.features[lo:hi], batch.feature_truth[lo:hi],
                      batch.spatial_truth[lo:hi])
