"""Reference on-disk dataset ingest.

Mirror of ``load_data_syn`` (`input_data.py:54-142`) and the spanning-tree
sampler it calls (`input_data.py:18-38`), producing the host arrays the
reference returns and, from them, block-diagonal CSR ``GraphBatch`` objects
for the device path.

Directory layout (``<path>/<split>/``, `input_data.py:56-60,97-101`)::

    2D_adj.npy        per-graph adjacency: object array of scipy sparse
                      matrices in the reference (a pickle), or a dense
                      numeric [G, N, N] array
    2D_adj.npz        (this package's pickle-free alternative) CSR arrays
                      ``indptr`` [G*(N+1)], ``indices`` [nnz], ``graph_nnz`` [G],
                      ``n_nodes`` -- written by :func:`save_adj_npz`
    2D_node.npy       node attributes, divided by 120 on load
    2D_geometry.npy   coordinates, divided by 600 on load
    2D_rel.npy        pairwise distances, divided by 600 (optional here: only
                      the SpatialGraphConvolution encoder reads them)
    2D_prop.npy       generative factors (the test splits read train/'s copy,
                      exactly as `input_data.py:101`)

Semantics kept from the reference:

* each adjacency is densified, its diagonal zeroed and symmetry asserted
  (`input_data.py:62-67`);
* ``sampling_num`` spanning trees per graph, each the scipy minimum spanning
  tree of the edge list under weights ``np.random.random(num_edges) + 1``
  (`input_data.py:18-38,70-83`), symmetrised;
* one ``np.random.shuffle`` of the graph order after the sampling
  (`input_data.py:86-93`), so the permutation depends on the RNG draws of the
  sampler exactly as in the reference.  ``rng`` defaults to the global
  ``np.random`` state (the reference seeds it with ``np.random.seed(1)`` when
  ``FLAGS.seeded``, `main.py:124-125`).

Loading an object-array ``2D_adj.npy`` unpickles the file, so it is refused
unless the caller passes ``allow_pickle=True`` for a dataset it trusts;
:func:`save_adj_npz` converts one into the pickle-free form once.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np

from .config import SNDConfig
from .data import GraphBatch, csr_from_dense, stack_csr

NODE_SCALE = 120.0      # input_data.py:57
COORD_SCALE = 600.0     # input_data.py:58-59
TEST_TYPES = ("test_generation", "test_disentangle", "test_reconstruct", "test")


# ----------------------------------------------------------------------------- adjacency files
def _adj_from_npz(fn: str) -> List[Tuple[np.ndarray, np.ndarray]]:
    z = np.load(fn, allow_pickle=False)
    n = int(z["n_nodes"])
    gn = z["graph_nnz"].astype(np.int64)
    indptr = z["indptr"].astype(np.int64).reshape(len(gn), n + 1)
    indices = z["indices"].astype(np.int64)
    out, base = [], 0
    for g in range(len(gn)):
        out.append((indptr[g], indices[base:base + gn[g]]))
        base += int(gn[g])
    return out


def load_adjacency(split_dir: str, allow_pickle: bool = False) -> Tuple[int, list]:
    """Per-graph adjacency of one split as a list of dense-or-CSR items.

    Returns (n_nodes, items) where each item is either a dense [N, N] array or
    an (indptr, indices) CSR pair.  Prefers the pickle-free ``2D_adj.npz``.
    """
    npz = os.path.join(split_dir, "2D_adj.npz")
    if os.path.exists(npz):
        items = _adj_from_npz(npz)
        n = len(items[0][0]) - 1 if items else 0
        return n, items
    fn = os.path.join(split_dir, "2D_adj.npy")
    try:
        a = np.load(fn, allow_pickle=False, mmap_mode="r")
    except ValueError:
        if not allow_pickle:
            raise ValueError(
                f"{fn} is an object array (pickled scipy matrices, the reference format); "
                "pass allow_pickle=True only for a dataset you trust, or convert it once "
                "with snd_vae_amd.input_data.save_adj_npz") from None
        a = np.load(fn, allow_pickle=True)
    if a.dtype == object:
        items = []
        for m in a:
            m = m.tocsr() if hasattr(m, "tocsr") else np.asarray(m)
            items.append(m)
        n = items[0].shape[0] if items else 0
        return n, items
    if a.ndim != 3 or a.shape[1] != a.shape[2]:
        raise ValueError(f"{fn}: expected [G, N, N], got {a.shape}")
    return a.shape[1], [a[g] for g in range(a.shape[0])]


def _graph_csr(item, n: int) -> Tuple[np.ndarray, np.ndarray]:
    """Diagonal zeroed + symmetry asserted CSR of one graph (`input_data.py:62-67`).

    Entry order is row-major (np.where order, `input_data.py:72`).
    """
    if isinstance(item, tuple):
        indptr, indices = item
        rows = np.repeat(np.arange(n, dtype=np.int64), np.diff(indptr))
        cols = np.asarray(indices, np.int64)
    elif hasattr(item, "tocoo"):
        coo = item.tocoo()
        keep = coo.data != 0
        rows, cols = coo.row[keep].astype(np.int64), coo.col[keep].astype(np.int64)
    else:
        return csr_from_dense(np.asarray(item) != 0)
    keep = rows != cols                               # new_adj[n][i, i] = 0
    key = np.unique(rows[keep] * n + cols[keep])      # row-major, duplicates summed to 1
    r, c = key // n, key % n
    sym = np.unique(c * n + r)
    if not np.array_equal(key, sym):                  # assert new_adj[i,j] == new_adj[j,i]
        raise ValueError("adjacency must be symmetric (input_data.py:67)")
    rowptr = np.zeros(n + 1, np.int64)
    np.cumsum(np.bincount(r, minlength=n), out=rowptr[1:])
    return rowptr, c


def save_adj_npz(fn: str, items: Sequence, n_nodes: int) -> None:
    """Write adjacencies in the pickle-free ``2D_adj.npz`` form."""
    parts = [_graph_csr(it, n_nodes) for it in items]
    np.savez(fn, n_nodes=np.int64(n_nodes),
             graph_nnz=np.array([len(c) for _, c in parts], np.int64),
             indptr=np.concatenate([rp for rp, _ in parts]).astype(np.int64),
             indices=np.concatenate([c for _, c in parts]).astype(np.int32))


# ----------------------------------------------------------------------------- spanning trees
def scipy_spanning_tree(edge_index: np.ndarray, num_nodes: int, num_edges: int,
                        rng=np.random) -> np.ndarray:
    """`input_data.py:18-24`: MST of the edge list under U[1,2) weights; [k, 2] edges."""
    from scipy.sparse import csr_matrix
    from scipy.sparse.csgraph import minimum_spanning_tree
    row, col = edge_index[:, 0], edge_index[:, 1]
    cgraph = csr_matrix((rng.random(num_edges) + 1, (row, col)), shape=(num_nodes, num_nodes))
    tree_row, tree_col = minimum_spanning_tree(cgraph).nonzero()
    return np.concatenate([[tree_row], [tree_col]]).T


def spanning_tree_edges(edges: np.ndarray, num_nodes: int, rng=np.random) -> np.ndarray:
    """`build_spanning_tree_edge(..., 'scipy')` (`input_data.py:26-38`): [2, 2k] undirected."""
    st = scipy_spanning_tree(edges, num_nodes, len(edges), rng).T
    return np.array([np.concatenate([st[0], st[1]]), np.concatenate([st[1], st[0]])])


# ----------------------------------------------------------------------------- the dataset
@dataclass
class SynDataset:
    """What ``load_data_syn`` returns, with adjacency kept sparse.

    ``adj_truth`` holds the per-graph (rowptr, cols) CSR of the dense
    ``new_adj`` [G, N, N]; ``trees[g][s]`` the s-th sampled spanning tree of
    graph g as an edge array [2, 2k] (the reference's ``adj`` [G, S, N, N]).
    """
    node: np.ndarray          # [G, N, num_feature] (/120)
    spatial: np.ndarray       # [G, N, spatial_dim] (/600)
    adj_truth: list           # G x (rowptr int64 [N+1], cols int64 [nnz_g])
    trees: list               # G x sampling_num x int64 [2, 2k]
    rel: Optional[np.ndarray]  # [G, N, N] (/600) or None when absent
    factor: Optional[np.ndarray]
    n_nodes: int

    @property
    def n_graphs(self) -> int:
        return len(self.adj_truth)

    def dense_adj(self, g: int) -> np.ndarray:
        n = self.n_nodes
        a = np.zeros((n, n), np.float32)
        rp, c = self.adj_truth[g]
        a[np.repeat(np.arange(n), np.diff(rp)), c] = 1
        return a

    def dense_trees(self, g: int) -> np.ndarray:
        """[S, N, N] 0/1 spanning-tree adjacencies of graph g (`input_data.py:80-82`)."""
        n = self.n_nodes
        out = np.zeros((len(self.trees[g]), n, n), np.float32)
        for s, e in enumerate(self.trees[g]):
            out[s, e[0], e[1]] = 1
        return out

    def batch(self, cfg: SNDConfig, graphs: Sequence[int]) -> GraphBatch:
        """GraphBatch of the given graphs (the `main.py:316-323` slice, feed order)."""
        n = self.n_nodes
        if n != cfg.n_nodes:
            raise ValueError(f"dataset has N={n}, config N={cfg.n_nodes}")
        graphs = list(graphs)
        rowptr, colidx = stack_csr([self.adj_truth[g] for g in graphs], n)
        x = self.node[graphs].reshape(len(graphs) * n, -1).astype(np.float32)
        s = self.spatial[graphs].reshape(len(graphs) * n, -1).astype(np.float32)
        if x.shape[1] != cfg.num_feature or s.shape[1] != cfg.spatial_dim:
            raise ValueError(f"feature widths {x.shape[1]}/{s.shape[1]} != config "
                             f"{cfg.num_feature}/{cfg.spatial_dim}")
        f = np.concatenate([x, s], 1) if cfg.encoder_coords else x
        return GraphBatch(len(graphs), n, rowptr, colidx, np.ascontiguousarray(f, np.float32),
                          np.ascontiguousarray(x), np.ascontiguousarray(s))


def class_balance(n_matrices: int, n_nodes: int, n_ones: int) -> Tuple[float, float]:
    """(pos_weight, norm) of `main.py:246-247` for ``n_matrices`` N x N 0/1 matrices
    holding ``n_ones`` ones in all:
        pos_weight = (M N^2 - sum) / sum,  norm = M N^2 / ((M N^2 - sum) 2)."""
    total = float(n_matrices) * n_nodes * n_nodes
    if n_ones <= 0 or n_ones >= total:
        raise ValueError("class balance needs both zero and nonzero adjacency entries")
    return (total - n_ones) / n_ones, total / ((total - n_ones) * 2.0)


def dataset_class_balance(ds: "SynDataset") -> Tuple[float, float]:
    """`main.py:246-247` over the spanning-tree adjacency ``adj`` [G*S, N, N] that
    `main.py:177` reshapes from load_data_syn (the trees, not adj_truth)."""
    n = ds.n_nodes
    mats = ones = 0
    for g in range(ds.n_graphs):
        for e in ds.trees[g]:
            mats += 1
            ones += len(np.unique(np.asarray(e[0], np.int64) * n + np.asarray(e[1], np.int64)))
    if mats == 0:
        raise ValueError("the dataset holds no spanning trees (sampling_num=0)")
    return class_balance(mats, n, ones)


def dataset_sg_batch(ds: "SynDataset", cfg: SNDConfig, graphs: Sequence[int]):
    """The SGBatch of the given graphs (main.py:316-323 slices of adj / features /
    rel and the truths): their sampled spanning trees and rel (input_data.py:59,76-83)."""
    from .data import make_sg_batch
    if ds.rel is None:
        raise ValueError("the spatial-graph encoder needs 2D_rel.npy (load_rel=True)")
    graphs = list(graphs)
    if any(len(ds.trees[g]) != cfg.sampling_num for g in graphs):
        raise ValueError(f"dataset sampled {len(ds.trees[graphs[0]])} trees, config sampling_num "
                         f"{cfg.sampling_num}")
    base = ds.batch(cfg, graphs)
    return make_sg_batch(base, [ds.trees[g] for g in graphs], np.asarray(ds.rel[graphs], np.float32),
                         cfg.num_feature)


def load_data_syn(type_: str, path: str, sampling_num: int = 10, num_feature: int = 1,
                  rng=None, allow_pickle: bool = False, shuffle: bool = True,
                  load_rel: bool = True) -> SynDataset:
    """`input_data.py:54-142` for ``type_`` in {'train', 'test*'}.

    ``rng``: object with ``random`` and ``shuffle`` (np.random.RandomState /
    the ``np.random`` module, the default, as in the reference).
    ``sampling_num=0`` skips the spanning trees (the GCN path does not read
    them), which also changes the RNG stream the shuffle sees.
    """
    rng = np.random if rng is None else rng
    if type_ == "train":
        d, factor_dir = os.path.join(path, "train"), os.path.join(path, "train")
    elif type_ in TEST_TYPES:
        d, factor_dir = os.path.join(path, "test"), os.path.join(path, "train")   # input_data.py:101
    else:
        raise ValueError(f"unknown type {type_!r}")
    n, items = load_adjacency(d, allow_pickle)
    node = np.load(os.path.join(d, "2D_node.npy"), allow_pickle=False) / NODE_SCALE
    spatial = np.load(os.path.join(d, "2D_geometry.npy"), allow_pickle=False) / COORD_SCALE
    rel_fn = os.path.join(d, "2D_rel.npy")
    rel = (np.load(rel_fn, allow_pickle=False) / COORD_SCALE
           if load_rel and os.path.exists(rel_fn) else None)
    fac_fn = os.path.join(factor_dir, "2D_prop.npy")
    factor = np.load(fac_fn, allow_pickle=False) if os.path.exists(fac_fn) else None
    G = len(items)
    node = node.reshape(G, n, -1)          # main.py:249 feature.reshape([-1, N, num_features])
    if node.shape[2] != num_feature:
        raise ValueError(f"2D_node.npy has {node.shape[2]} features, expected {num_feature}")
    spatial = spatial.reshape(G, n, -1)
    adj_truth = [_graph_csr(it, n) for it in items]
    trees = []
    for rp, c in adj_truth:
        r = np.repeat(np.arange(n, dtype=np.int64), np.diff(rp))
        raw = np.stack([r, c], 1)                    # np.where order (input_data.py:72-74)
        trees.append([spanning_tree_edges(raw, n, rng) for _ in range(sampling_num)])
    if shuffle:
        index = list(range(G))                       # input_data.py:86-87
        rng.shuffle(index)
        adj_truth = [adj_truth[i] for i in index]
        trees = [trees[i] for i in index]
        node, spatial = node[index], spatial[index]
        rel = rel[index] if rel is not None else None
        factor = factor[index] if factor is not None else None
    return SynDataset(node, spatial, adj_truth, trees, rel, factor, n)


def write_synthetic_dataset(path: str, cfg: SNDConfig, n_graphs: int, seed: int = 0,
                            split: str = "train", adj_format: str = "npz") -> str:
    """Write seeded RGG graphs in the reference directory layout (scaled back
    by 120 / 600 so ``load_data_syn`` recovers the generator's values)."""
    from .data import synthetic_batch
    b = synthetic_batch(cfg.replace(encoder_coords=False), n_graphs, seed=seed)
    n = cfg.n_nodes
    d = os.path.join(path, split)
    os.makedirs(d, exist_ok=True)
    items = [(b.rowptr[g * n:(g + 1) * n + 1].astype(np.int64) - b.rowptr[g * n],
              b.colidx[b.rowptr[g * n]:b.rowptr[(g + 1) * n]].astype(np.int64) - g * n)
             for g in range(n_graphs)]
    if adj_format == "npz":
        save_adj_npz(os.path.join(d, "2D_adj.npz"), items, n)
    elif adj_format == "dense":
        dense = np.stack([b.dense_adj(g) for g in range(n_graphs)])
        np.save(os.path.join(d, "2D_adj.npy"), dense)
    else:
        raise ValueError(adj_format)
    np.save(os.path.join(d, "2D_node.npy"), b.feature_truth.reshape(n_graphs, n, -1) * NODE_SCALE)
    np.save(os.path.join(d, "2D_geometry.npy"),
            b.spatial_truth.reshape(n_graphs, n, -1) * COORD_SCALE)
    np.save(os.path.join(d, "2D_prop.npy"), np.arange(n_graphs, dtype=np.float64)[:, None])
    return d
