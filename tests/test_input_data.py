"""Reference on-disk ingest (`input_data.py:18-142`) and the checkpoint format.

The literal restatement below follows `load_data_syn` line by line (dense
matrices, np.where edge lists, scipy MST under U[1,2) weights, one global
shuffle) and is the oracle for the sparse ingest's array contents, spanning
trees and graph order under the same global RNG seed (`main.py:124-125`).
"""
import os

import numpy as np
import pytest
import scipy.sparse as sp

from snd_vae_amd.config import tscale
from snd_vae_amd.input_data import (COORD_SCALE, NODE_SCALE, load_adjacency, load_data_syn,
                                    write_synthetic_dataset)


def literal_load(path, sampling_num):
    """`input_data.py:54-95` with the reference's own data structures (small N)."""
    from scipy.sparse import csr_matrix
    from scipy.sparse.csgraph import minimum_spanning_tree
    a = np.load(os.path.join(path, "train", "2D_adj.npy"), allow_pickle=True)
    node = np.load(os.path.join(path, "train", "2D_node.npy")) / 120
    spatial = np.load(os.path.join(path, "train", "2D_geometry.npy")) / 600
    new_adj = []
    for n in range(len(a)):
        m = a[n].toarray() if hasattr(a[n], "toarray") else np.array(a[n])
        for i in range(len(m)):
            m[i, i] = 0
            for j in range(len(m)):
                assert m[i, j] == m[j, i]
        new_adj.append(m)
    new_adj = np.array(new_adj)
    trees = []
    for adj in new_adj:
        x, y = np.where(adj)
        edges = np.concatenate((x.reshape(-1, 1), y.reshape(-1, 1)), axis=1)
        sub = []
        for _ in range(sampling_num):
            row, col = edges[:, 0], edges[:, 1]
            cg = csr_matrix((np.random.random(len(edges)) + 1, (row, col)),
                            shape=(node.shape[1], node.shape[1]))
            tr, tc = minimum_spanning_tree(cg).nonzero()
            st = np.concatenate([[tr], [tc]]).T.T
            und = np.array([np.concatenate([st[0], st[1]]), np.concatenate([st[1], st[0]])])
            t = np.zeros_like(adj)
            t[und[0], und[1]] = 1
            sub.append(t)
        trees.append(sub)
    trees = np.array(trees)
    index = [i for i in range(len(node))]
    np.random.shuffle(index)
    return node[index], spatial[index], trees[index], new_adj[index]


@pytest.fixture(scope="module")
def ds_dir(tmp_path_factory):
    cfg = tscale(40, 16, mean_degree=5.0)
    root = str(tmp_path_factory.mktemp("syn"))
    d = write_synthetic_dataset(root, cfg, 6, seed=3, adj_format="dense")
    # the reference's own adjacency format: an object array of scipy sparse matrices
    dense = np.load(os.path.join(d, "2D_adj.npy"))
    obj = np.empty(len(dense), dtype=object)
    for g in range(len(dense)):
        m = dense[g].copy()
        m[0, 0] = 1.0                                 # a diagonal entry the loader must zero
        obj[g] = sp.csr_matrix(m)
    os.makedirs(os.path.join(root, "pickled", "train"))
    for f in ("2D_node.npy", "2D_geometry.npy", "2D_prop.npy"):
        os.link(os.path.join(d, f), os.path.join(root, "pickled", "train", f))
    np.save(os.path.join(root, "pickled", "train", "2D_adj.npy"), obj, allow_pickle=True)
    return cfg, root


def test_matches_literal_reference(ds_dir):
    cfg, root = ds_dir
    path = os.path.join(root, "pickled")
    np.random.seed(1)
    node, spatial, trees, new_adj = literal_load(path, 3)
    np.random.seed(1)
    ds = load_data_syn("train", path, sampling_num=3, allow_pickle=True)
    n = cfg.n_nodes
    assert ds.n_graphs == 6 and ds.n_nodes == n
    np.testing.assert_array_equal(ds.node.reshape(6, n, 1), node.reshape(6, n, 1))
    np.testing.assert_array_equal(ds.spatial, spatial)
    for g in range(6):
        np.testing.assert_array_equal(ds.dense_adj(g), new_adj[g])
        np.testing.assert_array_equal(ds.dense_trees(g), trees[g])


def test_pickle_refused_without_opt_in(ds_dir):
    _, root = ds_dir
    with pytest.raises(ValueError, match="allow_pickle"):
        load_data_syn("train", os.path.join(root, "pickled"), sampling_num=0)


def test_npz_dense_and_values(ds_dir, tmp_path):
    cfg, root = ds_dir
    write_synthetic_dataset(str(tmp_path), cfg, 6, seed=3, adj_format="npz")
    a = load_data_syn("train", str(tmp_path), sampling_num=0, shuffle=False)
    b = load_data_syn("train", root, sampling_num=0, shuffle=False)
    from snd_vae_amd.data import synthetic_batch
    ref = synthetic_batch(cfg, 6, seed=3)
    n = cfg.n_nodes
    for g in range(6):
        np.testing.assert_array_equal(a.dense_adj(g), ref.dense_adj(g))
        np.testing.assert_array_equal(b.dense_adj(g), ref.dense_adj(g))
    np.testing.assert_allclose(a.node.reshape(-1, 1), ref.feature_truth, rtol=1e-6)
    np.testing.assert_allclose(a.spatial.reshape(-1, 2), ref.spatial_truth, rtol=1e-6)
    # the batch for the device path equals the generator's batch (same CSR, same features)
    bb = a.batch(cfg, range(6))
    np.testing.assert_array_equal(bb.rowptr, ref.rowptr)
    np.testing.assert_array_equal(bb.colidx, ref.colidx)
    np.testing.assert_allclose(bb.features, ref.features, rtol=1e-6)
    assert NODE_SCALE == 120 and COORD_SCALE == 600


def test_test_split_reads_train_factor(ds_dir, tmp_path):
    cfg, _ = ds_dir
    write_synthetic_dataset(str(tmp_path), cfg, 4, seed=1, split="train")
    write_synthetic_dataset(str(tmp_path), cfg, 2, seed=9, split="test")
    ds = load_data_syn("test_reconstruct", str(tmp_path), sampling_num=0, shuffle=False)
    assert ds.n_graphs == 2 and ds.factor.shape[0] == 4      # input_data.py:101 quirk kept


def test_asymmetric_rejected(tmp_path):
    d = tmp_path / "train"
    d.mkdir()
    a = np.zeros((1, 4, 4), np.float32)
    a[0, 0, 1] = 1
    np.save(d / "2D_adj.npy", a)
    np.save(d / "2D_node.npy", np.zeros((1, 4)))
    np.save(d / "2D_geometry.npy", np.zeros((1, 4, 2)))
    n, items = load_adjacency(str(d))
    assert n == 4 and len(items) == 1
    with pytest.raises(ValueError, match="symmetric"):
        load_data_syn("train", str(tmp_path), sampling_num=0)


def test_checkpoint_roundtrip_metadata(tmp_path):
    """Checkpoint metadata round trip without a GPU (layout/config checks)."""
    from snd_vae_amd import checkpoint as ck
    from snd_vae_amd.params import flat_layout
    import torch

    cfg = tscale(40, 16)

    class M:                                       # the attributes checkpoint.save reads
        pass
    m = M()
    m.cfg, m.layout = cfg, flat_layout(cfg)
    m.param_count = m.layout.total
    m.params = torch.arange(m.param_count + 8, dtype=torch.float32)
    fn = str(tmp_path / "c.safetensors")
    ck.save(fn, m)
    assert ck.read_config(fn) == cfg
    m2 = M()
    m2.cfg, m2.layout, m2.param_count = cfg, m.layout, m.param_count
    m2.params = torch.zeros_like(m.params)
    ck.restore(fn, m2)
    assert torch.equal(m2.params[:m.param_count], m.params[:m.param_count])
    m3 = M()
    m3.cfg = tscale(40, 32)
    m3.layout = flat_layout(m3.cfg)
    m3.param_count = m3.layout.total
    m3.params = torch.zeros(m3.param_count)
    with pytest.raises(ValueError, match="layout"):
        ck.restore(fn, m3)


def test_class_balance_matches_main_formula(ds_dir):
    """Row a15: pos_weight / norm of `main.py:246-247`, literally, over the spanning-tree
    adjacency `adj` [G*S, N, N] of `main.py:177` -- against dataset_class_balance on the
    sparse ingest (same trees under the same seed)."""
    from snd_vae_amd.input_data import class_balance, dataset_class_balance
    cfg, root = ds_dir
    path = os.path.join(root, "pickled")
    np.random.seed(1)
    _, _, trees, _ = literal_load(path, 3)
    adj = trees.reshape(-1, trees.shape[-2], trees.shape[-1])          # main.py:177
    pos_weight = float(adj.shape[0] * adj.shape[1] * adj.shape[1] - adj.sum()) / adj.sum()
    norm = adj.shape[0] * adj.shape[1] * adj.shape[1] / float(
        (adj.shape[0] * adj.shape[1] * adj.shape[1] - adj.sum()) * 2)
    np.random.seed(1)
    ds = load_data_syn("train", path, sampling_num=3, allow_pickle=True)
    pw, nm = dataset_class_balance(ds)
    assert pw == pytest.approx(pos_weight, rel=1e-12) and nm == pytest.approx(norm, rel=1e-12)
    assert class_balance(2, 4, 4) == (7.0, 32 / 56)
    with pytest.raises(ValueError):
        class_balance(1, 4, 0)
    with pytest.raises(ValueError, match="spanning"):
        dataset_class_balance(load_data_syn("train", path, sampling_num=0, allow_pickle=True))
