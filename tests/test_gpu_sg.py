"""SpatialGraphConvolution HIP layer (csrc/snd_sg.hip) vs the literal float64
oracle (oracle/ref_sg.py, `layers.py:143-198`, `model_joint.py:77-80`).

fp32 kernels against float64: outputs and every gradient within 1e-5 of the
block's max-abs; the encoder stack (2 layers, BN + lrelu) end to end.
Adjacency: sampled spanning trees of seeded RGGs (`input_data.py:18-38`, the
SG encoder's input) and the full RGG adjacency; rel = pairwise distances.
"""
import numpy as np
import pytest
import torch

from oracle import ref_sg as S

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu(lib_built):
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm device")


def graphs(B, N, tree, seed=0):
    from snd_vae_amd.data import csr_from_pairs, rgg_edges, stack_csr
    from snd_vae_amd.input_data import spanning_tree_edges
    rng = np.random.default_rng(seed)
    parts, dense, rel = [], [], []
    for b in range(B):
        pos, pairs = rgg_edges(N, 6.0, rng)
        if tree:
            und = np.concatenate([pairs, pairs[:, ::-1]])
            e = spanning_tree_edges(und, N, np.random.RandomState(seed + b))
            pairs = e.T[e[0] < e[1]]
        parts.append(csr_from_pairs(N, pairs))
        a = np.zeros((N, N))
        a[pairs[:, 0], pairs[:, 1]] = 1
        dense.append(a + a.T)
        rel.append(np.linalg.norm(pos[:, None] - pos[None], axis=-1) - 0.15)
    rp, ci = stack_csr(parts, N)
    return rp, ci, np.stack(dense), np.stack(rel)


def close(got, ref, tol=1e-5):
    got = got.double().cpu().numpy() if torch.is_tensor(got) else got
    err = np.abs(got - ref).max()
    assert err <= tol * max(1.0, np.abs(ref).max()), (err, np.abs(ref).max())


@pytest.mark.parametrize("tree", [True, False])
def test_layer_fwd_bwd(tree):
    from snd_vae_amd.sg import SGGraph, SpatialGraphConvolution, sg_pack, sg_unpack
    B, N, F, hid = 3, 24, 3, (20, 20, 20)
    rp, ci, A, rel = graphs(B, N, tree)
    rng = np.random.default_rng(5)
    p = S.init_sg_layer(F, hid, rng, stddev=0.3)
    for k, n in (("b1", 20), ("b2", 20), ("b3", 20)):
        p[k] = rng.normal(size=n) * 0.1
    x = rng.normal(size=(B, N, F))
    dO = rng.normal(size=(B, N, hid[2]))
    ref, g = S.sgconv_grads(A, x, rel, p, dO)
    g_dev = SGGraph(rp, ci, N, torch.from_numpy(rel.astype(np.float32)).cuda())
    blocks = {"Matrix1": p["M1"], "bias1": p["b1"], "Matrix2": p["M2"], "bias2": p["b2"],
              "Matrix3": p["M3"], "bias3": p["b3"]}
    flat = torch.from_numpy(sg_pack(F, hid, blocks).astype(np.float32)).cuda()
    layer = SpatialGraphConvolution(F, hid, flat, bn_act=False)
    xd = torch.from_numpy(x.reshape(B * N, F).astype(np.float32)).cuda()
    out, y = layer.forward(g_dev, xd)
    close(y, ref.reshape(B * N, -1))
    grads, dx = layer.backward(torch.from_numpy(dO.reshape(B * N, -1).astype(np.float32)).cuda())
    gb = sg_unpack(F, hid, grads.double().cpu().numpy())
    for mine, theirs in (("Matrix1", "M1"), ("bias1", "b1"), ("Matrix2", "M2"), ("bias2", "b2"),
                         ("Matrix3", "M3"), ("bias3", "b3")):
        close(gb[mine], g[theirs])
    close(dx, g["x"].reshape(B * N, F))


def test_encoder_stack_bn():
    """Two layers, reference widths [[20,20,20],[50,50,50]], BN + lrelu between."""
    from snd_vae_amd.sg import SGEncoder, SGGraph, sg_unpack
    import torch as T
    B, N, F = 2, 20, 1
    rp, ci, A, rel = graphs(B, N, True, seed=3)
    rng = np.random.default_rng(8)
    layers = []
    f = F
    for hid in ((20, 20, 20), (50, 50, 50)):
        p = S.init_sg_layer(f, hid, rng, stddev=0.2)
        p["gamma"] = 1.0 + 0.1 * rng.normal(size=hid[2])
        p["beta"] = 0.1 * rng.normal(size=hid[2])
        layers.append(p)
        f = hid[2]
    x = rng.random((B, N, F))
    ref = S.sg_encoder(A, x, rel, layers)
    names = {"M1": "Matrix1", "b1": "bias1", "M2": "Matrix2", "b2": "bias2", "M3": "Matrix3",
             "b3": "bias3", "gamma": "gamma", "beta": "beta"}
    enc = SGEncoder(F, blocks=[{names[k]: v for k, v in p.items()} for p in layers])
    g_dev = SGGraph(rp, ci, N, T.from_numpy(rel.astype(np.float32)).cuda())
    out = enc.forward(g_dev, T.from_numpy(x.reshape(B * N, F).astype(np.float32)).cuda())
    close(out, ref.reshape(B * N, -1))
    # gradients of sum(out * dO) through both layers vs torch autograd on the literal graph
    dO = rng.normal(size=ref.shape)
    tp = [{k: T.tensor(v, requires_grad=True) for k, v in p.items()} for p in layers]
    s = T.tensor(x)
    for q in tp:
        yv = S.sgconv_torch(T.tensor(A), s, T.tensor(rel), q)
        t = yv * (q["gamma"] * S.BN_C) + q["beta"]
        s = T.maximum(t, 0.2 * t)
    (s * T.tensor(dO)).sum().backward()
    grads, _ = enc.backward(T.from_numpy(dO.reshape(B * N, -1).astype(np.float32)).cuda())
    for li, (p, q) in enumerate(zip(layers, tp)):
        f = F if li == 0 else 20
        hid = ((20, 20, 20), (50, 50, 50))[li]
        gb = sg_unpack(f, hid, grads[li].double().cpu().numpy())
        for k, v in q.items():
            close(gb[names[k]], v.grad.numpy())


def test_asymmetric_rejected():
    from snd_vae_amd.sg import SGGraph
    rp = np.array([0, 1, 1], np.int32)
    ci = np.array([1], np.int32)
    with pytest.raises(ValueError, match="symmetric"):
        SGGraph(rp, ci, 2, torch.zeros(1, 2, 2, device="cuda"))
