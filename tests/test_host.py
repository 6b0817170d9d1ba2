"""CPU tests of host logic: CSR ingest (bit-exact vs scipy), batching,
sharding, the flat parameter layout, and the C ABI library's exports."""
import ctypes
import os
import re

import numpy as np
import pytest
import scipy.sparse as sp

from snd_vae_amd.config import PRESETS, tscale
from snd_vae_amd.data import (batch_from_dense, csr_from_dense, csr_from_pairs, rgg_edges,
                              shard, synthetic_batch)
from snd_vae_amd.params import block_shapes, flat_layout, init_blocks

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_rgg_sizes_match_survey():
    # SURVEY.md §8d seed-0 sizes
    for n, k, nnz in [(200, 8, 1434), (4096, 16, 64548)]:
        rng = np.random.default_rng(0)
        _, pairs = rgg_edges(n, k, rng)
        rp, cols = csr_from_pairs(n, pairs)
        assert int(rp[-1]) == nnz


@pytest.mark.parametrize("n,k", [(50, 5), (200, 8), (1, 0), (30, 0.0)])
def test_csr_bit_exact_vs_scipy(n, k):
    rng = np.random.default_rng(n)
    _, pairs = rgg_edges(n, k, rng)
    rp, cols = csr_from_pairs(n, pairs)
    dense = np.zeros((n, n))
    if len(pairs):
        dense[pairs[:, 0], pairs[:, 1]] = 1
        dense[pairs[:, 1], pairs[:, 0]] = 1
    ref = sp.csr_matrix(dense)
    ref.sort_indices()
    assert np.array_equal(rp, ref.indptr) and np.array_equal(cols, ref.indices)
    rp2, cols2 = csr_from_dense(dense)
    assert np.array_equal(rp2, ref.indptr) and np.array_equal(cols2, ref.indices)
    # np.where order == sparse_to_tuple order (preprocessing.py:7-13)
    r, c = np.where(dense)
    assert np.array_equal(np.repeat(np.arange(n), np.diff(rp)), r) and np.array_equal(cols, c)


def test_csr_from_dense_rejects_asymmetric():
    a = np.zeros((3, 3))
    a[0, 1] = 1
    with pytest.raises(ValueError):
        csr_from_dense(a)


def test_diagonal_dropped():
    a = np.eye(4) + np.diag(np.ones(3), 1) + np.diag(np.ones(3), -1)
    rp, cols = csr_from_dense(a)
    assert int(rp[-1]) == 6 and all(c != r for r in range(4) for c in cols[rp[r]:rp[r + 1]])


def test_batch_block_diagonal_and_dense_roundtrip():
    cfg = tscale(40, 16, mean_degree=5.0)
    b = synthetic_batch(cfg, 3, seed=2)
    adj = np.stack([b.dense_adj(i) for i in range(3)])
    b2 = batch_from_dense(cfg, adj, b.feature_truth.reshape(3, 40, 1), b.spatial_truth.reshape(3, 40, 2))
    assert np.array_equal(b.rowptr, b2.rowptr) and np.array_equal(b.colidx, b2.colidx)
    assert np.array_equal(b.features, b2.features)
    # columns of graph g stay inside [g*N, (g+1)*N)
    for g in range(3):
        s, e = b.rowptr[g * 40], b.rowptr[(g + 1) * 40]
        assert (b.colidx[s:e] >= g * 40).all() and (b.colidx[s:e] < (g + 1) * 40).all()


def test_shard_partitions_graphs():
    cfg = tscale(30, 16, mean_degree=5.0)
    b = synthetic_batch(cfg, 4, seed=0)
    parts = [shard(b, r, 2) for r in range(2)]
    for r, p in enumerate(parts):
        ref = synthetic_batch(cfg, 2, seed=2 * r)
        assert np.array_equal(p.rowptr, ref.rowptr) and np.array_equal(p.colidx, ref.colidx)
        assert np.array_equal(p.features, ref.features)


def test_flat_layout_alignment_and_counts():
    cfg = PRESETS["C2"]
    lay = flat_layout(cfg)
    assert all(o % 64 == 0 for o in lay.offsets.values())
    n = sum(int(np.prod(s)) for s in block_shapes(cfg).values())
    assert 55_000 < n < 70_000         # ~61K params (~245 KB)
    blocks = init_blocks(cfg, 0)
    flat = lay.pack(blocks)
    back = lay.unpack(flat)
    assert all(np.allclose(back[k], blocks[k].astype(np.float32)) for k in blocks)


def _header_functions():
    src = open(os.path.join(ROOT, "include", "snd_vae.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[\w\s\*]+?\b(snd_\w+)\s*\(", src, flags=re.M)))


def test_library_exports_every_header_symbol(lib_built):
    names = _header_functions()
    assert len(names) >= 20
    so = ctypes.CDLL(lib_built)
    missing = [n for n in names if not hasattr(so, n)]
    assert not missing, missing
    from snd_vae_amd import _lib
    assert set(_lib.EXPORTS) == set(names)


def test_abi_version_agrees_everywhere(lib_built):
    """One ABI number: the header's SND_ABI_VERSION, the library's snd_abi_version(), the
    Python binding's ABI_VERSION and the ctypes stub a maintainer copies from
    INTEGRATION.md (round 5 shipped a stub asserting 14 against a library at 17)."""
    from snd_vae_amd import _lib
    hdr = open(os.path.join(ROOT, "include", "snd_vae.h")).read()
    m = re.search(r"#define\s+SND_ABI_VERSION\s+(\d+)", hdr)
    assert m, "include/snd_vae.h must define SND_ABI_VERSION"
    so = ctypes.CDLL(lib_built)
    so.snd_abi_version.restype = ctypes.c_int
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    stub = [int(v) for v in re.findall(r"^SND_ABI_VERSION\s*=\s*(\d+)", doc, flags=re.M)]
    assert "assert lib.snd_abi_version() == SND_ABI_VERSION" in doc
    assert stub == [int(m.group(1))], stub
    assert so.snd_abi_version() == int(m.group(1)) == _lib.ABI_VERSION


def test_plan_layout_matches_python(lib_built):
    """snd_plan_create needs no GPU: check its flat layout against params.py."""
    from snd_vae_amd import _lib
    from snd_vae_amd.model import c_config
    for preset in ("C1", "C1s", "C2", "C4", "C5", "SG25"):
        cfg = PRESETS[preset]
        L = _lib.lib()
        h = ctypes.c_void_p()
        cc = c_config(cfg, "bf16")
        rc = L.snd_plan_create(ctypes.byref(cc), 8, ctypes.byref(h))
        if rc != 0 and "hipFuncSetAttribute" in _lib.last_error():
            pytest.skip("HIP runtime unavailable on this host")
        _lib.check(rc)
        lay = flat_layout(cfg)
        assert L.snd_plan_param_count(h) == lay.total
        for i, k in enumerate(lay.shapes):
            nm, off, n = ctypes.c_char_p(), ctypes.c_longlong(), ctypes.c_longlong()
            _lib.check(L.snd_plan_param_block(h, i, ctypes.byref(nm), ctypes.byref(off), ctypes.byref(n)))
            assert (nm.value.decode(), off.value, n.value) == (k, lay.offsets[k], lay.numel(k))
        L.snd_plan_destroy(h)


@pytest.mark.parametrize("n,B,kbar,tile_rows,locality", [(4096, 2, 16.0, 64, True), (300, 3, 10.0, 64, False),
                                                          (96, 2, 0.0, 32, True), (200, 1, 8.0, 7, True),
                                                          (256, 2, 12.0, 128, True)])
def test_spmm_tile_plan(lib_built, n, B, kbar, tile_rows, locality):
    """snd_spmm_tile_plan (host C++) against a numpy restatement: each tile holds
    its schedule slots' rows sorted by degree (descending, stable), its set is the
    ascending distinct neighbour rows padded with -1 to ustride, and the slot-order
    lcol maps every entry back to its column id in colidx order."""
    from snd_vae_amd.data import GraphBatch, locality_order, row_tiles, csr_from_pairs, rgg_edges, stack_csr
    parts = []
    for b in range(B):
        _, pairs = rgg_edges(n, kbar, np.random.default_rng(11 + b))
        parts.append(csr_from_pairs(n, pairs))
    rp, ci = stack_csr(parts, n)
    gb = GraphBatch(B, n, rp, ci, np.zeros((n * B, 1), np.float32), np.zeros((n * B, 1), np.float32),
                    np.zeros((n * B, 2), np.float32))
    order = locality_order(gb) if locality else None
    rt = row_tiles(gb, order, tile_rows)
    R = n * B
    sched = np.arange(R) if order is None else order.astype(np.int64)
    T = (R + tile_rows - 1) // tile_rows
    deg = np.diff(rp.astype(np.int64))
    assert rt.trp[0] == 0 and rt.trp[-1] == len(ci) and len(rt.ucol) >= T * rt.ustride
    sizes = []
    for t in range(T):
        sl = sched[t * tile_rows:(t + 1) * tile_rows]
        want_rows = sl[np.argsort(-deg[sl], kind="stable")]
        got_rows = rt.rows[t * tile_rows:t * tile_rows + len(sl)]
        assert np.array_equal(got_rows, want_rows)
        cols = np.concatenate([ci[rp[r]:rp[r + 1]] for r in sl] + [np.zeros(0, ci.dtype)])
        u = np.unique(cols)
        us = rt.ucol[t * rt.ustride:(t + 1) * rt.ustride]
        assert np.array_equal(us[:len(u)], u) and np.all(us[len(u):] == -1)
        sizes.append(len(u))
        for i, r in enumerate(got_rows):
            slot = t * tile_rows + i
            s, e = rt.trp[slot], rt.trp[slot + 1]
            assert e - s == deg[r]
            assert np.all(rt.lcol[s:e] >= 1)
            assert np.array_equal(us[rt.lcol[s:e].astype(np.int64) - 1], ci[rp[r]:rp[r + 1]])
    assert rt.ustride == max(sizes)


@pytest.mark.parametrize("topology", ["tscale", "tref"])
def test_reference_checkpoint_names_roundtrip(topology):
    """checkpoint.reference_to_blocks / blocks_to_reference: the tf.train.Saver
    variable names of the hot path (params.logical_names) map onto the flat layout
    and back, with TF1 Adam slots (<var>/Adam, <var>/Adam_1) and the global step
    recovered from beta1_power (optimizer.py:125,197)."""
    import numpy as np

    from snd_vae_amd import checkpoint
    from snd_vae_amd.config import tref, tscale
    from snd_vae_amd.params import init_blocks, logical_names
    cfg = tscale(40, 8) if topology == "tscale" else tref(40, 8, g_hidden=12, latent=6)
    b = init_blocks(cfg, 5)
    rng = np.random.default_rng(0)
    m = {k: rng.standard_normal(v.shape) for k, v in b.items()}
    v = {k: rng.random(v.shape) for k, v in b.items()}
    ref = checkpoint.blocks_to_reference(cfg, b, m, v, global_step=17)
    assert set(logical_names(cfg)) <= set(ref)
    # a TF session dump carries an outer scope and ":0" suffixes
    dumped = {f"SGCNModelVAE/{k}:0": a for k, a in ref.items()}
    b2, m2, v2, step = checkpoint.reference_to_blocks(cfg, dumped)
    assert step == 17
    for k in b:
        np.testing.assert_array_equal(b2[k], b[k].astype(np.float32))
        np.testing.assert_array_equal(m2[k], m[k].astype(np.float32))
        np.testing.assert_array_equal(v2[k], v[k].astype(np.float32))
    # the mu / log-std heads are separate reference variables fused in enc.Wms
    L = cfg.latent
    np.testing.assert_array_equal(ref["encoder/g_g3_lin/Matrix"], b["enc.Wms"][:, L:].astype(np.float32))
    bad = dict(ref)
    bad["decoder/d_bn_s0/moving_variance"] = bad["decoder/d_bn_s0/moving_variance"] * 2
    with pytest.raises(ValueError, match="frozen"):
        checkpoint.reference_to_blocks(cfg, bad)
    del bad["encoder/g_g0_conv/w"]
    with pytest.raises(KeyError):
        checkpoint.reference_to_blocks(cfg, bad)


def test_reference_adam_power_convention():
    """TF1 AdamOptimizer starts beta1_power at beta1 and multiplies after each
    apply (optimizer.py:125,197): a fresh state (0.9, 0.999) is step 0, a state
    after t steps holds beta^(t+1).  beta1_power underflows float32 after ~830
    steps, so the step then comes from beta2_power; slots without any power raise."""
    import numpy as np

    from snd_vae_amd import checkpoint
    from snd_vae_amd.config import tscale
    from snd_vae_amd.params import init_blocks
    cfg = tscale(24, 4)
    b = init_blocks(cfg, 1)
    m = {k: np.zeros_like(a) for k, a in b.items()}
    ref0 = checkpoint.blocks_to_reference(cfg, b, m, m, global_step=0)
    assert ref0["beta1_power"] == np.float32(0.9) and ref0["beta2_power"] == np.float32(0.999)
    fresh = dict(ref0)
    fresh["beta1_power"] = np.float32(0.9)
    fresh["beta2_power"] = np.float32(0.999)
    assert checkpoint.reference_to_blocks(cfg, fresh)[3] == 0
    for t in (1, 5, 829, 1500, 20000, 50000, 86000):
        st = dict(ref0)
        # as TF builds them: repeated float32 multiplication by float32(beta)
        st["beta1_power"] = checkpoint.tf_power(0.9, t)
        st["beta2_power"] = checkpoint.tf_power(0.999, t)
        assert checkpoint.reference_to_blocks(cfg, st)[3] == t, t
        assert checkpoint.blocks_to_reference(cfg, b, m, m, global_step=t)["beta2_power"] == st["beta2_power"]
    dead = dict(ref0)
    dead["beta1_power"] = np.float32(0.0)
    dead["beta2_power"] = np.float32(0.0)
    with pytest.raises(ValueError, match="global_step"):
        checkpoint.reference_to_blocks(cfg, dead)
    assert checkpoint.reference_to_blocks(cfg, dead, global_step=123456)[3] == 123456
    nopow = {k: a for k, a in ref0.items() if not k.endswith("_power")}
    with pytest.raises(ValueError, match="global_step"):
        checkpoint.reference_to_blocks(cfg, nopow)


@pytest.mark.parametrize("n,B,kbar", [(500, 3, 8.0), (4096, 2, 16.0), (97, 4, 5.0)])
def test_window_plan_matches_literal(n, B, kbar):
    """data.window_plan (sliding-window SpMM plan) against a per-row restatement:
    position q holds row order[q]; its list = ring slots of its neighbours'
    positions in colidx order, then the zero row's slot 1096 up to its wavefront
    group's largest degree (at most 32), in 8s; meta = (start8 << 6) | degree,
    listed (with rows) by degree descending inside every aligned 128-position
    block, a group = 8 consecutive rows of that listing (one wavefront)."""
    from snd_vae_amd.config import tscale
    from snd_vae_amd.data import locality_order, synthetic_batch, window_plan
    b = synthetic_batch(tscale(n, 16, mean_degree=kbar), B, seed=n)
    order = locality_order(b)
    wp = window_plan(b, order)
    R = n * B
    pos = np.empty(R, np.int64)
    pos[order] = np.arange(R) % n
    deg = np.array([b.rowptr[r + 1] - b.rowptr[r] for r in order], np.int64)
    keys, gmax = {}, np.zeros(R, np.int64)
    for g in range(B):
        for lo in range(0, n, 128):
            qs = list(range(g * n + lo, g * n + min(lo + 128, n)))
            key = sorted(qs, key=lambda q: (-deg[q], q))
            keys[(g, lo)] = (qs, key)
            for i, q in enumerate(key):
                gmax[q] = deg[key[i - i % 8]]
    start, beta = 0, 0
    meta = np.zeros(R, np.int64)
    for q in range(R):
        row = int(order[q])
        nb = b.colidx[b.rowptr[row]:b.rowptr[row + 1]].astype(np.int64)
        meta[q] = (start // 8) << 6 | len(nb)
        plen = (max(len(nb), min(int(gmax[q]), 32)) + 7) // 8 * 8
        np.testing.assert_array_equal(wp.slots[start:start + len(nb)], pos[nb] % 1096)
        assert (wp.slots[start + len(nb):start + plen] == 1096).all()
        assert all(nb // n == row // n)                       # block diagonal
        if len(nb):
            beta = max(beta, int(np.abs(pos[nb] - q % n).max()))
        start += plen
    assert wp.beta == beta
    assert len(wp.slots) >= start + 24 and (wp.slots[start:] == 1096).all()   # the kernel's 32-entry reads
    np.testing.assert_array_equal(wp.order, order)
    for qs, key in keys.values():
        np.testing.assert_array_equal(wp.meta[qs[0]:qs[-1] + 1], meta[key])
        np.testing.assert_array_equal(wp.rows[qs[0]:qs[-1] + 1], order[key])




def test_grad_event_points_and_buckets(lib_built):
    """snd_plan_grad_event (ABI 13): the graph-latent d_sg_lin1 weight and bias complete
    at point 1 (after the projection backward), the graph-latent head weight at point 2
    (after the head backward), everything else at the final reduction; the bucket plan
    of C4 at 8 ranks shards the two 100 MB runs and all-reduces the small rest; C2 is one
    all-reduce of the whole gradient and the loss tail."""
    from snd_vae_amd import _lib
    from snd_vae_amd.model import c_config
    from snd_vae_amd.parallel import plan_buckets
    for preset in ("C4", "C2"):
        cfg = PRESETS[preset]
        L = _lib.lib()
        h = ctypes.c_void_p()
        cc = c_config(cfg, "bf16")
        rc = L.snd_plan_create(ctypes.byref(cc), 8, ctypes.byref(h))
        if rc != 0 and "hipFuncSetAttribute" in _lib.last_error():
            pytest.skip("HIP runtime unavailable on this host")
        _lib.check(rc)
        lay = flat_layout(cfg)
        names = list(lay.shapes)
        pts = [L.snd_plan_grad_event(h, i, None) for i in range(len(names))]
        want = {"dec.Wp": 1, "dec.bp": 1, "enc.Wh": 2} if preset == "C4" else {}
        assert pts == [want.get(k, 0) for k in names]
        assert L.snd_plan_grad_event(h, len(names), None) < 0
        blocks = [(lay.offsets[k], (lay.offsets[names[i + 1]] if i + 1 < len(names) else lay.total)
                   - lay.offsets[k]) for i, k in enumerate(names)]
        bk = plan_buckets(blocks, pts, lay.total, lay.total + 8, 8)
        if preset == "C4":
            assert [(b.point, b.sharded) for b in bk] == [(1, True), (2, True), (0, False), (0, False),
                                                          (0, False)]
            assert (bk[0].lo, bk[0].hi) == (lay.offsets["dec.Wp"], lay.offsets["dec.K1"])
            assert (bk[1].lo, bk[1].hi) == (lay.offsets["enc.Wh"], lay.offsets["enc.bh"])
            assert bk[-1].hi == lay.total + 8
        else:
            assert [(b.lo, b.hi, b.point, b.sharded) for b in bk] == [(0, lay.total + 8, 0, False)]
        L.snd_plan_destroy(h)


def test_fused_adam_block_kinds(lib_built):
    """snd_plan_block_fused (ABI 16) after snd_plan_fuse_adam: the node-latent plans
    update every block inside the final slab reduction (2); the graph-latent plans
    update d_sg_lin1 (weight and bias) / the head weight in their weight streams (1),
    and the rest in the reduction: no separate Adam launch on any preset.  Without m / v nothing is fused."""
    from snd_vae_amd import _lib
    from snd_vae_amd.model import c_config
    L = _lib.lib()
    state = (ctypes.c_float * 4)()
    for preset in ("C2", "C3", "C4", "C5"):
        cfg = PRESETS[preset]
        h = ctypes.c_void_p()
        cc = c_config(cfg, "bf16")
        rc = L.snd_plan_create(ctypes.byref(cc), 1 if preset == "C3" else 8, ctypes.byref(h))
        if rc != 0 and "hipFuncSetAttribute" in _lib.last_error():
            pytest.skip("HIP runtime unavailable on this host")
        _lib.check(rc)
        names = list(flat_layout(cfg).shapes)
        assert [L.snd_plan_block_fused(h, i) for i in range(len(names))] == [0] * len(names)
        _lib.check(L.snd_plan_fuse_adam(h, state, state, 1e-3, 0.9, 0.999, 1e-8))
        kinds = {k: L.snd_plan_block_fused(h, i) for i, k in enumerate(names)}
        want = {"enc.Wh": 1, "dec.Wp": 1, "dec.bp": 1} if preset == "C4" else {}
        assert kinds == {k: want.get(k, 2) for k in names}, preset
        _lib.check(L.snd_plan_fuse_adam(h, None, None, 1e-3, 0.9, 0.999, 1e-8))
        assert [L.snd_plan_block_fused(h, i) for i in range(len(names))] == [0] * len(names)
        L.snd_plan_destroy(h)


def test_reduce_adam_option(lib_built):
    """Plan option "reduce_adam" = 0 leaves the reduction-completed blocks to the caller's
    snd_adam_tf1 (kind 0); the weight-stream kinds are unaffected."""
    from snd_vae_amd import _lib
    from snd_vae_amd.model import c_config
    L = _lib.lib()
    state = (ctypes.c_float * 4)()
    cfg = PRESETS["C4"]
    h = ctypes.c_void_p()
    rc = L.snd_plan_create(ctypes.byref(c_config(cfg, "bf16")), 2, ctypes.byref(h))
    if rc != 0 and "hipFuncSetAttribute" in _lib.last_error():
        pytest.skip("HIP runtime unavailable on this host")
    _lib.check(rc)
    names = list(flat_layout(cfg).shapes)
    assert L.snd_plan_set_option(h, b"reduce_adam", 0) == 0
    _lib.check(L.snd_plan_fuse_adam(h, state, state, 1e-3, 0.9, 0.999, 1e-8))
    kinds = {k: L.snd_plan_block_fused(h, i) for i, k in enumerate(names)}
    assert kinds == {k: 1 if k in ("enc.Wh", "dec.Wp", "dec.bp") else 0 for k in names}
    # the kinds cannot change under a fused update (a cached range list would skip or
    # double a block's update): unfuse first
    assert L.snd_plan_set_option(h, b"reduce_adam", 1) == -1   # SND_ERR_ARG
    assert L.snd_plan_set_option(h, b"reduce_adam", 0) == 0
    _lib.check(L.snd_plan_fuse_adam(h, None, None, 1e-3, 0.9, 0.999, 1e-8))
    assert L.snd_plan_set_option(h, b"reduce_adam", 1) == 1
    _lib.check(L.snd_plan_fuse_adam(h, state, state, 1e-3, 0.9, 0.999, 1e-8))
    assert L.snd_plan_block_fused(h, names.index("enc.W0")) == 2
    L.snd_plan_destroy(h)


# kernels that may spill, with the most they may spill (VGPRs per lane); every other
# kernel of the library must not.  Not on the C2 step: the register-gather fallbacks,
# the v1 zz^T at d = 128 and the fp32 parity zz^T.
KNOWN_SPILLS = {
    "spmm_bf16_tiled_kernelILi1ELi1ELi1E": 4, "spmm_bf16_tiled_kernelILi1ELi1ELi2E": 30,
    "zzt_dense_bf16ILi128E": 0, "zzt_dense_f32ILi128E": 42,
    "zzt_dense_bf16_v7": 2,            # C5's zz^T
    "rowconv_kernelILi3ELi4E": 6,      # RC_ENC1 at 4 column blocks (C5 widths)
}


def test_no_register_spills_in_shipped_kernels(lib_built):
    """hipcc's kernel-resource remarks, recorded by build.py per object: a kernel that
    starts spilling (round 4: dec_bwd_kernel, 72 VGPRs, 26 us per C2 step) fails here on
    the CPU, before any GPU run."""
    from snd_vae_amd.build import kernel_resources
    res = kernel_resources()
    assert len(res) > 50
    bad = {}
    for k, v in res.items():
        allow = next((n for sub, n in KNOWN_SPILLS.items() if sub in k), 0)
        if v.get("vgpr_spill", 0) > allow or (v.get("scratch", 0) and not any(s in k for s in KNOWN_SPILLS)):
            bad[k] = v
    assert not bad, bad
    for hot in ("dec_bwd_kernel", "dec_fwd_kernel", "head_bwd_kernel", "head_fwd_kernel",
                "enc_front_kernel", "zzt_dense_bf16_v4", "wgrad_multi_kernel", "spmm_win_kernel"):
        ks = [k for k in res if hot in k]
        assert ks and all(res[k].get("vgpr_spill", 0) == 0 and res[k].get("scratch", 0) == 0 for k in ks), hot
