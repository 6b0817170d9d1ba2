"""Launch only the bf16 SpMM (snd_csr_spmm_bf16) on a large block-diagonal batch.

    rocprofv3 --kernel-trace --stats -- python tools/prof_spmm.py [--copies 32 --reps 20]
    rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -- python tools/prof_spmm.py
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--copies", type=int, default=32)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--width", type=int, default=64)
    ap.add_argument("--natural-order", action="store_true", help="no XCD-aware row-block order")
    ap.add_argument("--no-locality", action="store_true", help="no RCM row schedule")
    ap.add_argument("--tile-rows", type=int, default=0, help="> 0: the row-tiled LDS kernel")
    args = ap.parse_args()
    import numpy as np
    import torch

    from snd_vae_amd import _lib
    from snd_vae_amd.config import tscale
    from snd_vae_amd.data import synthetic_batch
    host = synthetic_batch(tscale(4096, 64), 8, seed=1000)
    rp0, ci0 = host.rowptr.astype(np.int64), host.colidx.astype(np.int64)
    nnz0, R0 = int(rp0[-1]), host.n_graphs * host.n_nodes
    c = args.copies
    rp = np.concatenate([rp0[:-1] + k * nnz0 for k in range(c)] + [np.array([c * nnz0])])
    ci = np.concatenate([ci0 + k * R0 for k in range(c)])
    R = R0 * c
    from snd_vae_amd.data import locality_order
    o0 = locality_order(host).astype(np.int64)
    d_order = None if args.no_locality else torch.from_numpy(
        np.concatenate([o0 + k * R0 for k in range(c)]).astype(np.int32)).cuda()
    d_rp = torch.from_numpy(rp.astype(np.int32)).cuda()
    d_ci = torch.from_numpy(ci.astype(np.int32)).cuda()
    h = torch.randn(R, args.width, device="cuda").to(torch.bfloat16)
    out = torch.empty_like(h)
    L = _lib.lib()
    npg, ng = (0, 0) if args.natural_order else (host.n_nodes, host.n_graphs * c)
    if args.tile_rows > 0:
        import ctypes
        from snd_vae_amd.data import GraphBatch, row_tiles
        z = np.zeros((1, 1), np.float32)
        big = GraphBatch(host.n_graphs * c, host.n_nodes, rp.astype(np.int32), ci.astype(np.int32), z, z, z)
        order = None if d_order is None else d_order.cpu().numpy()
        from snd_vae_amd.model import DeviceTiles
        rt = row_tiles(big, order, args.tile_rows)
        dt = DeviceTiles(rt)
        tiles = dt.c_struct()
        print("tile rows", args.tile_rows, "ustride", rt.ustride)
        for _ in range(args.reps):
            _lib.check(L.snd_csr_spmm_bf16_tiled(d_rp.data_ptr(), d_ci.data_ptr(), R, ctypes.byref(tiles),
                                                 h.data_ptr(), args.width, args.width, out.data_ptr(),
                                                 args.width, npg, ng,
                                                 0 if d_order is None else d_order.data_ptr(),
                                                 _lib.stream_ptr()))
    for _ in range(args.reps if args.tile_rows <= 0 else 0):
        _lib.check(L.snd_csr_spmm_bf16(d_rp.data_ptr(), d_ci.data_ptr(), R, h.data_ptr(), args.width,
                                       args.width, out.data_ptr(), args.width, npg, ng,
                                       0 if d_order is None else d_order.data_ptr(),
                                       _lib.stream_ptr()))
    torch.cuda.synchronize()
    print("ok", R, len(ci))


if __name__ == "__main__":
    main()
