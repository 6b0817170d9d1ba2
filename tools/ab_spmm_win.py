"""A/B the window SpMM (snd_csr_spmm_bf16_window) on bench.py's 256-graph batch under
snd_debug_set flags, alternating the flags within one process (HIP events).

    python tools/ab_spmm_win.py --flags 0,524288 --rounds 4
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--flags", default="0")
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--copies", type=int, default=32)
    args = ap.parse_args()
    import ctypes

    import numpy as np
    import torch

    import bench
    from snd_vae_amd import _lib
    from snd_vae_amd.config import tscale
    from snd_vae_amd.data import GraphBatch, locality_order, synthetic_batch, window_plan
    from snd_vae_amd.layers import DeviceWindowPlan
    host = synthetic_batch(tscale(4096, 64), 8, seed=1000)
    rp0, ci0 = host.rowptr.astype(np.int64), host.colidx.astype(np.int64)
    nnz0, R0 = int(rp0[-1]), host.n_graphs * host.n_nodes
    c = args.copies
    rp = np.concatenate([rp0[:-1] + k * nnz0 for k in range(c)] + [np.array([c * nnz0])])
    ci = np.concatenate([ci0 + k * R0 for k in range(c)])
    o0 = locality_order(host).astype(np.int64)
    order = np.concatenate([o0 + k * R0 for k in range(c)]).astype(np.int32)
    R = R0 * c
    z = np.zeros((1, 1), np.float32)
    big = GraphBatch(host.n_graphs * c, host.n_nodes, rp.astype(np.int32), ci.astype(np.int32), z, z, z)
    wp = window_plan(big, order)
    dw = DeviceWindowPlan(wp)
    h = torch.randn(R, 64, device="cuda").to(torch.bfloat16)
    out = torch.empty_like(h)
    L = _lib.lib()
    ng = host.n_graphs * c
    byts = 4 * (R + 1) + 4 * len(ci) + 2 * 2 * R * 64
    run = lambda sp: _lib.check(L.snd_csr_spmm_bf16_window(
        dw.meta.data_ptr(), dw.slots.data_ptr(), dw.rows.data_ptr(), dw.order.data_ptr(), R, host.n_nodes, ng,
        wp.beta, h.data_ptr(), 64, 64, out.data_ptr(), 64, sp))
    print(f"beta {wp.beta} nnz {len(ci)}", flush=True)
    flags = [int(f, 0) for f in args.flags.split(",")]
    ref = None
    res = {f: [] for f in flags}
    for rnd in range(args.rounds):
        for f in flags:
            _lib.check(L.snd_debug_set(f))
            ms = bench.time_launches(run, 10)
            res[f].append(ms)
            if rnd == 0:
                torch.cuda.synchronize()
                o = out.float()
                if ref is None:
                    ref = o.clone()
                print(f"flags {f}: max |out - out(flags {flags[0]})| = {float((o - ref).abs().max()):.3e}",
                      flush=True)
    _lib.check(L.snd_debug_set(0))
    for f in flags:
        t = sorted(res[f])
        print(f"flags {f:>9d}: median {t[len(t) // 2] * 1e3:7.2f} us  min {t[0] * 1e3:7.2f} us  "
              f"{byts / (t[len(t) // 2] * 1e-3) / 8e12:.4f} of 8 TB/s")


if __name__ == "__main__":
    main()
