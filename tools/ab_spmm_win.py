"""A/B the window SpMM (snd_csr_spmm_bf16_window_ring) on bench.py's 256-graph batch under
snd_debug_set flags and LDS rings, alternating the variants within one process (HIP events).

    python tools/ab_spmm_win.py --flags 0,524288 --rings 1096,1024 --rounds 4
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
    ap.add_argument("--rings", default="1096")
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
    rings = [int(r) for r in args.rings.split(",")]
    plans = {r: window_plan(big, order, r) for r in rings}
    dws = {r: DeviceWindowPlan(p) for r, p in plans.items()}
    h = torch.randn(R, 64, device="cuda").to(torch.bfloat16)
    out = torch.empty_like(h)
    L = _lib.lib()
    ng = host.n_graphs * c
    byts = 4 * (R + 1) + 4 * len(ci) + 2 * 2 * R * 64

    def runner(r):
        dw, wp = dws[r], plans[r]
        return lambda sp: _lib.check(L.snd_csr_spmm_bf16_window_ring(
            dw.meta.data_ptr(), dw.slots.data_ptr(), dw.rows.data_ptr(), dw.order.data_ptr(), R, host.n_nodes, ng,
            wp.beta, h.data_ptr(), 64, 64, out.data_ptr(), 64, r, sp))
    print(f"beta {plans[rings[0]].beta}", flush=True)
    flags = [int(f, 0) for f in args.flags.split(",")]
    variants = [(r, f) for r in rings for f in flags]
    ref = None
    res = {v: [] for v in variants}
    for rnd in range(args.rounds):
        for r, f in variants:
            _lib.check(L.snd_debug_set(f))
            ms = bench.time_launches(runner(r), 10)
            res[(r, f)].append(ms)
            if rnd == 0:
                torch.cuda.synchronize()
                o = out.float()
                if ref is None:
                    ref = o.clone()
                print(f"ring {r} flags {f}: max |out - out(first variant)| = {float((o - ref).abs().max()):.3e}",
                      flush=True)
    _lib.check(L.snd_debug_set(0))
    for r, f in variants:
        t = sorted(res[(r, f)])
        print(f"ring {r} flags {f:>9d}: median {t[len(t) // 2] * 1e3:7.2f} us  min {t[0] * 1e3:7.2f} us  "
              f"{byts / (t[len(t) // 2] * 1e-3) / 8e12:.4f} of 8 TB/s")


if __name__ == "__main__":
    main()
