"""A/B of the window SpMM on the bench's 256-graph batch under measurement-only
skip bits (snd_debug_set(bits << 16)): 1 no sums, 2 no window DMA, 4 no slot DMA,
8 neighbour groups of 8 instead of 4.  A flag with a trailing "p" runs the pair-sum
kernel (snd_csr_spmm_bf16_window_pairs, plan window_plan_pairs).

    python tools/ab_spmm_win.py [--flags 0,1,2,4,3,0p,1p] [--check]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--flags", default="0,8,1,2,4,6")
    ap.add_argument("--copies", type=int, default=32)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--check", action="store_true")
    args = ap.parse_args()
    import numpy as np
    import torch
    import bench
    from snd_vae_amd import _lib
    from snd_vae_amd.config import tscale
    from snd_vae_amd.data import GraphBatch, locality_order, synthetic_batch, window_plan, window_plan_pairs
    from snd_vae_amd.layers import DeviceWindowPlan
    host = synthetic_batch(tscale(4096, 64), 8, seed=0)
    rp0, ci0 = host.rowptr.astype(np.int64), host.colidx.astype(np.int64)
    nnz0, R0 = int(rp0[-1]), host.n_graphs * host.n_nodes
    c = args.copies
    rp = np.concatenate([rp0[:-1] + k * nnz0 for k in range(c)] + [np.array([c * nnz0])])
    ci = np.concatenate([ci0 + k * R0 for k in range(c)])
    o0 = locality_order(host).astype(np.int64)
    order = np.concatenate([o0 + k * R0 for k in range(c)]).astype(np.int32)
    z = np.zeros((1, 1), np.float32)
    big = GraphBatch(host.n_graphs * c, host.n_nodes, rp.astype(np.int32), ci.astype(np.int32), z, z, z)
    toks = args.flags.split(",")
    wp = window_plan(big, order)
    plans = {False: (wp, DeviceWindowPlan(wp))}
    if any(t.endswith("p") for t in toks):
        wpp = window_plan_pairs(big, order)
        plans[True] = (wpp, DeviceWindowPlan(wpp))

    def launch(pairs, sp):
        w, d = plans[pairs]
        fn = L.snd_csr_spmm_bf16_window_pairs if pairs else L.snd_csr_spmm_bf16_window
        _lib.check(fn(d.meta.data_ptr(), d.slots.data_ptr(), d.rows.data_ptr(), d.order.data_ptr(), R, host.n_nodes,
                      ng, w.beta, h.data_ptr(), 64, 64, out.data_ptr(), 64, sp))
    R, ng = R0 * c, host.n_graphs * c
    h = torch.randn(R, 64, device="cuda").to(torch.bfloat16)
    out = torch.empty_like(h)
    L = _lib.lib()
    byts = 4 * (R + 1) + 4 * len(ci) + 2 * 2 * R * 64
    if args.check:   # every flag's output against the register-gather kernel (fp32 sums in colidx order)
        from snd_vae_amd import layers
        ref = layers.spmm_bf16(torch.from_numpy(rp.astype(np.int32)).cuda(), torch.from_numpy(ci.astype(np.int32)).cuda(),
                               h, host.n_nodes, ng, torch.from_numpy(order).cuda())
        for t in toks:
            f = int(t.rstrip("p"))
            _lib.check(L.snd_debug_set(f << 16))
            out.zero_()
            launch(t.endswith("p"), _lib.stream_ptr())
            torch.cuda.synchronize()
            neq = int((out.view(torch.int16) != ref.view(torch.int16)).sum())
            d = (out.float() - ref.float()).abs()
            print(f"check {t}: {neq} of {out.numel()} bf16 outputs differ, max |diff| {float(d.max()):.3e}, "
                  f"max |ref| {float(ref.float().abs().max()):.3e}", flush=True)
        _lib.check(L.snd_debug_set(0))
    for t in toks:
        _lib.check(L.snd_debug_set(int(t.rstrip("p")) << 16))
        ms = bench.time_launches(lambda sp: launch(t.endswith("p"), sp), args.reps)
        print(f"skip {t}: {ms * 1e3:8.1f} us  {byts / (ms * 1e-3) / 1e12:5.2f} TB/s algorithmic", flush=True)
    _lib.check(L.snd_debug_set(0))


if __name__ == "__main__":
    main()
