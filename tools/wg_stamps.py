"""Per-workgroup phase timeline of wgrad_multi from its measurement-only s_memrealtime
stamps (debug bit 1 << 21, a -DSND_MEAS=1 library through SND_LIB_PATH): for every
workgroup the start, the segment/argument load, the prologue, each 128-row unit's
barrier and the end, with the CU (HW_ID, XCC_ID) it ran on.

    SND_LIB_PATH=ab/meas.so python tools/wg_stamps.py
"""
import argparse
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--graphs", type=int, default=8)
    ap.add_argument("--flags", default="0", help="extra measurement-only debug bits, comma list")
    ap.add_argument("--per-seg", default="64",
                    help="items per segment (C2: 64 row chunks), or a comma list, one count per segment")
    args = ap.parse_args()
    import numpy as np
    import torch
    from snd_vae_amd import _lib
    from snd_vae_amd.config import tscale
    from snd_vae_amd.data import synthetic_batch
    from snd_vae_amd.model import DeviceBatch, SGCNModelVAE
    from snd_vae_amd.optimizer import OptimizerVAE
    cfg = tscale(4096, 64)
    db = DeviceBatch(synthetic_batch(cfg, args.graphs, seed=1000))
    model = SGCNModelVAE(cfg, args.graphs, dtype="bf16")
    opt = OptimizerVAE(model)
    opt.step(db)
    torch.cuda.synchronize()
    bc = db.c_struct()
    L = _lib.lib()
    buf = model.buffer("PDHS", torch.float32).view(torch.int32)
    for fl in [int(f, 0) for f in args.flags.split(",")]:
        _lib.check(L.snd_debug_set((1 << 21) | fl))
        for _ in range(5):
            buf.zero_()
            _lib.check(L.snd_plan_launch(model.plan, bc, model.workspace.data_ptr(), b"wgrad_multi",
                                         _lib.stream_ptr()))
        torch.cuda.synchronize()
        _lib.check(L.snd_debug_set(0))
        raw = (buf.cpu().numpy().astype(np.int64) & 0xFFFFFFFF)
        n = len(raw) // 12
        st = raw[:n * 12].reshape(n, 12)
        st = st[st[:, 9] != 0]
        nwg = len(st)
        t = st[:, :10].astype(np.float64)
        t0 = t[:, 0].min()
        rel = np.where(t > 0, (t - t0) * 0.01, np.nan)   # 100 MHz ticks -> us
        print(f"== wgrad_multi flags {fl}: {nwg} workgroups, span {np.nanmax(rel[:, 9]):.2f} us")
        names = ["start", "args", "prologue", "u0", "u1", "u2", "u3", "u4", "u5", "end"]
        for k, nm in enumerate(names):
            c = rel[:, k]
            if np.all(np.isnan(c)):
                continue
            print(f"  {nm:9s} min {np.nanmin(c):7.2f}  median {np.nanmedian(c):7.2f}  max {np.nanmax(c):7.2f} us")
        # per-workgroup phase durations (consecutive stamps present)
        seq = [0, 1, 2, 3, 4, 5, 6, 7, 8, 9]
        for a_, b_ in zip(seq[:-1], seq[1:]):
            d = rel[:, b_] - rel[:, a_]
            d = d[~np.isnan(d)]
            if len(d):
                print(f"  {names[a_]:>9s} -> {names[b_]:9s} median {np.median(d):6.2f}  p90 {np.percentile(d, 90):6.2f}  n {len(d)}")
        # per segment (items are numbered segment-major; --per-seg items per segment)
        idx = np.nonzero(raw[:n * 12].reshape(n, 12)[:, 9] != 0)[0]
        ps = [int(v) for v in args.per_seg.split(",")]
        seg = idx // ps[0] if len(ps) == 1 else np.searchsorted(np.cumsum(ps), idx, side="right")
        for sg in np.unique(seg):
            m = seg == sg
            lf = rel[m, 9] - rel[m, 0]
            u = rel[m, 6] - rel[m, 3]
            print(f"  segment {int(sg):2d}: {int(m.sum())} wg, start median {np.median(rel[m, 0]):6.2f}, "
                  f"lifetime median {np.median(lf):6.2f} max {lf.max():6.2f}, units u0->u3 median {np.nanmedian(u):5.2f} us")
        life = rel[:, 9] - rel[:, 0]
        print(f"  lifetime median {np.median(life):.2f}  p10 {np.percentile(life, 10):.2f}  p90 {np.percentile(life, 90):.2f} us")
        # per CU: workgroups and the idle gaps between one workgroup's end and the next start
        hw, xcc = st[:, 10], st[:, 11]
        cu = (xcc & 0xF) * 4096 + ((hw >> 13) & 7) * 512 + ((hw >> 12) & 1) * 256 + ((hw >> 8) & 15)
        per = collections.defaultdict(list)
        for i in range(nwg):
            per[int(cu[i])].append((rel[i, 0], rel[i, 9]))
        cnt = collections.Counter(len(v) for v in per.values())
        print(f"  CUs used {len(per)}; workgroups per CU: {dict(sorted(cnt.items()))}")
        conc = []
        for v in per.values():
            v.sort()
            # max overlap on the CU
            ev = sorted([(s, 1) for s, _ in v] + [(e, -1) for _, e in v])
            c = m = 0
            for _, dlt in ev:
                c += dlt
                m = max(m, c)
            conc.append(m)
        print(f"  max concurrent workgroups per CU: {dict(sorted(collections.Counter(conc).items()))}")
        busy = [max(e for _, e in v) - min(s for s, _ in v) for v in per.values()]
        print(f"  CU busy span median {np.median(busy):.2f} max {np.max(busy):.2f} us")


if __name__ == "__main__":
    main()
