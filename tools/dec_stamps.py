"""Phase timelines of the fused step kernels from their measurement-only s_memrealtime
stamps (debug bit 1 << 21): per workgroup, the time at each phase boundary.

    python tools/dec_stamps.py [--graphs 8]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

KERNELS = {
    # key: (plan buffer, stride in 32-bit words per workgroup (dec:bwd: 3 x the 106-wide U1 layout), labels)
    "dec:fwd": ("PDHS", 52, ["start", "J+W1 staged", "conv1 done", "W2 staged", "conv2 done",
                             "W3 staged", "conv3 done", "head rows done", "partials done"]),
    "dec:bwd": ("PDC1", 3 * 106, ["start", "dY3+W3t staged", "conv3T done", "W2t staged", "conv2T done",
                               "W1t staged", "conv1T (wave 0)", "end"]),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--graphs", type=int, default=8)
    ap.add_argument("--keys", default="dec:fwd,dec:bwd")
    ap.add_argument("--flags", default="0", help="extra measurement-only debug bits, comma list (one run each)")
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
    # tile rows as snd_dec.hip dec_rows (default knobs): 128, 64 under 128 tiles, 32 under 128 of 64
    t128 = args.graphs * 4096 // 128
    rows = 128 if t128 >= 128 else (32 if 2 * t128 < 128 else 64)
    nb = args.graphs * 4096 // rows
    for key, fl in [(k, int(f, 0)) for k in args.keys.split(",") for f in args.flags.split(",")]:
        buf, stride, names = KERNELS[key]
        _lib.check(L.snd_debug_set((1 << 21) | fl))
        for _ in range(5):
            _lib.check(L.snd_plan_launch(model.plan, bc, model.workspace.data_ptr(), key.encode(), _lib.stream_ptr()))
        torch.cuda.synchronize()
        _lib.check(L.snd_debug_set(0))
        raw = model.buffer(buf, torch.float32).view(torch.int32)[:nb * stride].cpu().numpy().astype(np.int64)
        st = (raw.reshape(nb, stride)[:, :len(names)] & 0xFFFFFFFF).astype(np.float64)
        rel = (st - st[:, 0].min()) * 0.01   # 100 MHz ticks -> us
        print(f"== {key} flags {fl} ({nb} workgroups)")
        for k, n in enumerate(names):
            c = rel[:, k]
            print(f"  {n:18s} min {c.min():7.2f}  median {np.median(c):7.2f}  max {c.max():7.2f} us")
        d = np.diff(rel, axis=1)
        for k in range(len(names) - 1):
            print(f"  {names[k]:>18s} -> {names[k + 1]:18s} median {np.median(d[:, k]):6.2f}  max {d[:, k].max():6.2f}")


if __name__ == "__main__":
    main()
