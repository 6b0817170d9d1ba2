"""Phase timeline of the v4 zz^T kernel from its measurement-only s_memrealtime stamps
(variant bit 32 << 8): per workgroup start, prologue, tile loop, corrections + stores.

    python tools/zzt_stamps.py [--skip 0]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--skip", type=int, default=0)
    args = ap.parse_args()
    import numpy as np
    import torch
    from snd_vae_amd import _lib
    from snd_vae_amd.config import tscale
    from snd_vae_amd.data import synthetic_batch
    from snd_vae_amd.model import DeviceBatch, SGCNModelVAE
    from snd_vae_amd.optimizer import OptimizerVAE
    cfg = tscale(4096, 64)
    db = DeviceBatch(synthetic_batch(cfg, 8, seed=1000))
    model = SGCNModelVAE(cfg, 8, dtype="bf16")
    opt = OptimizerVAE(model)
    opt.step(db)
    bc = db.c_struct()
    L = _lib.lib()
    name = f"zzt_dense_v{(32 | args.skip) << 8}".encode()
    for _ in range(5):
        _lib.check(L.snd_plan_launch(model.plan, bc, model.workspace.data_ptr(), name, _lib.stream_ptr()))
    torch.cuda.synchronize()
    nb = 256
    raw = model.buffer("PZZT", torch.float64).view(torch.int32)[:4 * nb].cpu().numpy().astype(np.int64)
    st = (raw & 0xFFFFFFFF).reshape(nb, 4).astype(np.float64)
    t0 = st[:, 0].min()
    rel = (st - t0) * 0.01   # 100 MHz ticks -> us
    names = ["start", "prologue done", "loop done", "end"]
    for k, n in enumerate(names):
        c = rel[:, k]
        print(f"{n:16s} min {c.min():7.2f}  median {np.median(c):7.2f}  max {c.max():7.2f} us")
    name = f"zzt_dense_v{(32 | 128 | args.skip) << 8}".encode()
    for _ in range(3):
        _lib.check(L.snd_plan_launch(model.plan, bc, model.workspace.data_ptr(), name, _lib.stream_ptr()))
    torch.cuda.synchronize()
    rc = model.buffer("PZZT", torch.float64).view(torch.int32)[:4 * nb].cpu().numpy().astype(np.int64)
    rc = (rc & 0xFFFFFFFF).reshape(nb, 4)
    us = ((rc[:, 1] - rc[:, 0]) % 2**32) * 0.01
    cyc = ((rc[:, 3] - rc[:, 2]) % 2**32).astype(np.float64)
    print(f"tile loop: median {np.median(cyc):.0f} shader cycles in {np.median(us):.2f} us "
          f"-> clock {np.median(cyc / us) / 1e3:.3f} GHz")
    d = np.diff(rel, axis=1)
    for k in range(3):
        print(f"phase {names[k]:>16s} -> {names[k+1]:16s} median {np.median(d[:, k]):7.2f}  max {d[:, k].max():7.2f} us")


if __name__ == "__main__":
    main()
