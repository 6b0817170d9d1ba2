"""Launch only the fused zz^T + CE kernel (after one full step) for profiling.

    rocprofv3 --kernel-trace --stats -- python tools/prof_zzt.py [--reps 50]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--graphs", type=int, default=8)
    ap.add_argument("--nodes", type=int, default=4096)
    ap.add_argument("--latent", type=int, default=64)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--kernel", default="zzt_dense")
    args = ap.parse_args()
    import torch
    from snd_vae_amd import _lib
    from snd_vae_amd.config import tscale
    from snd_vae_amd.data import synthetic_batch
    from snd_vae_amd.model import DeviceBatch, SGCNModelVAE
    from snd_vae_amd.optimizer import OptimizerVAE
    cfg = tscale(args.nodes, args.latent)
    db = DeviceBatch(synthetic_batch(cfg, args.graphs, seed=1000))
    model = SGCNModelVAE(cfg, args.graphs, dtype=args.dtype)
    opt = OptimizerVAE(model)
    opt.step(db)
    bc = db.c_struct()
    L = _lib.lib()
    for _ in range(args.reps):
        _lib.check(L.snd_plan_launch(model.plan, bc, model.workspace.data_ptr(),
                                     args.kernel.encode(), _lib.stream_ptr()))
    torch.cuda.synchronize()
    print("ok", args.kernel, args.reps)


if __name__ == "__main__":
    main()
