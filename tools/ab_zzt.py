"""Interleaved in-process A/B timing of the zz^T kernel variants (HIP events).

    python tools/ab_zzt.py [--rounds 5 --reps 20]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--graphs", type=int, default=8)
    ap.add_argument("--nodes", type=int, default=4096)
    ap.add_argument("--latent", type=int, default=64)
    ap.add_argument("--variants", default="zzt_dense,zzt_dense_v1")
    args = ap.parse_args()
    import torch
    from snd_vae_amd import _lib
    from snd_vae_amd.config import tscale
    from snd_vae_amd.data import synthetic_batch
    from snd_vae_amd.model import DeviceBatch, SGCNModelVAE
    from snd_vae_amd.optimizer import OptimizerVAE
    cfg = tscale(args.nodes, args.latent)
    db = DeviceBatch(synthetic_batch(cfg, args.graphs, seed=1000))
    model = SGCNModelVAE(cfg, args.graphs, dtype="bf16")
    opt = OptimizerVAE(model)
    for _ in range(3):
        opt.step(db)
    bc = db.c_struct()
    L = _lib.lib()
    names = args.variants.split(",")
    res = {n: [] for n in names}
    pz = model.buffer("PZZT", torch.float64)
    djd = model.buffer("DJD")
    outs = {}
    for rnd in range(args.rounds):
        for n in names:
            st = _lib.stream_ptr()
            _lib.check(L.snd_plan_launch(model.plan, bc, model.workspace.data_ptr(), n.encode(), st))
            if rnd == 0:
                torch.cuda.synchronize()
                outs[n] = (pz.view(-1, 2).sum(0).cpu().numpy(), djd.clone())
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                _lib.check(L.snd_plan_launch(model.plan, bc, model.workspace.data_ptr(), n.encode(), st))
            e1.record()
            e1.synchronize()
            res[n].append(e0.elapsed_time(e1) / args.reps)
    flops = 4.0 * args.nodes ** 2 * args.latent * args.graphs
    ref = outs[names[-1]]
    for n in names:
        t = sorted(res[n])
        s, d = outs[n]
        dd = (d - ref[1]).abs().max().item() / ref[1].abs().max().item()
        print(f"{n:16s} median {t[len(t)//2]*1e3:8.2f} us  min {t[0]*1e3:8.2f} us  "
              f"{flops / (t[len(t)//2] * 1e-3) / 1e12:7.1f} TF/s  loss {s[0]:.6e} cnt {s[1]:.0f}  "
              f"dJ rel-diff vs {names[-1]} {dd:.2e}")


if __name__ == "__main__":
    main()
