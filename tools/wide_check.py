"""Per-block bf16 gradient errors of one step against the float64 oracle under several
snd_debug_set flags (plan-time engine choices), for a tscale(n, d) batch.

    python tools/wide_check.py --n 512 --d 128 --graphs 2 --flags 0,524288,256
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--d", type=int, default=128)
    ap.add_argument("--graphs", type=int, default=2)
    ap.add_argument("--seed", type=int, default=552)
    ap.add_argument("--flags", default="0")
    ap.add_argument("--dtype", default="bf16")
    args = ap.parse_args()
    import numpy as np
    import torch
    from oracle import ref_numpy as R
    from snd_vae_amd import _lib
    from snd_vae_amd.config import tscale
    from snd_vae_amd.data import synthetic_batch
    from snd_vae_amd.model import DeviceBatch, SGCNModelVAE
    from snd_vae_amd.optimizer import OptimizerVAE
    from snd_vae_amd.params import init_blocks
    cfg = tscale(args.n, args.d)
    B = args.graphs
    batch = synthetic_batch(cfg, B, seed=args.seed)
    p0 = {k: v.astype(np.float32).astype(np.float64) for k, v in init_blocks(cfg, 0).items()}
    eps = np.random.default_rng(9).standard_normal((B * args.n, args.d)).astype(np.float32)
    adj = [batch.sparse_adj(b) for b in range(B)]
    ref, rg, _ = R.forward_backward(p0, adj, batch.features, batch.feature_truth, batch.spatial_truth,
                                    eps.astype(np.float64), cfg, row_chunk=1024, amb_tol=1e-4)
    for f in [int(x) for x in args.flags.split(",")]:
        _lib.check(_lib.lib().snd_debug_set(f))
        model = SGCNModelVAE(cfg, B, dtype=args.dtype, blocks=p0)
        opt = OptimizerVAE(model, fuse_adam=False)
        opt.step(DeviceBatch(batch), torch.from_numpy(eps).cuda())
        torch.cuda.synchronize()
        _lib.check(_lib.lib().snd_debug_set(0))
        g = opt.grad_blocks()
        errs = {k: np.abs(g[k] - rg[k]).max() / max(np.abs(rg[k]).max(), 1e-30) for k in rg}
        worst = sorted(errs.items(), key=lambda kv: -kv[1])[:6]
        ld = opt.loss_dict()
        print(f"flags {f}: cost {ld['cost']:.6f} (ref {ref['cost']:.6f}) worst "
              + ", ".join(f"{k} {v:.4f}" for k, v in worst), flush=True)
        del model, opt
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
