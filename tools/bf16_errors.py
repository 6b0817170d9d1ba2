"""Per-block gradient error of the bf16 step vs the float64 oracle, for the
fast path (default), fast decoder + generic encoder (512) and the generic
engine (256).  Measurement aid for tolerance decisions."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np


def main():
    import torch
    from oracle import ref_numpy as R
    from snd_vae_amd import _lib
    from snd_vae_amd.config import tscale
    from snd_vae_amd.data import synthetic_batch
    from snd_vae_amd.model import DeviceBatch, SGCNModelVAE
    from snd_vae_amd.optimizer import OptimizerVAE
    from snd_vae_amd.params import init_blocks
    for n, d, B in ((200, 16, 4), (4096, 64, 1)):
        cfg = tscale(n, d)
        batch = synthetic_batch(cfg, B, seed=0)
        p0 = {k: v.astype(np.float32).astype(np.float64) for k, v in init_blocks(cfg, 0).items()}
        eps = np.random.default_rng(9).standard_normal((B * n, d)).astype(np.float32)
        adj = [batch.dense_adj(b) for b in range(B)]
        ref, rg, _ = R.forward_backward(p0, adj, batch.features, batch.feature_truth,
                                        batch.spatial_truth, eps.astype(np.float64), cfg)
        res = {}
        for flag in (0, 512, 256):
            _lib.check(_lib.lib().snd_debug_set(flag))
            model = SGCNModelVAE(cfg, B, dtype="bf16", blocks=p0)
            _lib.check(_lib.lib().snd_debug_set(0))
            opt = OptimizerVAE(model, fuse_adam=False)
            opt.forward_backward(DeviceBatch(batch), torch.from_numpy(eps).cuda())
            torch.cuda.synchronize()
            g = opt.grad_blocks()
            res[flag] = {k: np.linalg.norm(g[k] - rg[k]) / max(np.linalg.norm(rg[k]), 1e-30) for k in rg}
        print(f"N={n} d={d} B={B}: block  fast  fastdec  generic")
        for k in rg:
            print(f"  {k:18s} {res[0][k]:.4f} {res[512][k]:.4f} {res[256][k]:.4f}")


if __name__ == "__main__":
    main()
