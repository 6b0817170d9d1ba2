"""Diagnostic: the first Adam update per block at the C4 bench shape, bf16 vs f32.

After one step from p0 with zero moments, TF1 Adam moves every parameter by
-lr * m / (sqrt(v) + eps) ~ -lr * sign(g): prints, per block, the fraction of
elements whose move agrees with -sign(m), the median |move| / lr, and how the bf16
run's moves and moments compare with the f32 run's."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from snd_vae_amd.config import tref
    from snd_vae_amd.data import synthetic_batch
    from snd_vae_amd.model import DeviceBatch, SGCNModelVAE
    from snd_vae_amd.optimizer import OptimizerVAE
    from snd_vae_amd.params import init_blocks
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    cfg = tref(n, 64)
    batch = synthetic_batch(cfg, B, seed=1000)
    p0 = {k: v.astype(np.float32).astype(np.float64) for k, v in init_blocks(cfg, 0).items()}
    eps = np.random.default_rng(9).standard_normal((B, cfg.latent)).astype(np.float32)
    res = {}
    for dtype in ("f32", "bf16"):
        m = SGCNModelVAE(cfg, B, dtype=dtype, blocks=p0)
        o = OptimizerVAE(m, fuse_adam=True)
        before = m.blocks()
        o.step(DeviceBatch(batch), torch.from_numpy(eps).cuda())
        torch.cuda.synchronize()
        after = m.blocks()
        mm, vv = o.state_blocks()
        res[dtype] = (before, after, mm, vv)
        del m, o
    for k in ("enc.W0", "enc.W1", "enc.Wh", "enc.Wms", "dec.Wp", "dec.K1"):
        line = [k]
        for dtype in ("f32", "bf16"):
            b, a, mm, vv = res[dtype]
            d = (np.asarray(a[k], np.float64) - np.asarray(b[k], np.float64)) / cfg.learning_rate
            line.append(f"{dtype}: agree {np.mean(np.sign(d) == -np.sign(mm[k])):.3f} |d| {np.median(np.abs(d)):.3f} "
                        f"p0diff {np.abs(np.asarray(b[k], np.float64) - p0[k]).max():.2e}")
        b32, a32, m32, _ = res["f32"]
        b16, a16, m16, _ = res["bf16"]
        line.append(f"sign(m) agree {np.mean(np.sign(m16[k]) == np.sign(m32[k])):.4f} "
                    f"p1 diff/lr max {np.abs(np.asarray(a16[k]) - np.asarray(a32[k])).max() / cfg.learning_rate:.3f} "
                    f"|m| max {np.abs(m32[k]).max():.3e} median {np.median(np.abs(m32[k])):.3e}")
        print(" | ".join(line), flush=True)


if __name__ == "__main__":
    main()
