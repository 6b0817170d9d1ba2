"""Diagnose the fp32 C2 step-3 gradient gap on dec.K1 / dec.b1 / dec.bn1.beta.

Runs tests/test_gpu_c2_bench.py's fp32 sequence (the bench batch, init seed 0, eps seed
9, reduce-fused Adam) and, at each step, compares the GPU's decoder layer-1 pre-activation
T1 = BN(Y1) (generic engine buffer Y1, fp32) with the float64 oracle's, lists the elements
whose lrelu derivative differs (T >= 0 on one side only), and checks whether those flips
alone explain the gradient gap: the predicted change of dec.b1 from the flipped elements
(dU1 (lrelu'_gpu - lrelu'_ref) gamma c, summed per column) against the observed GPU -
oracle difference.  One JSON line per step.

    python tools/diag_kink.py > gpurun_out/diag_kink.jsonl
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import torch
    from oracle import ref_numpy as R
    from snd_vae_amd.config import tscale
    from snd_vae_amd.data import synthetic_batch
    from snd_vae_amd.model import DeviceBatch, SGCNModelVAE
    from snd_vae_amd.optimizer import OptimizerVAE
    from snd_vae_amd.params import init_blocks
    cfg = tscale(4096, 64)
    B, n = 8, 4096
    batch = synthetic_batch(cfg, B, seed=1000)
    adj = [batch.sparse_adj(b) for b in range(B)]
    p0 = {k: v.astype(np.float32).astype(np.float64) for k, v in init_blocks(cfg, 0).items()}
    rng = np.random.default_rng(9)
    eps = [rng.standard_normal((B * n, cfg.latent)).astype(np.float32) for _ in range(3)]
    model = SGCNModelVAE(cfg, B, dtype="f32", blocks=p0)
    opt = OptimizerVAE(model)
    db = DeviceBatch(batch)
    C1 = cfg.s_d_channel[0] + cfg.n_d_channel[0]
    c = R.BN_C
    for t in range(1, 4):
        p = {k: np.asarray(v, np.float64) for k, v in model.blocks().items()}
        opt.step(db, torch.from_numpy(eps[t - 1]).cuda())
        torch.cuda.synchronize()
        y1 = model.buffer("Y1")[:B * n * C1].view(B * n, C1).double().cpu().numpy()
        du1 = model.buffer("DU1")[:B * n * C1].view(B * n, C1).double().cpu().numpy()
        gg = {k: np.asarray(x, np.float64) for k, x in opt.grad_blocks().items()}
        _, rg, cache = R.forward_backward(p, adj, batch.features, batch.feature_truth, batch.spatial_truth,
                                          eps[t - 1].astype(np.float64), cfg, row_chunk=1024)
        gam, bet = p["dec.bn1.gamma"] * c, p["dec.bn1.beta"]
        t_ref = cache["Y1"] * gam + bet
        t_gpu = y1 * gam + bet
        flip = (t_ref >= 0) != (t_gpu >= 0)
        rows, cols = np.nonzero(flip)
        scale = np.abs(t_ref).max()
        d_gpu = np.where(t_gpu >= 0, 1.0, 0.2)
        d_ref = np.where(t_ref >= 0, 1.0, 0.2)
        pred_db = ((d_gpu - d_ref) * du1 * gam).sum(0)           # predicted dec.b1 change
        obs_db = gg["dec.b1"] - rg["dec.b1"]
        mx = np.abs(rg["dec.b1"]).max()
        rec = {"step": t, "flips": int(flip.sum()),
               "flip_elems": [{"row": int(r), "col": int(cc), "T_ref": float(t_ref[r, cc]),
                               "T_gpu": float(t_gpu[r, cc]), "T_rel": float(abs(t_ref[r, cc]) / scale),
                               "dU1": float(du1[r, cc])} for r, cc in list(zip(rows, cols))[:8]],
               "y1_max_rel_err": float(np.abs(y1 - cache["Y1"]).max() / np.abs(cache["Y1"]).max()),
               "db1_err_rel": float(np.abs(obs_db).max() / mx),
               "db1_err_after_flips_rel": float(np.abs(obs_db - pred_db).max() / mx),
               "dK1_err_rel": float(np.abs(gg["dec.K1"] - rg["dec.K1"]).max() / np.abs(rg["dec.K1"]).max())}
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
