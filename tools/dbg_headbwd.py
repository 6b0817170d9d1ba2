"""Debug: where the fused backward head and the chain differ (bf16 d[mu|s])."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from snd_vae_amd import _lib
from snd_vae_amd.config import tscale
from snd_vae_amd.data import synthetic_batch
from snd_vae_amd.model import DeviceBatch, SGCNModelVAE
from snd_vae_amd.optimizer import OptimizerVAE
from snd_vae_amd.params import init_blocks
n, d, B = [int(v) for v in sys.argv[1:4]]
cfg = tscale(n, d)
batch = synthetic_batch(cfg, B, seed=13)
p0 = init_blocks(cfg, 4)
runs = []
for flags in (262144, 0):
    _lib.check(_lib.lib().snd_debug_set(flags))
    m = SGCNModelVAE(cfg, B, dtype="bf16", blocks=p0); o = OptimizerVAE(m, fuse_adam=False)
    _lib.check(_lib.lib().snd_debug_set(0))
    o.forward_backward(DeviceBatch(batch)); torch.cuda.synchronize()
    runs.append((m, o))
R = B * n
a = runs[0][0].buffer("FDMS", torch.bfloat16)[:R * 2 * d].float().view(R, 2 * d).cpu().numpy()
b = runs[1][0].buffer("FDMS", torch.bfloat16)[:R * 2 * d].float().view(R, 2 * d).cpu().numpy()
diff = np.argwhere(a != b)
print("mismatches", len(diff), "of", a.size)
rows = np.unique(diff[:, 0]); cols = np.unique(diff[:, 1])
print("rows", rows[:20], len(rows)); print("cols", cols[:40])
deg = np.diff(batch.rowptr) if hasattr(batch, "rowptr") else None
if deg is not None: print("deg of rows", deg[rows[:20]], "max deg", deg.max())
for r, c in diff[:10]: print(r, c, a[r, c], b[r, c])
for nm in ("DJD", "DZDEC", "EPS", "MS"):
    x = runs[0][0].buffer(nm); y = runs[1][0].buffer(nm)
    print(nm, torch.equal(x, y))
