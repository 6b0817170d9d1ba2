import sys, numpy as np, torch
sys.path.insert(0, '/root/repo')
from snd_vae_amd.config import tref
from snd_vae_amd.data import synthetic_batch
from snd_vae_amd.params import init_blocks
from snd_vae_amd.model import DeviceBatch, SGCNModelVAE
from snd_vae_amd.optimizer import OptimizerVAE
cfg = tref(1024, 64); batch = synthetic_batch(cfg, 2, seed=4); p0 = init_blocks(cfg, 0)
res = {}
for fuse in (False, True, False, True):
    m = SGCNModelVAE(cfg, 2, dtype="bf16", blocks=p0); o = OptimizerVAE(m, fuse_adam=fuse); b = DeviceBatch(batch)
    for _ in range(3): o.step(b)
    torch.cuda.synchronize()
    pb = m.blocks()
    if fuse in res:
        print("fuse", fuse, "repeat bitwise:", all(np.array_equal(pb[k], res[fuse][k]) for k in pb))
    else:
        res[fuse] = pb
d = {k: float(np.abs(res[False][k] - res[True][k]).max()) for k in res[False]}
print(sorted(d.items(), key=lambda kv: -kv[1])[:6])
