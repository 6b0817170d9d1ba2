"""The bucketed data-parallel step (parallel.run_buckets via OptimizerVAE) on one GPU.

An RCCL process group of one rank runs the N > 1 code path: the step records the
graph-latent gradient completion events (snd_plan_grad_event), the early buckets'
collectives and Adam run on the communication stream while the backward pass goes
on, the large buckets are reduce-scattered, updated as shards and all-gathered.  At
world 1 every collective is an identity, so the parameters, Adam moments and loss
terms must equal those of the unbucketed distributed step (one all-reduce, one Adam
pass) bit for bit, eagerly and under HIP-graph replay -- a bucket started before its
gradient is complete, or an update racing the backward kernels, shows up as a
difference.  The sharding arithmetic at world 2 is tests/test_dist_cpu.py's.
"""
import os
import socket

import pytest
import torch

from snd_vae_amd.config import tref
from snd_vae_amd.data import synthetic_batch
from snd_vae_amd.params import init_blocks

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pg(lib_built):
    import torch.distributed as dist
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm device")
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    torch.cuda.set_device(0)
    own = not dist.is_initialized()
    if own:
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                                device_id=torch.device("cuda", 0))
    yield dist.group.WORLD
    if own:
        dist.destroy_process_group()


def _state(m, o):
    pc = m.param_count
    return [t[:pc].clone() for t in (m.params, o.m, o.v)] + [o.grads[pc:pc + 8].clone()]


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_bucketed_step_equals_single_allreduce(pg, dtype):
    from snd_vae_amd.model import DeviceBatch, SGCNModelVAE
    from snd_vae_amd.optimizer import OptimizerVAE
    cfg = tref(256, 16)
    B = 4
    batch = synthetic_batch(cfg, B, seed=5)
    p0 = init_blocks(cfg, 2)
    ma = SGCNModelVAE(cfg, B, dtype=dtype, blocks=p0)
    oa = OptimizerVAE(ma, process_group=pg, bucketed=True, shard_min=1024)
    mb = SGCNModelVAE(cfg, B, dtype=dtype, blocks=p0)
    ob = OptimizerVAE(mb, process_group=pg, bucketed=False)
    assert [(b.point, b.sharded) for b in oa.buckets][:2] == [(1, True), (2, True)]
    assert sorted(oa._events) == [1, 2] and oa._comm is not None
    db = DeviceBatch(batch)
    for _ in range(2):
        oa.step(db)
        ob.step(db)
    torch.cuda.synchronize()
    for x, y in zip(_state(ma, oa), _state(mb, ob)):
        assert torch.equal(x, y)
    oa.capture(db)
    ob.capture(db)
    for _ in range(3):
        oa.replay()
        ob.replay()
    torch.cuda.synchronize()
    for x, y in zip(_state(ma, oa), _state(mb, ob)):
        assert torch.equal(x, y)
    assert oa.global_step == ob.global_step == 5
    oa.sync_state()                       # world 1: the gathered moments are the moments
    assert torch.equal(oa.m[:ma.param_count], ob.m[:mb.param_count])


def test_c2_distributed_is_one_allreduce(pg):
    """The node-latent C2 plan has no early points and no large blocks: the bucketed
    exchange is exactly the one all-reduce of the gradient and the loss terms."""
    from snd_vae_amd.config import tscale
    from snd_vae_amd.model import SGCNModelVAE
    from snd_vae_amd.optimizer import OptimizerVAE
    m = SGCNModelVAE(tscale(4096, 64), 8, dtype="bf16")
    o = OptimizerVAE(m, process_group=pg, bucketed=True)
    assert [(b.lo, b.hi, b.point, b.sharded) for b in o.buckets] == [(0, m.param_count + 8, 0, False)]
    assert o._comm is None


def test_rebinding_bucketed_optimizer_keeps_events(pg):
    """`opt = OptimizerVAE(model, pg, bucketed=True)` twice on one model -- the
    old optimizer's __del__ runs after the new one registered its completion events and
    must not unregister them (snd_plan_grad_event_get reads what the plan holds)."""
    import ctypes as C
    import gc

    from snd_vae_amd import _lib
    from snd_vae_amd.model import SGCNModelVAE
    from snd_vae_amd.optimizer import OptimizerVAE
    cfg = tref(256, 16)
    m = SGCNModelVAE(cfg, 4, dtype="f32")
    L = _lib.lib()

    def held():
        out = {}
        for i in range(len(m.layout.shapes)):
            ev = C.c_void_p()
            pt = L.snd_plan_grad_event_get(m.plan, i, C.byref(ev))
            assert pt >= 0, _lib.last_error()
            if pt:
                out[i] = (pt, ev.value)
        return out

    opt = OptimizerVAE(m, process_group=pg, bucketed=True, shard_min=1024)
    first = held()
    assert first and all(v for _, v in first.values())
    opt = OptimizerVAE(m, process_group=pg, bucketed=True, shard_min=1024)   # rebinding frees the first
    gc.collect()
    now = held()
    assert {i: v for i, (_, v) in now.items()} == {i: opt._events[pt].cuda_event for i, (pt, _) in now.items()}
    opt.close()
    assert all(v is None for _, v in held().values())
