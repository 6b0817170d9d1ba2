"""OptimizerVAE on MI355X: ELBO terms, gradients and the TF1-Adam step.

Mirror of `optimizer.py:123-203` (``OptimizerVAE``, model_type 'base'):
``cost``/``overall_loss`` = [cost, spatial_cost, adj_cost, node_cost, kl]
(`optimizer.py:203`) plus the accuracy of `main.py:334`.  One ``step()`` is
one iteration of the reference train loop (`main.py:315-334`):

    snd_train_step   forward + backward, flat gradient, loss terms
    exchange         (data parallel only) RCCL over the gradient buckets
                     (parallel.plan_buckets): early buckets overlap the backward
                     pass on a communication stream, large ones are
                     reduce-scattered, updated as shards and all-gathered
    snd_adam_tf1     tf.train.AdamOptimizer(lr).minimize (`optimizer.py:125,197`)

All three are stream-ordered device work, so a step can be captured in a
HIP graph (``capture()``) and replayed with no host involvement; the loss
terms stay on the device until ``overall_loss`` is read.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional

import numpy as np
import torch

from . import _lib
from .model import TAIL, DeviceBatch, SGCNModelVAE

LOSS_NAMES = ("cost", "spatial_cost", "adj_cost", "node_cost", "kl", "acc", "adj_sum", "correct")


class OptimizerVAE:
    def __init__(self, model: SGCNModelVAE, learning_rate: Optional[float] = None,
                 beta1: Optional[float] = None, beta2: Optional[float] = None,
                 epsilon: Optional[float] = None, process_group=None, seed: int = 1234,
                 fuse_adam: Optional[bool] = None, bucketed: Optional[bool] = None,
                 shard_min: Optional[int] = None):
        """fuse_adam (default: on without a process group): Adam runs inside the step
        (snd_plan_fuse_adam) -- in the weight-gradient streams of the blocks one kernel
        produces complete (graph-latent heads / d_sg_lin1; their gradient is then not
        written), and in the final slab reduction for every block it writes complete
        (gradient written); snd_adam_tf1 updates whatever is left (nothing on the
        node-latent plans, so the step is one launch shorter).

        process_group: data parallel.  Its presence (not its size) selects the
        distributed step: the all-reduce always runs and Adam is never fused, so a
        forced world of 1 executes exactly the N > 1 code path.  The device Philox
        stream is offset to this rank's rows of the global batch
        (snd_plan_set_rng_offset), so the ranks draw the normals one device would
        draw for the whole batch.

        bucketed (default OFF, opt-in): the exchange of parallel.run_buckets instead of
        one all-reduce of the whole gradient; a model without early completion points or
        large blocks (C2) has one bucket, i.e. the same single all-reduce.  Its
        side-stream overlap of early buckets with the backward pass has been checked
        bit for bit at world 1 (RCCL) and world 2 (gloo, CPU) only, never on 2+ GPUs, so
        the default stays the single all-reduce.  shard_min: floats from
        which a bucket is sharded (parallel.SHARD_MIN)."""
        cfg = model.cfg
        self.model = model
        self.lr = cfg.learning_rate if learning_rate is None else learning_rate
        self.beta1 = cfg.adam_beta1 if beta1 is None else beta1
        self.beta2 = cfg.adam_beta2 if beta2 is None else beta2
        self.eps = cfg.adam_eps if epsilon is None else epsilon
        self.seed = seed
        dev = model.device
        n = model.param_count + TAIL
        self.grads = torch.zeros(n, dtype=torch.float32, device=dev)
        self.m = torch.zeros(n, dtype=torch.float32, device=dev)
        self.v = torch.zeros(n, dtype=torch.float32, device=dev)
        self.step_counter = torch.zeros(1, dtype=torch.int32, device=dev)   # TF global step
        self.losses = torch.zeros(8, dtype=torch.float64, device=dev)
        self.group = process_group
        self.distributed = process_group is not None
        self.world, self.rank = 1, 0
        L = _lib.lib()
        if self.distributed:
            import torch.distributed as dist
            self.world = dist.get_world_size(process_group)
            self.rank = dist.get_rank(process_group)
            _lib.check(L.snd_plan_set_rng_offset(model.plan, self.rank * model.head_rows),
                       "snd_plan_set_rng_offset")
        self._graph = None
        self._batch_c = None
        if fuse_adam is None:
            fuse_adam = not self.distributed
        if fuse_adam and self.distributed:
            raise ValueError("fused Adam updates before the all-reduce: not with a process group")
        self.fused = bool(fuse_adam)
        _lib.check(L.snd_plan_fuse_adam(
            model.plan, _lib.ptr(self.m) if self.fused else None,
            _lib.ptr(self.v) if self.fused else None, self.lr, self.beta1, self.beta2, self.eps),
            "snd_plan_fuse_adam")
        # contiguous [offset, count) ranges of the blocks snd_adam_tf1 still updates
        self._adam_ranges = []
        lay = model.layout
        names = list(lay.shapes)
        for i, k in enumerate(names):
            if L.snd_plan_block_fused(model.plan, i):
                continue
            off = lay.offsets[k]
            end = lay.offsets[names[i + 1]] if i + 1 < len(names) else model.param_count
            if self._adam_ranges and self._adam_ranges[-1][0] + self._adam_ranges[-1][1] == off:
                self._adam_ranges[-1][1] += end - off
            else:
                self._adam_ranges.append([off, end - off])
        # host copies for snd_adam_tf1_ranges (read at call time, so the arrays outlive it)
        self._roff = (C.c_longlong * max(1, len(self._adam_ranges)))(*[o for o, _ in self._adam_ranges])
        self._rcnt = (C.c_longlong * max(1, len(self._adam_ranges)))(*[n for _, n in self._adam_ranges])
        self.bucketed = self.distributed and bool(bucketed)
        self.buckets = []
        self._events = {}
        # the plan records raw hipEvent_t pointers for the early buckets: drop whatever a
        # previous optimizer of this plan registered (its torch events may be freed), and
        # take ownership, so that the previous optimizer's close() / __del__ (which may
        # run after this constructor: `opt = OptimizerVAE(model, ...)` rebinding) leaves
        # this optimizer's events alone
        self._owner = object()
        model._grad_event_owner = self._owner
        self._unregister_events()
        if self.bucketed:
            self._init_buckets(shard_min)

    def _unregister_events(self):
        plan = getattr(self.model, "plan", None)
        if plan is None:
            return
        L = _lib.lib()
        for i in range(len(self.model.layout.shapes)):
            L.snd_plan_grad_event(plan, i, None)

    def close(self):
        """Unregister this optimizer's completion events from the plan (idempotent);
        called by __del__, so a freed optimizer never leaves dangling events behind.
        Only while this optimizer still owns the plan's events: a newer optimizer of the
        same model has replaced them with its own."""
        if getattr(self, "_events", None):
            if getattr(self.model, "_grad_event_owner", None) is self._owner:
                self._unregister_events()
            self._events = {}

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _init_buckets(self, shard_min):
        """Bucket plan, completion events and chunk buffers of the bucketed exchange."""
        from .parallel import SHARD_MIN, plan_buckets
        m, L = self.model, _lib.lib()
        lay = m.layout
        names = list(lay.shapes)
        blocks, points = [], []
        for i, k in enumerate(names):
            off = lay.offsets[k]
            end = lay.offsets[names[i + 1]] if i + 1 < len(names) else m.param_count
            blocks.append((off, end - off))
            pt = int(L.snd_plan_grad_event(m.plan, i, None))
            if pt < 0:
                _lib.check(pt, "snd_plan_grad_event")
            points.append(pt)
        total = m.param_count + 8       # + the loss terms the step writes (TAIL layout)
        self.buckets = plan_buckets(blocks, points, m.param_count, total, self.world,
                                    SHARD_MIN if shard_min is None else shard_min)
        # one event per early point, recorded by snd_train_step after the kernel that
        # completes it (created now: torch creates events lazily on their first record)
        for i, pt in enumerate(points):
            if pt and any(b.point == pt for b in self.buckets):
                if pt not in self._events:
                    ev = torch.cuda.Event()
                    ev.record()
                    self._events[pt] = ev
                if L.snd_plan_grad_event(m.plan, i, C.c_void_p(self._events[pt].cuda_event)) != pt:
                    raise _lib.SNDError(f"snd_plan_grad_event: block {k}: {_lib.last_error()}")
        self._comm = torch.cuda.Stream(device=m.device) if self._events else None
        self.step_next = torch.zeros(1, dtype=torch.int32, device=m.device)

    # ------------------------------------------------------------------ step
    def forward_backward(self, batch: DeviceBatch, eps: Optional[torch.Tensor] = None,
                         stream=None):
        """snd_train_step: forward, backward, gradients into `self.grads`.

        With the update fused (`self.fused`, the single-device default) this call ALSO
        applies TF1 Adam in place to every block the plan reports fused
        (snd_plan_block_fused != 0: on C2/C3/C5 all of them, inside the final reduction)
        and advances the step counter; `apply()` then updates only the rest.  A caller
        that wants gradients without an update builds the optimizer with fuse_adam=False."""
        m = self.model
        self._batch_c = batch.c_struct()
        _lib.check(_lib.lib().snd_train_step(
            m.plan, C.byref(self._batch_c), _lib.ptr(m.params), _lib.ptr(self.grads),
            _lib.ptr(m.workspace), _lib.ptr(eps), self.seed, _lib.ptr(self.step_counter),
            _lib.ptr(self.losses), _lib.stream_ptr(stream)), "snd_train_step")

    def allreduce(self):
        """One RCCL all-reduce (sum) of [flat grads || loss terms]."""
        if self.distributed:
            import torch.distributed as dist
            dist.all_reduce(self.grads[:self.model.param_count + 8], group=self.group)

    def _adam(self, off: int, n: int, grad: torch.Tensor, stream=None, step=None):
        """snd_adam_tf1 on params/m/v[off:off+n] with the gradient at `grad`; `step`:
        the device global step it reads (default the step counter)."""
        m, b = self.model, 4 * off
        _lib.check(_lib.lib().snd_adam_tf1(
            _lib.ptr(m.params) + b, _lib.ptr(grad), _lib.ptr(self.m) + b, _lib.ptr(self.v) + b,
            n, self.lr, self.beta1, self.beta2, self.eps, 1.0 / self.world,
            _lib.ptr(self.step_counter if step is None else step), _lib.stream_ptr(stream)),
            "snd_adam_tf1")

    def apply(self, stream=None):
        if len(self._adam_ranges) > 1:   # the blocks a fused update leaves: one launch
            m = self.model
            _lib.check(_lib.lib().snd_adam_tf1_ranges(
                _lib.ptr(m.params), _lib.ptr(self.grads), _lib.ptr(self.m), _lib.ptr(self.v),
                self._roff, self._rcnt, len(self._adam_ranges), self.lr, self.beta1, self.beta2,
                self.eps, 1.0 / self.world, _lib.ptr(self.step_counter), _lib.stream_ptr(stream)),
                "snd_adam_tf1_ranges")
            return
        for off, n in self._adam_ranges:
            self._adam(off, n, self.grads[off:off + n], stream)

    def exchange_apply(self):
        """The bucketed exchange + update (parallel.run_buckets) after forward_backward:
        early buckets on the communication stream, ordered after their completion
        events, the rest after the step; the step's stream then waits for all of it."""
        import torch.distributed as dist

        from .parallel import run_buckets
        g = self.group
        main = torch.cuda.current_stream()
        comm = self._comm if self._comm is not None else main

        def wait(b):
            if comm is main:
                return
            if b.point:
                self._events[b.point].wait(comm)
            else:
                comm.wait_stream(main)

        with torch.cuda.stream(comm):
            # an early bucket's update may run before the step's final reduction
            # increments the global step: it reads step_next (set before the step)
            run_buckets(self.buckets, self.grads, self.model.params, self.model.param_count,
                        self.world, self.rank,
                        lambda off, n, gr, b: self._adam(off, n, gr, step=self.step_next if b.point else None),
                        None,   # in-place reduce-scatter into this rank's chunk of grads
                        lambda out, inp: dist.reduce_scatter_tensor(out, inp, group=g),
                        lambda out, inp: dist.all_gather_into_tensor(out, inp, group=g),
                        lambda t: dist.all_reduce(t, group=g), wait)
        if comm is not main:
            main.wait_stream(comm)

    def step(self, batch: DeviceBatch, eps: Optional[torch.Tensor] = None):
        """One optimisation step (`main.py:331`): fwd+bwd, gradient exchange, Adam."""
        if self.bucketed:
            if self._events:   # the global step the early buckets' Adam updates use
                torch.add(self.step_counter, 1, out=self.step_next)
            self.forward_backward(batch, eps)
            self.exchange_apply()
            return
        self.forward_backward(batch, eps)
        self.allreduce()
        self.apply()

    def sync_state(self):
        """All-gather the Adam moments of the sharded buckets (each rank keeps only its
        chunk current) so that m and v are complete on every rank, e.g. before a
        checkpoint.  No-op without sharded buckets."""
        if not self.bucketed:
            return
        import torch.distributed as dist
        for b in self.buckets:
            if b.sharded:
                lo, c = b.shard(self.world, self.rank)
                for t in (self.m, self.v):
                    dist.all_gather_into_tensor(t[b.lo:b.hi], t[lo:lo + c].clone(), group=self.group)

    # ------------------------------------------------------------ HIP graph
    def _state(self):
        return [t.clone() for t in (self.model.params, self.m, self.v, self.step_counter,
                                    self.grads, self.losses)]

    def _set_state(self, saved):
        for dst, src in zip((self.model.params, self.m, self.v, self.step_counter,
                             self.grads, self.losses), saved):
            dst.copy_(src)

    def capture(self, batch: DeviceBatch, warmup: int = 2):
        """Capture one full step (device Philox eps) into a HIP graph.

        The ``warmup`` eager steps (kernel attributes, RCCL communicator) and the
        captured step run on the live state; parameters, Adam moments, the step
        counter, gradients and loss terms are restored afterwards, so capturing
        leaves the training state exactly as it was."""
        saved = self._state()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self.step(batch)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self.step(batch)
        torch.cuda.synchronize()
        self._set_state(saved)
        self._graph = g
        self._graph_batch = batch
        return g

    def replay(self):
        self._graph.replay()

    # ------------------------------------------------------------ readback
    @property
    def overall_loss(self):
        """[cost, spatial_cost, adj_cost, node_cost, kl_sg] (`optimizer.py:203`)."""
        v = self.losses.cpu().numpy()
        return [float(x) for x in v[:5]]

    def loss_dict(self, global_mean: bool = False):
        """All loss terms; ``global_mean`` reads the all-reduced copy (DP)."""
        if global_mean and self.distributed:
            t = self.grads[self.model.param_count:self.model.param_count + 6].double().cpu().numpy()
            t = t / self.world
            return dict(zip(LOSS_NAMES[:6], [float(x) for x in t]))
        return dict(zip(LOSS_NAMES, [float(x) for x in self.losses.cpu().numpy()]))

    @property
    def global_step(self) -> int:
        return int(self.step_counter.item())

    def grad_blocks(self):
        """Flat gradient by block (blocks updated in a weight-gradient stream --
        snd_plan_block_fused == 1 -- are not stored; the reduction-fused ones are).

        With sharded buckets (bucketed exchange) only this rank's chunk of each sharded
        bucket holds the reduced gradient; the rest of such a bucket is this rank's local,
        unreduced gradient."""
        m = self.model
        return m.layout.unpack(self.grads[:m.param_count].double().cpu().numpy())

    def state_blocks(self):
        """Adam moments by block.  COLLECTIVE under the bucketed exchange (sync_state
        all-gathers the sharded moments): call it on every rank, not on rank 0 only."""
        self.sync_state()
        m = self.model
        pc = m.param_count
        return (m.layout.unpack(self.m[:pc].double().cpu().numpy()),
                m.layout.unpack(self.v[:pc].double().cpu().numpy()))
