"""Training loop: the `main.py:296-353` train branch on device-resident batches.

Reference loop per epoch: slice ``batch_size`` graphs (`main.py:316-323`),
feed them (`main.py:327-329`, dropout 1, global_iter = epoch), run
``[opt_op, overall_loss, generated_adj]`` (`main.py:331`), compute the
accuracy on the host (`main.py:334`), append to the epoch ``storer``
(`main.py:335-346`), print, and save a checkpoint every 100 epochs
(`main.py:350-352`).

Here the whole split is uploaded to HBM once (one block-diagonal CSR per
batch; the reference re-feeds dense [B, N, N] arrays every step), each batch's
step is captured into its own HIP graph on first use and replayed afterwards,
and the loss terms (accuracy included, counted on device in the zz^T kernel)
are copied into a device history that is read back once per epoch.  Data
parallel: each global batch of ``batch_size`` graphs is split contiguously
over the ranks.
"""
from __future__ import annotations

import os
import time
from collections import defaultdict
from typing import Dict, List, Optional

import numpy as np
import torch

from . import checkpoint as ckpt
from .config import SNDConfig
from .data import default_tile_rows
from .input_data import SynDataset, dataset_class_balance, dataset_sg_batch
from .model import DeviceBatch, SGCNModelVAE
from .optimizer import LOSS_NAMES, OptimizerVAE

# storer keys of main.py:336-346 ('base' model: the single KL is 'sg_kl')
STORER = (("loss", "cost"), ("spatial_loss", "spatial_cost"), ("adj_loss", "adj_cost"),
          ("adj_acc", "acc"), ("node_loss", "node_cost"), ("sg_kl", "kl"))


class Trainer:
    def __init__(self, cfg: SNDConfig, dataset: SynDataset, batch_size: int,
                 dtype: str = "bf16", process_group=None, seed: int = 1234,
                 use_graphs: bool = True, locality: bool = True, blocks=None, device="cuda",
                 weighted: bool = False):
        """weighted: the weighted-BCE structure loss (SURVEY §8 decision ii) with the
        dataset's pos_weight / norm of `main.py:246-247` over its spanning trees.
        Off by default, as in the reference, whose loss ignores both (`optimizer.py:144`)."""
        if weighted:
            pw, nm = dataset_class_balance(dataset)
            cfg = cfg.replace(weighted_bce=True, pos_weight=pw, norm=nm)
        world, rank = 1, 0
        if process_group is not None:
            import torch.distributed as dist
            world, rank = dist.get_world_size(process_group), dist.get_rank(process_group)
        if batch_size % world:
            raise ValueError("batch_size must divide evenly over the ranks")
        self.cfg, self.batch_size, self.world, self.rank = cfg, batch_size, world, rank
        per = batch_size // world
        self.batch_num = dataset.n_graphs // batch_size           # main.py:312
        if self.batch_num < 1:
            raise ValueError(f"{dataset.n_graphs} graphs < batch_size {batch_size}")
        self.batches: List[DeviceBatch] = []
        for i in range(self.batch_num):
            lo = i * batch_size + rank * per
            graphs = range(lo, lo + per)
            hb = (dataset_sg_batch(dataset, cfg, graphs) if cfg.topology == "sgjoint"
                  else dataset.batch(cfg, graphs))
            self.batches.append(DeviceBatch(hb, device=device, locality=locality,
                                            tile_rows=default_tile_rows(cfg.g_conv_hidden[1])))
        self.model = SGCNModelVAE(cfg, per, dtype=dtype, device=device, blocks=blocks)
        self.opt = OptimizerVAE(self.model, process_group=process_group, seed=seed)
        self.use_graphs = use_graphs
        self._graphs: Dict[int, torch.cuda.CUDAGraph] = {}
        self._warm = False
        self.epoch = 0
        self.history: List[Dict[str, np.ndarray]] = []

    # --------------------------------------------------------------- one step
    def _state(self):
        o = self.opt
        return [t.clone() for t in (self.model.params, o.m, o.v, o.step_counter, o.grads)]

    def _set_state(self, s):
        o = self.opt
        for dst, src in zip((self.model.params, o.m, o.v, o.step_counter, o.grads), s):
            dst.copy_(src)

    def _capture(self, i: int):
        """HIP graph of batch i's step; the training state is left untouched."""
        saved = self._state()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            if not self._warm:          # kernel attributes, RCCL communicator: set up eagerly
                self.opt.step(self.batches[i])
                self._warm = True
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self.opt.step(self.batches[i])
        torch.cuda.synchronize()
        self._set_state(saved)
        self._graphs[i] = g
        return g

    def step(self, i: int):
        if not self.use_graphs:
            self.opt.step(self.batches[i])
            return
        g = self._graphs.get(i) or self._capture(i)
        g.replay()

    # ------------------------------------------------------------------ epochs
    def train_epoch(self, verbose: bool = False) -> Dict[str, np.ndarray]:
        hist = torch.zeros(self.batch_num, len(LOSS_NAMES), dtype=torch.float64,
                           device=self.opt.losses.device)
        t0 = time.time()
        for i in range(self.batch_num):
            self.step(i)
            if self.opt.distributed:   # global means ride in the all-reduced gradient tail
                pc = self.model.param_count
                hist[i, :6].copy_(self.opt.grads[pc:pc + 6].double() / self.world)
            else:
                hist[i].copy_(self.opt.losses)
        h = hist.cpu().numpy()
        storer = defaultdict(list)
        for key, name in STORER:
            storer[key] = h[:, LOSS_NAMES.index(name)].copy()
        storer = dict(storer)
        storer["epoch_time"] = np.array([time.time() - t0])
        self.history.append(storer)
        if verbose and self.rank == 0:
            print("Epoch:", "%04d" % (self.epoch + 1), "loss=", "{:.5f}".format(storer["loss"][-1]),
                  "time=", "{:.5f}".format(storer["epoch_time"][0]))
        self.epoch += 1
        return storer

    def train(self, epochs: int, checkpoint_dir: Optional[str] = None, save_every: int = 100,
              verbose: bool = False) -> List[Dict[str, np.ndarray]]:
        """`main.py:310-353`; checkpoints at epochs 0, save_every, ... (rank 0)."""
        out = []
        for _ in range(epochs):
            e = self.epoch
            out.append(self.train_epoch(verbose))
            if checkpoint_dir and e % save_every == 0:
                self.opt.sync_state()   # collective: sharded Adam moments onto every rank
                if self.rank == 0:
                    os.makedirs(checkpoint_dir, exist_ok=True)
                    self.save(os.path.join(checkpoint_dir, f"model_dgt_global_{e}.safetensors"))
        return out

    def save(self, path: str):
        ckpt.save(path, self.model, self.opt)

    def restore(self, path: str):
        return ckpt.restore(path, self.model, self.opt)
