"""Checkpoint save / restore (the ``tf.train.Saver`` of `main.py:299,351-352,376`).

The reference saves every TF variable plus the Adam slots every 100 epochs
and restores them for the test modes.  Here trainable state is the flat fp32
parameter buffer and TF1-Adam's m / v of the same layout (`params.py`), plus
the global step; one safetensors file holds them, with the config and the
block table in the metadata so a restore into a different architecture fails
loudly instead of silently mis-slicing.
"""
from __future__ import annotations

import dataclasses
import json
from typing import Optional

import torch

from .config import SNDConfig


def _meta(model) -> dict:
    lay = model.layout
    return {
        "format": "snd_vae_amd/1",
        "config": json.dumps(dataclasses.asdict(model.cfg)),
        "blocks": json.dumps([[k, int(lay.offsets[k]), int(lay.numel(k))] for k in lay.shapes]),
        "param_count": str(model.param_count),
    }


def save(path: str, model, optimizer=None) -> None:
    """Write params (+ Adam m, v, global step when ``optimizer`` is given)."""
    from safetensors.torch import save_file
    pc = model.param_count
    t = {"params": model.params[:pc].detach().cpu().contiguous()}
    if optimizer is not None:
        t["adam_m"] = optimizer.m[:pc].detach().cpu().contiguous()
        t["adam_v"] = optimizer.v[:pc].detach().cpu().contiguous()
        t["global_step"] = optimizer.step_counter.detach().cpu().to(torch.int64).contiguous()
    save_file(t, path, metadata=_meta(model))


def read_config(path: str) -> SNDConfig:
    from safetensors import safe_open
    with safe_open(path, framework="pt") as f:
        d = json.loads(f.metadata()["config"])
    for k, v in d.items():
        if isinstance(v, list):
            d[k] = tuple(v)
    return SNDConfig(**d)


def restore(path: str, model, optimizer=None, strict_config: bool = True) -> Optional[int]:
    """Load a checkpoint into ``model`` (and ``optimizer``); returns the global step."""
    from safetensors import safe_open
    with safe_open(path, framework="pt") as f:
        meta = f.metadata()
        if meta.get("format") != "snd_vae_amd/1":
            raise ValueError(f"{path}: not an snd_vae_amd checkpoint")
        want = _meta(model)
        if meta["blocks"] != want["blocks"]:
            raise ValueError(f"{path}: parameter layout differs from the model's")
        if strict_config and meta["config"] != want["config"]:
            raise ValueError(f"{path}: config differs from the model's "
                             f"({meta['config']} vs {want['config']})")
        pc = model.param_count
        model.params[:pc].copy_(f.get_tensor("params"))
        step = None
        if optimizer is not None and "adam_m" in f.keys():
            optimizer.m[:pc].copy_(f.get_tensor("adam_m"))
            optimizer.v[:pc].copy_(f.get_tensor("adam_v"))
            step = int(f.get_tensor("global_step")[0])
            optimizer.step_counter.fill_(step)
    return step
