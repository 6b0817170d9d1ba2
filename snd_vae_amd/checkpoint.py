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

import numpy as np
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
    """Write params (+ Adam m, v, global step when ``optimizer`` is given).  With a
    bucketed data-parallel optimizer whose large buckets keep sharded Adam moments,
    call ``optimizer.sync_state()`` on every rank first (a collective)."""
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
            d[k] = tuple(tuple(e) if isinstance(e, list) else e for e in v)
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


# ---------------------------------------------------------------------------
# Reference (tf.train.Saver) variable names <-> the flat layout.
#
# The reference checkpoint is TF's binary bundle, which needs TensorFlow to
# read.  The bridge here works on a plain {variable name: array} mapping -- what
# ``{n: tf.train.load_variable(ckpt, n) for n, _ in tf.train.list_variables(ckpt)}``
# returns in a TF environment, saved with ``np.savez`` -- and on the same
# mapping in the other direction.  Names are the TF variable names of the hot
# path (params.logical_names: e.g. "encoder/g_g1_lin/Matrix", Keras BN
# "decoder/d_bn_s0/gamma", tf.layers.conv1d "decoder/s1_deconv/kernel"); any
# outer scope prefix and a ":0" suffix are accepted.  TF1 Adam keeps its slots
# as "<var>/Adam" (m) and "<var>/Adam_1" (v) and the bias-correction powers
# "beta1_power" / "beta2_power" (optimizer.py:125,197), from which the global
# step is recovered.  Keras BN moving statistics must be the frozen
# inference-mode values (mean 0, variance 1).

def _strip(name: str) -> str:
    return name[:-2] if name.endswith(":0") else name


def _lookup(variables: dict, name: str):
    hits = [k for k in variables if _strip(k) == name or _strip(k).endswith("/" + name)]
    if len(hits) > 1:
        raise ValueError(f"ambiguous reference variable {name!r}: {hits}")
    return variables[hits[0]] if hits else None


def reference_to_blocks(cfg: SNDConfig, variables: dict, beta1: float = 0.9, beta2: float = 0.999,
                        global_step: Optional[int] = None):
    """{TF variable name: array} -> (blocks, adam_m, adam_v, global_step).

    blocks / adam_m / adam_v are dicts in the params.py layout (adam_m / adam_v /
    global_step are None when the mapping holds no Adam slots).  Raises on a
    missing variable, a shape mismatch, or BN moving statistics that are not the
    frozen (0, 1) the hot path assumes, and when Adam slots come without the
    bias-correction powers (unless ``global_step`` gives the step)."""

    from .params import block_shapes, logical_names
    shapes = block_shapes(cfg)
    blocks = {k: np.zeros(s) for k, s in shapes.items()}
    has_adam = any(_strip(k).endswith("/Adam") for k in variables)
    m = {k: np.zeros(s) for k, s in shapes.items()} if has_adam else None
    v = {k: np.zeros(s) for k, s in shapes.items()} if has_adam else None
    for name, entry in logical_names(cfg).items():
        blk, sl = entry[:2]
        flat = len(entry) == 3          # stored flattened inside the block (shape entry[2])
        val = _lookup(variables, name)
        if val is None:
            raise KeyError(f"reference variable {name!r} not found")
        val = np.asarray(val, dtype=np.float64)
        dst = blocks[blk][..., sl]
        want = entry[2] if flat else dst.shape
        if val.shape != tuple(want):
            raise ValueError(f"{name}: shape {val.shape} != {tuple(want)} of {blk}")
        blocks[blk][..., sl] = val.reshape(-1) if flat else val
        if has_adam:
            for slot, tgt in (("Adam", m), ("Adam_1", v)):
                s = _lookup(variables, f"{name}/{slot}")
                if s is None:
                    raise KeyError(f"Adam slot {name}/{slot} not found")
                s = np.asarray(s, dtype=np.float64)
                tgt[blk][..., sl] = s.reshape(-1) if flat else s
        if name.endswith("/gamma"):       # Keras BN: frozen moving statistics only
            scope = name[:-len("gamma")]
            for stat, want in (("moving_mean", 0.0), ("moving_variance", 1.0)):
                s = _lookup(variables, scope + stat)
                if s is not None and not np.allclose(s, want):
                    raise ValueError(f"{scope}{stat} is not the frozen value {want}: "
                                     "the hot path runs Keras BN in inference mode (SURVEY §0.3)")
    if global_step is not None:
        return blocks, m, v, int(global_step)
    step = _step_from_powers(_lookup(variables, "beta1_power"), _lookup(variables, "beta2_power"),
                             beta1, beta2)
    if has_adam and step is None:
        raise ValueError("reference Adam slots present but no beta1_power / beta2_power: the "
                         "bias correction of the next step is unknown; pass global_step")
    return blocks, m, v, step


# The smallest normal float32: TF keeps the bias-correction powers in float32, so
# below this a power carries fewer than 24 significant bits (0.9^t at t ~ 830).
_F32_TINY = float(np.finfo(np.float32).tiny)


def _step_from_powers(b1p, b2p, beta1: float, beta2: float) -> Optional[int]:
    """Completed steps t from TF1 Adam's powers.

    TF1 ``AdamOptimizer`` creates beta1_power = beta1 and multiplies it by beta1
    after every apply (optimizer.py:125,197), so after t steps it holds
    beta1^(t+1); the step counter here holds t (Adam's step k uses beta^k).
    beta1_power leaves the float32 normal range after ~830 steps and flushes to
    0 near ~980, so the beta2 power (0.999^(t+1), normal until t ~ 87 K) is used
    whenever beta1_power is subnormal or zero.  TF multiplies by float32(beta)
    (0.999 -> 0.99900001287), so the logarithm is taken of that float32 value:
    with float64 0.999 the estimate drifts by a whole step from t ~ 39 K."""
    for p, beta in ((b1p, beta1), (b2p, beta2)):
        if p is None:
            continue
        val = float(np.asarray(p, dtype=np.float64))
        if not (val >= _F32_TINY) or val > 1.0:
            continue
        return int(round(np.log(val) / np.log(float(np.float32(beta))))) - 1
    if b1p is not None or b2p is not None:
        raise ValueError("beta1_power and beta2_power are both zero or subnormal: the global step "
                         "cannot be recovered; pass global_step")
    return None


def blocks_to_reference(cfg: SNDConfig, blocks: dict, adam_m: Optional[dict] = None,
                        adam_v: Optional[dict] = None, global_step: Optional[int] = None,
                        beta1: float = 0.9, beta2: float = 0.999) -> dict:
    """The inverse of reference_to_blocks: {TF variable name: float32 array},
    with the Adam slots, bias-correction powers and frozen BN statistics."""

    from .params import logical_names
    out = {}
    for name, entry in logical_names(cfg).items():
        blk, sl = entry[:2]
        shp = (lambda a: a.reshape(entry[2])) if len(entry) == 3 else (lambda a: a)
        out[name] = np.ascontiguousarray(shp(blocks[blk][..., sl]), dtype=np.float32)
        if adam_m is not None:
            out[name + "/Adam"] = np.ascontiguousarray(shp(adam_m[blk][..., sl]), dtype=np.float32)
            out[name + "/Adam_1"] = np.ascontiguousarray(shp(adam_v[blk][..., sl]), dtype=np.float32)
        if name.endswith("/gamma"):
            scope = name[:-len("gamma")]
            out[scope + "moving_mean"] = np.zeros_like(out[name])
            out[scope + "moving_variance"] = np.ones_like(out[name])
    if global_step is not None:                      # TF1: beta^(t+1) after t steps
        out["beta1_power"] = tf_power(beta1, global_step)
        out["beta2_power"] = tf_power(beta2, global_step)
    return out


def tf_power(beta: float, steps: int) -> np.float32:
    """TF1 Adam's bias-correction power after `steps` applies: float32(beta) times
    float32(beta) `steps` times, every product rounded to float32 (optimizer.py:125,197;
    the variable starts at beta).  Past 2^18 steps (both powers long subnormal) the
    float64 closed form."""
    b = np.float32(beta)
    if steps > (1 << 18):
        return np.float32(float(b) ** (steps + 1))
    p = b
    for _ in range(steps):
        p = np.float32(p * b)
    return p


def load_reference(path: str, model, optimizer=None,
                   global_step: Optional[int] = None) -> Optional[int]:
    """Load an .npz of reference variables (np.load, allow_pickle=False) into the
    device model (and optimizer); returns the recovered global step."""
    with np.load(path, allow_pickle=False) as z:
        variables = {k: z[k] for k in z.files}
    b1 = optimizer.beta1 if optimizer is not None else model.cfg.adam_beta1
    b2 = optimizer.beta2 if optimizer is not None else model.cfg.adam_beta2
    blocks, m, v, step = reference_to_blocks(model.cfg, variables, beta1=b1, beta2=b2,
                                             global_step=global_step)
    model.load_blocks(blocks)
    if optimizer is not None and m is not None:
        lay = model.layout
        pc = model.param_count
        optimizer.m[:pc].copy_(torch.from_numpy(lay.pack(m, np.float32)))
        optimizer.v[:pc].copy_(torch.from_numpy(lay.pack(v, np.float32)))
        if step is not None:
            optimizer.step_counter.fill_(step)
    return step


def save_reference(path: str, model, optimizer=None) -> None:
    """Write the device state under the reference variable names (.npz)."""
    m = v = step = None
    if optimizer is not None:
        m, v = optimizer.state_blocks()
        step = optimizer.global_step
    out = blocks_to_reference(model.cfg, model.blocks(), m, v, step,
                              *((optimizer.beta1, optimizer.beta2) if optimizer is not None else ()))
    np.savez(path, **out)
