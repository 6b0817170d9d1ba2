"""ORACLE -- test infrastructure only.  Never imported by the product path.

NumPy restatement of the device normal stream of the reparameterisation
(z = mu + eps * exp(s), model.py:155-159; TF's tf.random.normal stream itself
cannot be matched, SURVEY.md §7 "RNG"): Philox4x32-10 keyed by the 64-bit
seed, counter (q_lo, q_hi, step, 0) for the element quad q, then two
Box-Muller pairs per block (snd_common.hpp philox4x32_10 / philox_normal4).

The integer Philox rounds are exact; Box-Muller is evaluated in float64 here
and with fast float32 log/sincos on the device, so device values agree to
~1e-5 absolute (tests state the tolerance).

Data parallel: element (global row r, column c) of an [rows, L] draw has index
r * L + c, and a rank whose head rows start at global row r0 draws from
r0 * L on (snd_plan_set_rng_offset), so the shards of a global batch see
exactly the draws one device would make for the whole batch.
"""
from __future__ import annotations

import numpy as np

_M0, _M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
_W0, _W1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)
_MASK = np.uint64(0xFFFFFFFF)


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Vectorised Philox4x32-10 over uint32 arrays (snd_common.hpp:92-103)."""
    c0, c1, c2, c3 = (np.asarray(v, dtype=np.uint32).copy() for v in (c0, c1, c2, c3))
    k0 = np.uint32(k0)
    k1 = np.uint32(k1)
    for _ in range(10):
        p0 = _M0 * c0.astype(np.uint64)
        p1 = _M1 * c2.astype(np.uint64)
        hi0, lo0 = (p0 >> np.uint64(32)).astype(np.uint32), (p0 & _MASK).astype(np.uint32)
        hi1, lo1 = (p1 >> np.uint64(32)).astype(np.uint32), (p1 & _MASK).astype(np.uint32)
        c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
        k0 = np.uint32((int(k0) + int(_W0)) & 0xFFFFFFFF)
        k1 = np.uint32((int(k1) + int(_W1)) & 0xFFFFFFFF)
    return c0, c1, c2, c3


def normal_quads(seed: int, step: int, q: np.ndarray) -> np.ndarray:
    """[len(q), 4] standard normals of element quads q (philox_normal4)."""
    q = np.asarray(q, dtype=np.uint64)
    r0, r1, r2, r3 = philox4x32_10((q & _MASK).astype(np.uint32), (q >> np.uint64(32)).astype(np.uint32),
                                   np.full(q.shape, step & 0xFFFFFFFF, np.uint32),
                                   np.zeros(q.shape, np.uint32), seed & 0xFFFFFFFF, seed >> 32)
    k = 2.3283064365386963e-10
    m1 = np.sqrt(-2.0 * np.log((r0.astype(np.float64) + 1.0) * k))
    m2 = np.sqrt(-2.0 * np.log((r2.astype(np.float64) + 1.0) * k))
    a1 = 2.0 * np.pi * (r1.astype(np.float64) * k)
    a2 = 2.0 * np.pi * (r3.astype(np.float64) * k)
    return np.stack([m1 * np.cos(a1), m1 * np.sin(a1), m2 * np.cos(a2), m2 * np.sin(a2)], axis=1)


def eps(seed: int, step: int, rows: int, latent: int, row0: int = 0) -> np.ndarray:
    """eps [rows, latent] of head rows row0 .. row0+rows-1 at TF global step `step`
    (the device reads the step counter before advancing it)."""
    idx = (np.arange(rows, dtype=np.uint64)[:, None] + np.uint64(row0)) * np.uint64(latent) \
        + np.arange(latent, dtype=np.uint64)[None, :]
    flat = idx.reshape(-1)
    quads = normal_quads(seed, step, flat >> np.uint64(2))
    return quads[np.arange(flat.size), (flat & np.uint64(3)).astype(np.int64)].reshape(rows, latent)
