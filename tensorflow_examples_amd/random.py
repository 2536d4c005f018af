"""Philox4x32-10 counter-based random numbers, identical on CPU and GPU.

``philox_fill(t, seed, subseq, dist, a, b)`` fills an f32 tensor: on the GPU with the HIP kernel
of csrc/kernels/philox.hip, on the CPU with the vectorised numpy twin below -- the same stream
bit for bit for uniform draws (normal draws agree to float rounding of log/cos/sin).  The
counter layout ``(block, round, subseq_lo, subseq_hi)`` keyed by ``seed`` makes every
(seed, tensor id, element) independent of launch shape, device and of every other tensor.

dist: 0 = uniform [a, b), 1 = normal(mean a, stddev b), 2 = normal truncated at 2 stddev.
"""
from __future__ import annotations

import numpy as np
import torch

from .ops import _native

UNIFORM, NORMAL, TRUNCATED_NORMAL = 0, 1, 2
_M0, _M1, _W0, _W1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57), np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)


def philox4x32_10(c0, c1, c2, c3, k0: int, k1: int):
    """Vectorised Philox4x32-10 over uint32 arrays; returns the four output words."""
    c0, c1, c2, c3 = (np.asarray(c, dtype=np.uint32) for c in (c0, c1, c2, c3))
    k0, k1 = np.uint32(k0 & 0xFFFFFFFF), np.uint32(k1 & 0xFFFFFFFF)
    with np.errstate(over="ignore"):
        for _ in range(10):
            p0 = _M0 * c0.astype(np.uint64)
            p1 = _M1 * c2.astype(np.uint64)
            hi0, lo0 = (p0 >> np.uint64(32)).astype(np.uint32), p0.astype(np.uint32)
            hi1, lo1 = (p1 >> np.uint64(32)).astype(np.uint32), p1.astype(np.uint32)
            c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
            k0 = np.uint32(k0 + _W0)
            k1 = np.uint32(k1 + _W1)
    return c0, c1, c2, c3


def _u01(x):
    return ((x >> np.uint32(8)).astype(np.float32) + np.float32(0.5)) * np.float32(1.0 / 16777216.0)


def _box_muller(a, b):
    r = np.sqrt(np.float32(-2.0) * np.log(_u01(a)))
    t = np.float32(6.283185307179586) * _u01(b)
    return (r * np.cos(t)).astype(np.float32), (r * np.sin(t)).astype(np.float32)


def philox_numpy(n: int, seed: int, subseq: int, dist: int, a: float, b: float) -> np.ndarray:
    blocks = (n + 3) // 4
    blk = np.arange(blocks, dtype=np.uint64).astype(np.uint32)
    zeros = np.zeros(blocks, np.uint32)
    s0 = np.full(blocks, subseq & 0xFFFFFFFF, np.uint32)
    s1 = np.full(blocks, (subseq >> 32) & 0xFFFFFFFF, np.uint32)
    k0, k1 = seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF
    x, y, z, w = philox4x32_10(blk, zeros, s0, s1, k0, k1)
    if dist == UNIFORM:
        out = np.stack([_u01(v) for v in (x, y, z, w)], 1)
        out = np.float32(a) + np.float32(b - a) * out
    else:
        z0, z1 = _box_muller(x, y)
        z2, z3 = _box_muller(z, w)
        zz = np.stack([z0, z1, z2, z3], 1)
        if dist == TRUNCATED_NORMAL:
            for rnd in range(1, 17):
                bad = np.abs(zz) > 2.0
                if not bad.any():
                    break
                rows = np.nonzero(bad.any(1))[0]
                q = philox4x32_10(blk[rows], np.full(len(rows), rnd, np.uint32), s0[rows], s1[rows], k0, k1)
                p0, p1 = _box_muller(q[0], q[1])
                p2, p3 = _box_muller(q[2], q[3])
                redraw = np.stack([p0, p1, p2, p3], 1)
                sub = zz[rows]
                sub[bad[rows]] = redraw[bad[rows]]
                zz[rows] = sub
            zz = np.clip(zz, -2.0, 2.0)
        out = np.float32(a) + np.float32(b) * zz
    return out.reshape(-1)[:n].astype(np.float32)


def philox_fill(t: torch.Tensor, seed: int, subseq: int, dist: int, a: float, b: float) -> torch.Tensor:
    """Fill contiguous f32 ``t`` in place (GPU kernel or numpy twin); returns ``t``."""
    assert t.dtype == torch.float32 and t.is_contiguous()
    seed &= 0x7FFFFFFFFFFFFFFF
    subseq &= 0x7FFFFFFFFFFFFFFF
    if _native.use_native(t):
        torch.ops.tfx.philox_fill(t, seed, subseq, dist, float(a), float(b))
    else:
        t.copy_(torch.from_numpy(philox_numpy(t.numel(), seed, subseq, dist, a, b)).view(t.shape))
    return t
