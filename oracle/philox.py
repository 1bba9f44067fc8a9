"""Philox4x32-10 counter-based RNG in NumPy (oracle copy; test infrastructure only).

Bit-identical to the device generator in ``mpc_blaster_amd/csrc/mpcb_inputs.hip``:
key = (seed_lo, seed_hi), counter = (instance_lo, instance_hi, draw, 0).  Each call yields
four uint32 words; a double in [0, 1) takes 53 bits from words 0 and 1
(``((w0 >> 5) * 2**26 + (w1 >> 6)) * 2**-53``), the second double from words 2 and 3.
(Salmon et al., "Parallel random numbers: as easy as 1, 2, 3", SC'11 — public algorithm.)
"""
from __future__ import annotations

import numpy as np

M0 = np.uint64(0xD2511F53)
M1 = np.uint64(0xCD9E8D57)
W0 = np.uint32(0x9E3779B9)
W1 = np.uint32(0xBB67AE85)
_MASK = np.uint64(0xFFFFFFFF)


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    c0 = np.asarray(c0, dtype=np.uint32).copy()
    c1 = np.asarray(c1, dtype=np.uint32).copy()
    c2 = np.asarray(c2, dtype=np.uint32).copy()
    c3 = np.asarray(c3, dtype=np.uint32).copy()
    k0 = np.asarray(k0, dtype=np.uint32) + np.zeros_like(c0)
    k1 = np.asarray(k1, dtype=np.uint32) + np.zeros_like(c0)
    for r in range(10):
        p0 = M0 * c0.astype(np.uint64)
        p1 = M1 * c2.astype(np.uint64)
        hi0 = (p0 >> np.uint64(32)).astype(np.uint32)
        lo0 = (p0 & _MASK).astype(np.uint32)
        hi1 = (p1 >> np.uint64(32)).astype(np.uint32)
        lo1 = (p1 & _MASK).astype(np.uint32)
        n0 = hi1 ^ c1 ^ k0
        n1 = lo1
        n2 = hi0 ^ c3 ^ k1
        n3 = lo0
        c0, c1, c2, c3 = n0, n1, n2, n3
        if r < 9:
            k0 = k0 + W0
            k1 = k1 + W1
    return c0, c1, c2, c3


def uniform2(seed: int, instance: np.ndarray, draw: int):
    """Two doubles in [0, 1) per instance for counter ``draw``."""
    inst = np.asarray(instance, dtype=np.uint64)
    lo = (inst & _MASK).astype(np.uint32)
    hi = (inst >> np.uint64(32)).astype(np.uint32)
    s = np.uint64(seed)
    k0 = np.uint32(int(s) & 0xFFFFFFFF)
    k1 = np.uint32((int(s) >> 32) & 0xFFFFFFFF)
    w0, w1, w2, w3 = philox4x32_10(lo, hi, np.full_like(lo, draw), np.zeros_like(lo), k0, k1)
    scale = 2.0 ** -53
    a = ((w0 >> np.uint32(5)).astype(np.float64) * 67108864.0 + (w1 >> np.uint32(6)).astype(np.float64)) * scale
    b = ((w2 >> np.uint32(5)).astype(np.float64) * 67108864.0 + (w3 >> np.uint32(6)).astype(np.float64)) * scale
    return a, b


def uniform(seed: int, instance: np.ndarray, n: int) -> np.ndarray:
    """``n`` doubles in [0, 1) per instance: shape (len(instance), n). Draw d feeds columns 2d, 2d+1."""
    inst = np.asarray(instance, dtype=np.uint64)
    out = np.empty((inst.shape[0], n))
    for d in range((n + 1) // 2):
        a, b = uniform2(seed, inst, d)
        out[:, 2 * d] = a
        if 2 * d + 1 < n:
            out[:, 2 * d + 1] = b
    return out
