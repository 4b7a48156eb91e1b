"""Host (numpy) Philox4x32-10, bit-identical to ``csrc/kernels/common.h``.

Used for CPU execution and as the oracle in the GPU RNG tests.  Random values
are keyed by (seed, global element index, stream) so they do not depend on how
rows are partitioned across GPUs.
"""
from __future__ import annotations

import numpy as np

_M0 = np.uint64(0xD2511F53)
_M1 = np.uint64(0xCD9E8D57)
_W0 = np.uint32(0x9E3779B9)
_W1 = np.uint32(0xBB67AE85)
_MASK32 = np.uint64(0xFFFFFFFF)


def philox4x32_10(c0, c1, c2, c3, k0: int, k1: int):
    c0 = np.asarray(c0, dtype=np.uint32)
    c1 = np.asarray(c1, dtype=np.uint32)
    c2 = np.broadcast_to(np.asarray(c2, dtype=np.uint32), c0.shape)
    c3 = np.broadcast_to(np.asarray(c3, dtype=np.uint32), c0.shape)
    k0 = np.uint32(k0 & 0xFFFFFFFF)
    k1 = np.uint32(k1 & 0xFFFFFFFF)
    with np.errstate(over="ignore"):
        for _ in range(10):
            p0 = _M0 * c0.astype(np.uint64)
            p1 = _M1 * c2.astype(np.uint64)
            hi0 = (p0 >> np.uint64(32)).astype(np.uint32)
            lo0 = (p0 & _MASK32).astype(np.uint32)
            hi1 = (p1 >> np.uint64(32)).astype(np.uint32)
            lo1 = (p1 & _MASK32).astype(np.uint32)
            n0 = hi1 ^ c1 ^ k0
            n1 = lo1
            n2 = hi0 ^ c3 ^ k1
            n3 = lo0
            c0, c1, c2, c3 = n0, n1, n2, n3
            k0 = np.uint32((int(k0) + int(_W0)) & 0xFFFFFFFF)
            k1 = np.uint32((int(k1) + int(_W1)) & 0xFFFFFFFF)
    return c0, c1, c2, c3


def uniform(n: int, seed: int, offset: int = 0, stream: int = 0) -> np.ndarray:
    """Uniform doubles in [0,1) for elements offset..offset+n-1."""
    seed &= 0xFFFFFFFFFFFFFFFF
    idx = np.arange(offset, offset + n, dtype=np.uint64)
    lo = (idx & _MASK32).astype(np.uint32)
    hi = (idx >> np.uint64(32)).astype(np.uint32)
    r0, r1, _, _ = philox4x32_10(lo, hi, np.uint32(stream & 0xFFFFFFFF), np.uint32(0x5EED), seed & 0xFFFFFFFF,
                                 seed >> 32)
    bits = ((r0 >> np.uint32(5)).astype(np.uint64) << np.uint64(26)) | (r1 >> np.uint32(6)).astype(np.uint64)
    return bits.astype(np.float64) * (1.0 / 9007199254740992.0)


def poisson_from_uniform(u: np.ndarray, lam: float) -> np.ndarray:
    """Vectorised CDF inversion, identical to cdna::poisson_from_uniform."""
    u = np.asarray(u, dtype=np.float64)
    k = np.zeros(u.shape, dtype=np.int64)
    p = np.full(u.shape, np.exp(-lam))
    F = p.copy()
    active = u > F
    kk = 0
    while active.any() and kk < 255:
        kk += 1
        p = np.where(active, p * (lam / kk), p)
        F = np.where(active, F + p, F)
        k = np.where(active, kk, k)
        active = active & (u > F)
    return k


def uniform32(n: int, seed: int, offset: int = 0, stream: int = 0) -> np.ndarray:
    """32-bit uniforms (as doubles in [0,1)) for elements offset..offset+n-1: one Philox call per quad of
    consecutive global indices (index >> 2), word index & 3 (``poisson_kernel`` in misc.hip)."""
    seed &= 0xFFFFFFFFFFFFFFFF
    if n <= 0:
        return np.zeros(0)
    q0, q1 = offset >> 2, (offset + n - 1) >> 2
    q = np.arange(q0, q1 + 1, dtype=np.uint64)
    lo = (q & _MASK32).astype(np.uint32)
    hi = (q >> np.uint64(32)).astype(np.uint32)
    r = philox4x32_10(lo, hi, np.uint32(stream & 0xFFFFFFFF), np.uint32(0xB00F), seed & 0xFFFFFFFF, seed >> 32)
    words = np.stack(r, 1).reshape(-1)[offset - 4 * q0: offset - 4 * q0 + n]
    return words.astype(np.float64) * (1.0 / 4294967296.0)


def normal32(n: int, seed: int, offset: int = 0, stream: int = 0) -> np.ndarray:
    """fp32 standard normals for elements offset..offset+n-1, the layout of ``normal_f32_kernel`` (misc.hip):
    quad q = index >> 2, words (0, 1) and (2, 3) are Box-Muller pairs (r cos, r sin), u = (w + 1/2) 2^-32 formed
    in fp32 exactly as the kernel forms it (w rounds to 24 significant bits first, so for w >= 2^32 - 128 the
    radius uniform is exactly 1.0 and the pair is (0, 0) on both sides); the log / sin / cos are float64 here,
    the kernel's hardware ones agree to ~1e-6 relative."""
    seed &= 0xFFFFFFFFFFFFFFFF
    if n <= 0:
        return np.zeros(0, dtype=np.float32)
    q0, q1 = offset >> 2, (offset + n - 1) >> 2
    q = np.arange(q0, q1 + 1, dtype=np.uint64)
    lo = (q & _MASK32).astype(np.uint32)
    hi = (q >> np.uint64(32)).astype(np.uint32)
    w = [((x.astype(np.float32) + np.float32(0.5)) * np.float32(1.0 / 4294967296.0)).astype(np.float64)
         for x in philox4x32_10(lo, hi, np.uint32(stream & 0xFFFFFFFF), np.uint32(0x4E0A), seed & 0xFFFFFFFF,
                                seed >> 32)]
    z = np.empty((len(q), 4))
    for p in range(2):
        rad = np.sqrt(-2.0 * np.log(w[2 * p]))
        th = 2.0 * np.pi * w[2 * p + 1]
        z[:, 2 * p], z[:, 2 * p + 1] = rad * np.cos(th), rad * np.sin(th)
    return z.reshape(-1)[offset - 4 * q0: offset - 4 * q0 + n].astype(np.float32)


def poisson(T: int, n: int, seed: int, offset: int, rate: float) -> np.ndarray:
    out = np.empty((T, n), dtype=np.uint8)
    for t in range(T):
        u = uniform32(n, seed, offset, 0x100 + t)
        out[t] = np.minimum(poisson_from_uniform(u, rate), 255).astype(np.uint8)
    return out
