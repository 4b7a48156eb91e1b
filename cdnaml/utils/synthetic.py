"""Partition-invariant synthetic tables for benchmarks and SPMD tests.

Every value is a pure function of (seed, GLOBAL row id, column): a rank that
owns rows [a, b) of the global table generates exactly those rows, so a job on
1, 2, 4 or 8 GPUs sees the same global table and trains the same model (the
BASELINE configs are quoted at 1/2/4/8 GPUs on one fixed dataset).  Draws are
the engine's Philox4x32-10 (K15, ``ops.kernels.uniform``: HIP on a GPU, numpy
on the host, bit-identical), turned into normals by Box-Muller.
"""
from __future__ import annotations

import math
from typing import Tuple

import torch

from ..ops import kernels as K

_CHUNK_ELEMS = 1 << 28  # elements per generation chunk (2 GiB of fp64 uniforms per stream)


def philox_normal(rows: int, d: int, seed: int, row_offset: int, stream: int, device,
                  dtype=torch.float32) -> torch.Tensor:
    """[rows, d] standard normals; element (r, f) is keyed by global index (row_offset + r) * d + f."""
    device = torch.device(device)
    out = torch.empty((rows, d), dtype=dtype, device=device)
    if rows == 0 or d == 0:
        return out
    step = max(1, _CHUNK_ELEMS // d)
    for r0 in range(0, rows, step):
        m = min(step, rows - r0)
        base = (row_offset + r0) * d
        u1 = K.uniform(m * d, seed, base, stream, device=device)
        u2 = K.uniform(m * d, seed, base, stream + 1, device=device)
        z = torch.sqrt(-2.0 * torch.log1p(-u1)) * torch.cos((2.0 * math.pi) * u2)  # 1 - u1 in (0, 1]
        out[r0:r0 + m] = z.view(m, d).to(dtype)
        del u1, u2, z
    return out


def regression_shard(n_total: int, d: int, seed: int, rank: int, world: int, device,
                     noise: float = 0.1) -> Tuple[torch.Tensor, torch.Tensor, int]:
    """This rank's contiguous shard of the headline table (features N(0, 1), nonlinear label).

    label = X . w + 2 sin(2 x0) + 3 [x1 > 0.5] + noise * N(0, 1), w ~ N(0, 1) from ``seed``.  The dot product
    is accumulated column by column in fp64, so each row's label is the same whatever the shard size.
    Returns (X f32 [n, d], y f64 [n], global row offset)."""
    a, b = n_total * rank // world, n_total * (rank + 1) // world
    n = b - a
    X = philox_normal(n, d, seed, a, 0x10, device)
    w = philox_normal(1, d, seed, 0, 0x20, "cpu", torch.float64)[0].tolist()
    y = torch.zeros(n, dtype=torch.float64, device=X.device)
    for f in range(d):
        y.add_(X[:, f].double(), alpha=w[f])
    if d > 0:
        y.add_(torch.sin(X[:, 0].double() * 2.0), alpha=2.0)
    if d > 1:
        y.add_((X[:, 1] > 0.5).double(), alpha=3.0)
    if noise:
        y.add_(philox_normal(n, 1, seed, a, 0x30, X.device, torch.float64)[:, 0], alpha=noise)
    return X, y, a


def forest_digest(forest) -> str:
    """Stable hash of a fitted forest's trees (splits, thresholds, leaf values), node-numbering independent:
    each tree is walked breadth-first from its root (cross-world-size / fused-vs-alone identity checks)."""
    import hashlib
    from collections import deque

    import numpy as np

    h = hashlib.sha256()
    feat, bins, is_cat, thr, left, right = (np.asarray(getattr(forest, n)) for n in
                                            ("feat", "bin", "is_cat", "thr", "left", "right"))
    catmask, value = forest.catmask, forest.value
    for r in forest.roots:
        q = deque([r])
        while q:
            i = q.popleft()
            f = int(feat[i])
            h.update(np.asarray([f, int(bins[i]) if f >= 0 else 0, int(bool(is_cat[i]))],
                                dtype=np.int64).tobytes())
            if f >= 0:
                h.update(np.asarray([thr[i]], dtype=np.float64).tobytes())
                if is_cat[i]:
                    h.update(np.asarray(catmask[i], dtype=np.uint32).tobytes())
                q.append(int(left[i]))
                q.append(int(right[i]))
            else:
                h.update(np.asarray(value[i], dtype=np.float64).reshape(-1).tobytes())
    return h.hexdigest()[:16]


def shard_bounds(n_total: int, rank: int, world: int) -> Tuple[int, int]:
    return n_total * rank // world, n_total * (rank + 1) // world


__all__ = ["philox_normal", "regression_shard", "forest_digest", "shard_bounds"]
