"""Helpers shared by the native-op wrappers (``kernels``, ``relops``): raw pointers and streams for the HIP
entry points, the device test, and the one-copy pinned upload of small host tables."""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else t.data_ptr()


def _stream(dev: torch.device):
    return torch.cuda.current_stream(dev).cuda_stream


def _native(t: torch.Tensor) -> bool:
    return t.is_cuda


_TORCH_DT = {}


def upload(dev, *arrays):
    """Host numpy arrays -> device tensors through ONE pinned staging block and one async copy.

    A pageable ``torch.from_numpy(x).to(dev)`` synchronises the stream (the copy must finish before the host
    buffer may change), so every small per-level table used to drain the GPU queue and expose the host work
    that followed as idle time (up to 0.5 ms per copy at the 8-GPU shard shape).  The staging block comes from
    PyTorch's caching pinned-host allocator, which keeps it until the copy's stream event has passed.
    On the CPU the arrays are wrapped as they are (no copy)."""
    dev = torch.device(dev)
    arrs = [np.ascontiguousarray(a) for a in arrays]
    if dev.type != "cuda":
        return [torch.from_numpy(a) for a in arrs]
    offs, o = [], 0
    for a in arrs:
        o = -(-o // 16) * 16
        offs.append(o)
        o += a.nbytes
    host = torch.empty(max(o, 16), dtype=torch.uint8, pin_memory=True)
    hv = host.numpy()
    for a, off in zip(arrs, offs):
        if a.nbytes:
            hv[off:off + a.nbytes] = a.reshape(-1).view(np.uint8)
    dbuf = host.to(dev, non_blocking=True)
    out = []
    for a, off in zip(arrs, offs):
        tdt = _TORCH_DT.get(a.dtype)
        if tdt is None:
            tdt = _TORCH_DT[a.dtype] = torch.from_numpy(np.empty(0, dtype=a.dtype)).dtype
        out.append(dbuf[off:off + a.nbytes].view(tdt).reshape(a.shape))
    return out
