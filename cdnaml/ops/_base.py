"""Helpers shared by the native-op wrappers (``kernels``, ``relops``): raw pointers and streams for the HIP
entry points, the device test, and the one-copy pinned upload of small host tables."""
from __future__ import annotations

import threading
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


# upload's staging blocks: a ring of pinned host blocks reused once their copy's event has passed.  PyTorch's caching
# pinned allocator recycles a block only after the OLDEST pending copy event has passed (it processes them in
# order), so behind a long kernel a per-level upload kept calling hipHostMalloc -- which waits for the device: a
# ~25-55 us idle gap per step at the 8-GPU shard size (hip API trace, profiles/r6/headline_ab.md).
PINNED_RING = 32
PINNED_SLOT = 64 << 10


class _PinnedRing:
    def __init__(self):
        self.lock = threading.Lock()
        self.slots = []   # [pinned uint8 tensor, event or None]
        self.i = 0

    def take(self, nbytes: int):
        """(slot index, pinned uint8 view of nbytes) -- call ``done(slot, stream)`` once the copy is queued."""
        with self.lock:
            if not self.slots:  # every slot at the first upload: the allocations stay out of later (timed) steps
                self.slots = [[torch.empty(PINNED_SLOT, dtype=torch.uint8, pin_memory=True), None]
                              for _ in range(PINNED_RING)]
            k = self.i
            self.i = (self.i + 1) % PINNED_RING
            ev = self.slots[k][1]
            if ev is not None and not ev.query():
                ev.synchronize()  # the slot's previous copy (PINNED_RING uploads ago) is still queued
            if self.slots[k][0].numel() < nbytes:
                self.slots[k][0] = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
            return k, self.slots[k][0][:nbytes]

    def done(self, k: int, stream) -> None:
        with self.lock:
            ev = self.slots[k][1]
            if ev is None:
                ev = self.slots[k][1] = torch.cuda.Event()
            ev.record(stream)


_RING = _PinnedRing()


def upload(dev, *arrays):
    """Host numpy arrays -> device tensors through ONE pinned staging block and one async copy.

    A pageable ``torch.from_numpy(x).to(dev)`` synchronises the stream (the copy must finish before the host
    buffer may change), so every small per-level table used to drain the GPU queue and expose the host work
    that followed as idle time (up to 0.5 ms per copy at the 8-GPU shard shape).  The staging block is a slot of
    a ring of pinned blocks (``_PinnedRing``), reused once the copy's stream event has passed.
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
    k, host = _RING.take(max(o, 16))
    hv = host.numpy()
    for a, off in zip(arrs, offs):
        if a.nbytes:
            hv[off:off + a.nbytes] = a.reshape(-1).view(np.uint8)
    dbuf = host.to(dev, non_blocking=True)
    _RING.done(k, torch.cuda.current_stream(dev))
    out = []
    for a, off in zip(arrs, offs):
        tdt = _TORCH_DT.get(a.dtype)
        if tdt is None:
            tdt = _TORCH_DT[a.dtype] = torch.from_numpy(np.empty(0, dtype=a.dtype)).dtype
        out.append(dbuf[off:off + a.nbytes].view(tdt).reshape(a.shape))
    return out
