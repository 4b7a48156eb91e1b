"""Columnar hash/range shuffles as RCCL all-to-all.

``exchange`` moves rows of a partition to their owner ranks: one counts
all-to-all plus ONE payload all-to-all of the row-packed column bytes.  String columns
are first re-encoded against a globally unified dictionary (all-gather of
the distinct values, which is tiny next to the rows) so only int32 codes
cross xGMI.
"""
from __future__ import annotations

from typing import List

import numpy as np
import torch

from ..sql import types as T
from ..sql.batch import Batch, ColumnData, recode


def unify_global_dictionaries(comm, batch: Batch) -> Batch:
    """Make every string column's dictionary identical on all ranks."""
    if not comm.distributed:
        return batch
    names = [k for k, c in batch.columns.items() if isinstance(c.dtype, T.StringType)]
    if not names:
        return batch
    local = {k: list(batch.columns[k].dictionary.tolist()) if batch.columns[k].dictionary is not None else []
             for k in names}
    allv = comm.all_gather_object(local)
    cols = dict(batch.columns)
    for k in names:
        uni = np.array(sorted(set(v for d in allv for v in d[k])), dtype=object)
        cols[k] = recode(cols[k], uni)
    return Batch(cols, batch.n, batch.device)


def exchange(comm, batch: Batch, dest: torch.Tensor) -> Batch:
    """Send row i of ``batch`` to rank ``dest[i]``; return the rows received.

    All columns travel together: each row's column bytes (and a validity byte for every column that has nulls
    on any rank) are packed into one [n, R] byte matrix, and every rank's send counts and null flags travel in
    one small all-gather, so a shuffle is that all-gather (the only host read) plus ONE payload all-to-all
    whatever the column count."""
    if not comm.distributed:
        return batch
    W = comm.world_size
    batch = unify_global_dictionaries(comm, batch)
    from ..ops import kernels as K
    order, counts = K.partition_dest(dest, W)  # K16 stable counting sort (HIP on the GPU)
    sorted_b = batch.take(order)
    names = list(sorted_b.columns)
    cols = [sorted_b.columns[k] for k in names]
    n = sorted_b.n
    # ONE all-gather (and one host read) carries every rank's send counts and column null flags: each rank
    # reads its receive counts (column `rank` of the count matrix) and the max of the flags from it
    flags = torch.tensor([1 if c.valid is not None else 0 for c in cols], dtype=torch.int64)
    info = torch.cat([counts.to(torch.int64).to(comm.device), flags.to(comm.device)])
    allinfo = comm.all_gather_tensor(info).cpu()
    counts = counts.cpu().tolist() if counts.is_cuda else counts.tolist()
    recv_counts = allinfo[:, comm.rank].tolist()
    nullable = [bool(f) for f in allinfo[:, W:].amax(0).tolist()] if cols else []
    parts, layout = [], []
    for c, nb in zip(cols, nullable):
        v = c.values.contiguous()
        tail = tuple(v.shape[1:])
        width = int(np.prod(tail)) if tail else 1
        raw = v.reshape(n, width)
        raw = raw.view(torch.uint8) if raw.dtype != torch.bool else raw.to(torch.uint8)
        parts.append(raw)
        layout.append((v.dtype, tail, raw.shape[1], nb))
        if nb:
            parts.append(c.valid_mask().to(torch.uint8).reshape(n, 1))
    packed = torch.cat(parts, 1) if parts else torch.zeros((n, 0), dtype=torch.uint8, device=batch.device)
    got = comm.all_to_all_v(list(torch.split(packed, counts)), recv_counts)
    recv = torch.cat(got) if got else packed[:0]
    m = recv.shape[0]
    out_cols, o = {}, 0
    for k, c, (dt, tail, nbytes, nb) in zip(names, cols, layout):
        # a fresh contiguous buffer (offset 0, row stride nbytes): views as wider dtypes need both
        blk = torch.empty((m, nbytes), dtype=torch.uint8, device=recv.device)
        blk.copy_(recv[:, o:o + nbytes])
        o += nbytes
        vals = (blk.view(dt) if dt != torch.bool else blk.bool()).reshape((m,) + tail)
        valid = None
        if nb:
            valid = recv[:, o].bool()
            o += 1
        out_cols[k] = ColumnData(vals, c.dtype, valid, c.dictionary, c.meta)
    return Batch(out_cols, m, batch.device)


def hash_keys(batch: Batch, keys: List[str]) -> torch.Tensor:
    """Per-row 31-bit hash of the key columns (stable across ranks after dictionary unification)."""
    from ..sql.functions import _hash_column, _mix
    h = torch.full((batch.n,), 17, dtype=torch.int64, device=batch.device)
    for k in keys:
        h = _mix(h * 31 + _hash_column(batch.columns[k])) & 0x7FFFFFFF
    return h
