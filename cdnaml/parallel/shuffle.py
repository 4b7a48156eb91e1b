"""Columnar hash/range shuffles as RCCL all-to-all.

``exchange`` moves rows of a partition to their owner ranks: one counts
all-to-all plus one payload all-to-all per column buffer.  String columns
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
    """Send row i of ``batch`` to rank ``dest[i]``; return the rows received."""
    if not comm.distributed:
        return batch
    W = comm.world_size
    batch = unify_global_dictionaries(comm, batch)
    from ..ops import kernels as K
    order, counts = K.partition_dest(dest, W)  # K16 stable counting sort (HIP on the GPU)
    counts = counts.cpu().tolist()
    sorted_b = batch.take(order)
    out_cols = {}
    recv_n = None
    for k, c in sorted_b.columns.items():
        chunks = list(torch.split(c.values, counts))
        got = comm.all_to_all_v(chunks)
        vals = torch.cat(got) if got else c.values[:0]
        valid = None
        has_null = torch.tensor([1.0 if c.valid is not None else 0.0], device=comm.device)
        comm.all_reduce(has_null, "max")
        if float(has_null) > 0:
            vchunks = list(torch.split(c.valid_mask(), counts))
            valid = torch.cat(comm.all_to_all_v(vchunks))
        out_cols[k] = ColumnData(vals, c.dtype, valid, c.dictionary, c.meta)
        recv_n = vals.shape[0]
    if recv_n is None:
        recv_n = 0
    return Batch(out_cols, recv_n, batch.device)


def hash_keys(batch: Batch, keys: List[str]) -> torch.Tensor:
    """Per-row 31-bit hash of the key columns (stable across ranks after dictionary unification)."""
    from ..sql.functions import _hash_column, _mix
    h = torch.full((batch.n,), 17, dtype=torch.int64, device=batch.device)
    for k in keys:
        h = _mix(h * 31 + _hash_column(batch.columns[k])) & 0x7FFFFFFF
    return h
