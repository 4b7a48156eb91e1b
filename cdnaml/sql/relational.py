"""Partition-local relational algorithms on device tensors.

On the GPU (K16, ``csrc/kernels/hashagg.hip``) the key columns become one int64 *key word* per row (the value
bits of a single column, or the columns packed mixed-radix over their value ranges) and the operators run in hash
tables: groupBy aggregates count / sum / avg / min / max / first / last in the slots of partitioned LDS tables,
dropDuplicates keeps the first row of every key (insert-if-absent + atomicMin of the row id), and joins build a
table on the right input and probe it with the left rows.  Only the G distinct groups are sorted (so results come
out in key order, as before); no operator sorts the n input rows.

Everything else (the CPU, aggregates such as percentiles / stddev / collect_*, float keys among several columns,
a partition whose keys overflow its table) uses the portable path: each key column is reduced to a code
(string dictionary code, or the ``torch.unique`` inverse of numeric values), codes are combined mixed-radix
into one int64 and densified again — after that every operator is a sort, ``searchsorted`` or a segmented
``scatter_reduce``.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from ..ops import kernels as K
from ..ops import relops as R
from . import types as T
from .batch import Batch, ColumnData, column_from_numpy, concat_columns, unify_dictionaries


def column_codes(c: ColumnData) -> Tuple[torch.Tensor, int]:
    """Dense int64 codes (nulls -> 0, values -> 1..k) and cardinality k+1."""
    v = c.values
    if v.dim() == 2:
        _, inv = torch.unique(v, dim=0, return_inverse=True)
        codes = inv + 1
    elif isinstance(c.dtype, T.StringType):
        codes = v.long() + 1
        if codes.numel():
            inv, _ = K.dense_ids(codes)  # K16 hash table on the GPU (sorted-rank ids, like torch.unique)
            codes = inv + 1
    else:
        x = v
        if x.dtype.is_floating_point:
            x = torch.where(x == 0, torch.zeros_like(x), x)  # -0.0 == 0.0
        inv, _ = K.dense_ids(x)
        codes = inv + 1
    if c.valid is not None:
        codes = torch.where(c.valid, codes, torch.zeros_like(codes))
    k = int(codes.max()) + 1 if codes.numel() else 1
    return codes, k


def combine_codes(cols: List[ColumnData], n: int, device) -> Tuple[torch.Tensor, int]:
    """Dense group id per row for the tuple of key columns; returns (gid, ngroups)."""
    if not cols:
        return torch.zeros(n, dtype=torch.int64, device=device), (1 if n else 0)
    combined = None
    for c in cols:
        codes, k = column_codes(c)
        if combined is None:
            combined = codes
        else:
            combined = combined * k + codes
            if combined.numel() and int(combined.max()) > 2 ** 60 // max(k, 1):
                _, combined = torch.unique(combined, return_inverse=True)
    gid, G = K.dense_ids(combined)
    return gid, G


def first_index_per_group(gid: torch.Tensor, ngroups: int) -> torch.Tensor:
    return K.group_first(gid, ngroups)


# ------------------------------------------------------------ K16 key words (GPU)
_EMPTY = -(1 << 63)
_INT_DT = (torch.int8, torch.uint8, torch.int16, torch.int32, torch.int64, torch.bool)


def _native_rows(dev, *ns) -> bool:
    return dev.type == "cuda" and sum(ns) >= R.HASH_MIN_ROWS and max(ns) < (1 << 31)


def _col_kind(c: ColumnData) -> Optional[str]:
    if c.values.dim() != 1:
        return None
    if isinstance(c.dtype, T.StringType):
        return "str"
    if c.values.dtype in (torch.float32, torch.float64):
        return "float"
    if c.values.dtype in _INT_DT:
        return "int"
    return None


def _key_words(sides: List[List[ColumnData]]):
    """One int64 word per row for every side's key tuple, equal exactly when the tuples are equal (nulls equal
    nulls), plus the order kind: 'int' (the signed word order is the tuple order, nulls first) or 'float' (a
    single float column: sort groups by value).  None when the keys have no exact word (float among several
    columns, > 2^62 packed combinations)."""
    cols0 = sides[0]
    kinds = [_col_kind(c) for c in cols0]
    for side in sides[1:]:
        if [_col_kind(c) for c in side] != kinds:
            return None
    if any(k is None for k in kinds):
        return None
    if len(cols0) == 1 and kinds[0] == "float":
        out = []
        for side in sides:
            c = side[0]
            w = K._key_bits(c.values)
            out.append(w if c.valid is None else torch.where(c.valid, w, torch.full_like(w, _EMPTY)))
        return out, "float"
    if len(cols0) == 1 and all(c.valid is None or c.values.dtype != torch.int64 for c in (s[0] for s in sides)):
        out = []
        for side in sides:
            c = side[0]
            w = c.values.to(torch.int64)
            out.append(w if c.valid is None else torch.where(c.valid, w, torch.full_like(w, _EMPTY)))
        return out, "int"
    if "float" in kinds:
        return None
    # mixed-radix packing over the joint value range of every column (one host sync for all ranges)
    stats = []
    for j, kind in enumerate(kinds):
        if kind == "str":
            continue
        for side in sides:
            c = side[j]
            v = c.values.to(torch.int64) if c.values.dtype == torch.bool else c.values
            if c.valid is not None:
                v = torch.where(c.valid, v, v.new_full((), int(torch.iinfo(v.dtype).max)))
                w = torch.where(c.valid, c.values.to(v.dtype), v.new_full((), int(torch.iinfo(v.dtype).min)))
            else:
                w = v
            if v.numel():
                stats.append(torch.stack([v.min().long(), w.max().long(), torch.ones((), dtype=torch.int64,
                                                                                     device=v.device)]))
            else:
                stats.append(torch.tensor([0, 0, 0], dtype=torch.int64, device=v.device))
    st = torch.stack(stats).cpu().tolist() if stats else []
    lo, radix, it = [], [], iter(st)
    for j, kind in enumerate(kinds):
        if kind == "str":
            nd = max(len(side[j].dictionary) if side[j].dictionary is not None else 0 for side in sides)
            lo.append(0)
            radix.append(nd + 1)
            continue
        mins, maxs = [], []
        for _ in sides:
            a, b, ok = next(it)
            if ok:
                mins.append(a)
                maxs.append(b)
        a = min(mins) if mins else 0
        b = max(maxs) if maxs else 0
        if b < a:          # all null
            a = b = 0
        lo.append(a)
        radix.append(b - a + 2)
    prod = 1
    for r in radix:
        prod *= r
    if prod >= (1 << 62):
        return None
    out = []
    for side in sides:
        n = side[0].values.shape[0]
        out.append(K.pack_keys([(c.values, c.valid, lo[j], radix[j]) for j, c in enumerate(side)], n,
                               side[0].values.device))
    return out, "int"


def _all_valid(cols: List[ColumnData]) -> Optional[torch.Tensor]:
    m = None
    for c in cols:
        if c.valid is not None:
            m = c.valid if m is None else (m & c.valid)
    return m


# ----------------------------------------------------------------- aggregation
def aggregate(batch: Batch, keys: List[str], aggs: List[Tuple[str, object]]) -> Batch:
    """Local hash aggregation: keys + one output column per (name, AggExpr)."""
    from .column import EvalContext
    n = batch.n
    dev = batch.device
    if keys and _native_rows(dev, n):
        out = _aggregate_native(batch, keys, aggs)
        if out is not None:
            return out
    gid, G = combine_codes([batch.columns[k] for k in keys], n, dev)
    if not keys:
        gid = torch.zeros(n, dtype=torch.int64, device=dev)
        G = 1
    first = first_index_per_group(gid, G) if G else torch.zeros(0, dtype=torch.int64, device=dev)
    out: Dict[str, ColumnData] = {}
    if keys and G:
        for k in keys:
            out[k] = batch.columns[k].take(first)
    elif keys:
        for k in keys:
            out[k] = batch.columns[k].slice(0, 0)
    ctx = EvalContext()
    for name, agg in aggs:
        out[name] = _agg_one(batch, agg, gid, G, first, ctx)
    return Batch(out, G, dev)


def _aggregate_native(batch: Batch, keys: List[str], aggs) -> Optional[Batch]:
    """K16 groupBy in partitioned LDS hash tables (hashagg.hip): count(*), count(col), sum, avg, min, max, first
    and last come out of the table slots; any other aggregate is computed by the portable code from every row's
    group id, which the same kernel writes.  None -> the caller takes the portable path."""
    from .column import EvalContext
    n, dev = batch.n, batch.device
    kw = _key_words([[batch.columns[k] for k in keys]])
    if kw is None:
        return None
    (words,), kind = kw
    ctx = EvalContext()
    values, vidx, accs, plan = [], {}, [], []
    generic = False

    def value(expr, c):
        k = str(expr)
        if k not in vidx:
            if len(values) == R.HP_MAX_ACC:
                return None
            vidx[k] = len(values)
            values.append((c.values, c.valid))
        return vidx[k]

    def acc(op, j):
        if len(accs) == R.HP_MAX_ACC:
            return None
        accs.append((op, j))
        return len(accs) - 1

    for name, agg in aggs:
        if agg.x is None:
            plan.append((name, "count*", None, ()))
            continue
        c = agg.x.eval(batch, ctx)
        simple = (not agg.distinct and c.values.dim() == 1 and c.values.dtype in R._VAL_DT and
                  not isinstance(c.dtype, T.StringType))
        step = None
        if agg.kind == "first" and not agg.distinct:
            step = (name, "first", c, ())
        elif agg.kind == "last" and not agg.distinct:
            a = acc("last", 0)
            step = None if a is None else (name, "last", c, (a,))
        elif agg.kind == "count" and not agg.distinct and c.valid is None:
            step = (name, "count*", None, ())
        elif simple and agg.kind in ("count", "sum", "avg", "min", "max"):
            j = value(agg.x, c)
            if j is not None:
                ids = []
                if agg.kind in ("sum", "avg", "min", "max"):
                    ids.append(acc(agg.kind if agg.kind != "avg" else "sum", j))
                if agg.kind == "count" or (agg.kind in ("sum", "avg") and c.valid is not None):
                    ids.append(acc("count", j))
                if None not in ids:
                    step = (name, agg.kind, c, tuple(ids))
        if step is None:
            generic = True
            step = (name, "generic", agg, ())
        plan.append(step)
    res = K.hash_groups(words, values, accs, mode=2 if generic else 0)
    if res is None:
        return None
    G, pos = res["G"], res["pos"]
    first_u = res["first"][pos].long()
    if kind == "float":
        kc = batch.columns[keys[0]]
        kv = kc.values[first_u].double()
        order = torch.argsort(kv, stable=True)
        if kc.valid is not None:
            order = order[torch.argsort(kc.valid[first_u][order].to(torch.int8), stable=True)]
    else:
        order = torch.argsort(res["key"][pos], stable=True)
    spos = pos[order]
    first = first_u[order]
    cnt = res["cnt"][spos].long()
    gid = None
    if generic:
        rank = torch.empty(n, dtype=torch.int64, device=dev)
        rank[spos] = torch.arange(G, device=dev)
        gid = rank[res["gpos"].long()]
    out: Dict[str, ColumnData] = {}
    for k in keys:
        out[k] = batch.columns[k].take(first)
    ctx = EvalContext()
    for name, what, c, ids in plan:
        if what == "count*":
            out[name] = ColumnData(cnt, T.LongType())
            continue
        if what == "first":
            out[name] = c.take(first)
            continue
        if what == "last":
            out[name] = c.take(res["acc"][ids[0]][spos])
            continue
        if what == "generic":
            out[name] = _agg_one(batch, c, gid, G, first, ctx)
            continue
        a = [res["acc"][i][spos] for i in ids]
        if what == "count":
            out[name] = ColumnData(a[0], T.LongType())
            continue
        nn = a[-1] if (what in ("sum", "avg") and c.valid is not None) else None
        if what in ("sum", "avg"):
            s_ = a[0].view(torch.float64)
            vnull = None if nn is None else (nn > 0)
            if vnull is not None and bool(vnull.all()):
                vnull = None
            if what == "avg":
                out[name] = ColumnData(s_ / (cnt if nn is None else nn).clamp_min(1).double(), T.DoubleType(), vnull)
            elif isinstance(c.dtype, T.IntegralType):
                out[name] = ColumnData(s_.to(torch.int64), T.LongType(), vnull)
            else:
                out[name] = ColumnData(s_, T.DoubleType(), vnull)
            continue
        u = a[0]
        has = u != (-1 if what == "min" else 0)
        r = torch.where(has, K.ordered_to_double(u), torch.zeros((), dtype=torch.float64, device=dev))
        vnull = None if bool(has.all()) else has
        dt = c.dtype
        if isinstance(dt, (T.IntegralType, T.DateType, T.TimestampType, T.BooleanType)):
            out[name] = ColumnData(r.to(dt.torch_dtype), dt, vnull)
        else:
            out[name] = ColumnData(r.to(c.values.dtype), dt, vnull)
    return Batch(out, G, dev)


def _seg_sum(vals, gid, G, dtype=torch.float64):
    if dtype == torch.float64 and vals.dim() == 1:
        return K.group_sum(vals, gid, G)  # LDS-privatised for few groups (no contended global fp64 atomics)
    s = torch.zeros(G, dtype=dtype, device=vals.device)
    s.index_add_(0, gid, vals.to(dtype))
    return s


def _agg_one(batch: Batch, agg, gid, G, first, ctx) -> ColumnData:
    kind = agg.kind
    dev = batch.device
    if agg.x is None:  # count(*)
        cnt = torch.bincount(gid, minlength=G).to(torch.int64) if batch.n else torch.zeros(G, dtype=torch.int64,
                                                                                           device=dev)
        return ColumnData(cnt[:G], T.LongType())
    c = agg.x.eval(batch, ctx)
    if kind == "summarizer":
        from ..ml.stat import summarize_groups
        w = None if agg.param.get("weight") is None else agg.param["weight"].eval(batch, ctx)
        return summarize_groups(c, w, gid, G, agg.param)
    valid = c.valid_mask()
    if agg.distinct:
        # dedupe (gid, value) pairs first
        vcodes, k = column_codes(c)
        pair = gid * k + vcodes
        keep = valid.clone()
        if batch.n:
            u, inv = torch.unique(pair, return_inverse=True)
            fi = first_index_per_group(inv, u.numel())
            mask = torch.zeros(batch.n, dtype=torch.bool, device=dev)
            mask[fi] = True
            keep = keep & mask
        valid = keep
    if kind == "count":
        cnt = torch.zeros(G, dtype=torch.int64, device=dev)
        cnt.index_add_(0, gid, valid.to(torch.int64))
        return ColumnData(cnt, T.LongType())
    if kind in ("first", "last"):
        idx = torch.arange(batch.n, device=dev)
        if kind == "first":
            pos = torch.full((G,), batch.n, dtype=torch.int64, device=dev)
            pos.scatter_reduce_(0, gid, idx, reduce="amin", include_self=True)
        else:
            pos = torch.full((G,), -1, dtype=torch.int64, device=dev)
            pos.scatter_reduce_(0, gid, idx, reduce="amax", include_self=True)
        return c.take(pos.clamp(0, max(batch.n - 1, 0))) if batch.n else c.slice(0, 0)
    if kind in ("collect_list", "collect_set"):
        vals = c.to_numpy()
        g = gid.cpu().numpy()
        lists = [[] for _ in range(G)]
        vm = valid.cpu().numpy()
        for i in range(batch.n):
            if vm[i]:
                v = vals[i]
                lists[g[i]].append(v.item() if isinstance(v, np.generic) else v)
        if kind == "collect_set":
            lists = [list(dict.fromkeys(x)) for x in lists]
        return ColumnData(torch.zeros(G, device=dev), T.ArrayType(c.dtype), meta={"_py": lists})
    if isinstance(c.dtype, T.StringType) and kind in ("min", "max"):
        v = c.values.long()
        fill = 2 ** 40 if kind == "min" else -1
        v = torch.where(valid, v, torch.full_like(v, fill))
        r = torch.full((G,), fill, dtype=torch.int64, device=dev)
        r.scatter_reduce_(0, gid, v, reduce="amin" if kind == "min" else "amax", include_self=True)
        ok = (r != fill)
        return ColumnData(torch.where(ok, r, torch.zeros_like(r)).to(torch.int32), c.dtype,
                          None if bool(ok.all()) else ok, c.dictionary)
    x = c.values.to(torch.float64) if c.values.dim() == 1 else c.values.to(torch.float64)
    xz = torch.where(valid, x, torch.zeros_like(x))
    cnt = K.group_sum(None if c.valid is None else valid.to(torch.float64), gid, G)
    nonempty = cnt > 0
    vnull = None if bool(nonempty.all()) else nonempty
    if kind == "sum":
        s = _seg_sum(xz, gid, G)
        if isinstance(c.dtype, T.IntegralType):
            return ColumnData(s.to(torch.int64), T.LongType(), vnull)
        return ColumnData(s, T.DoubleType(), vnull)
    if kind == "avg":
        s = _seg_sum(xz, gid, G)
        return ColumnData(s / cnt.clamp_min(1), T.DoubleType(), vnull)
    if kind in ("min", "max"):
        fill = float("inf") if kind == "min" else float("-inf")
        xv = torch.where(valid, x, torch.full_like(x, fill))
        r = torch.full((G,), fill, dtype=torch.float64, device=dev)
        r.scatter_reduce_(0, gid, xv, reduce="amin" if kind == "min" else "amax", include_self=True)
        r = torch.where(nonempty, r, torch.zeros_like(r))
        dt = c.dtype
        if isinstance(dt, (T.IntegralType, T.DateType, T.TimestampType, T.BooleanType)):
            return ColumnData(r.to(dt.torch_dtype), dt, vnull)
        return ColumnData(r.to(c.values.dtype), dt, vnull)
    if kind in ("stddev", "stddev_samp", "stddev_pop", "variance", "var_samp", "var_pop", "skewness", "kurtosis"):
        s = _seg_sum(xz, gid, G)
        mu = s / cnt.clamp_min(1)
        dev2 = torch.where(valid, x - mu[gid], torch.zeros_like(x))
        m2 = _seg_sum(dev2 * dev2, gid, G)
        if kind in ("skewness", "kurtosis"):
            m3 = _seg_sum(dev2 ** 3, gid, G)
            m4 = _seg_sum(dev2 ** 4, gid, G)
            nn = cnt.clamp_min(1)
            if kind == "skewness":
                r = torch.sqrt(nn) * m3 / m2.clamp_min(1e-300) ** 1.5
            else:
                r = nn * m4 / (m2 * m2).clamp_min(1e-300) - 3.0
            return ColumnData(r, T.DoubleType(), vnull)
        pop = kind in ("stddev_pop", "var_pop")
        denom = cnt if pop else cnt - 1
        var = m2 / denom.clamp_min(1)
        ok = denom > 0
        var = torch.where(ok, var, torch.full_like(var, float("nan")))
        r = torch.sqrt(var) if kind.startswith("stddev") else var
        return ColumnData(r, T.DoubleType(), vnull)
    if kind == "percentile":
        qs = agg.param
        multi = isinstance(qs, (list, tuple))
        qlist = list(qs) if multi else [qs]
        order = torch.argsort(torch.where(valid, x, torch.full_like(x, float("inf"))), stable=True)
        order = order[torch.argsort(gid[order], stable=True)]
        gs = gid[order]
        starts = torch.zeros(G + 1, dtype=torch.int64, device=dev)
        starts[1:] = torch.cumsum(cnt.to(torch.int64), 0)
        gcount_all = torch.bincount(gs, minlength=G)
        gstart_all = torch.zeros(G, dtype=torch.int64, device=dev)
        gstart_all[1:] = torch.cumsum(gcount_all, 0)[:-1]
        res = []
        for q in qlist:
            # Spark percentile_approx: smallest value with rank >= ceil(q * n)
            rk = torch.ceil(q * cnt).to(torch.int64).clamp_min(1) - 1
            pos = gstart_all + rk.clamp_min(0)
            pos = pos.clamp(0, max(batch.n - 1, 0))
            res.append(x[order][pos] if batch.n else torch.zeros(G, dtype=torch.float64, device=dev))
        if multi:
            return ColumnData(torch.stack(res, 1), T.ArrayType(T.DoubleType()), vnull)
        return ColumnData(res[0], T.DoubleType(), vnull)
    raise ValueError(f"unsupported aggregate {kind}")


# ----------------------------------------------------------------------- sort
def sort_indices(batch: Batch, orders) -> torch.Tensor:
    """Stable multi-key sort permutation. orders: list of (ColumnData, ascending, nulls_first)."""
    n = batch.n
    perm = torch.arange(n, device=batch.device)
    for c, asc, nulls_first in reversed(orders):
        c = c.take(perm)
        if isinstance(c.dtype, T.StringType):
            key = c.values.to(torch.float64)
        elif c.values.dim() == 2:
            key = c.values[:, 0].to(torch.float64)
        else:
            key = c.values.to(torch.float64)
        if key.dtype.is_floating_point:
            nan = torch.isnan(key)
            # Spark: NaN is larger than any other value
            key = torch.where(nan, torch.full_like(key, float("inf")), key)
        if not asc:
            key = -key
        valid = c.valid_mask()
        big = float("inf")
        nullkey = torch.full_like(key, -big if nulls_first else big)
        key = torch.where(valid, key, nullkey)
        # tie-break by null flag explicitly (inf ties)
        nulls = (~valid).to(torch.int8)
        if nulls_first:
            nulls = -nulls
        p1 = torch.argsort(key, stable=True)
        p2 = torch.argsort(nulls[p1], stable=True)
        perm = perm[p1][p2]
    return perm


# ----------------------------------------------------------------------- join
def join(left: Batch, right: Batch, lkeys: List[str], rkeys: List[str], how: str,
         drop_right_keys: bool = True) -> Batch:
    """Local equi-join of two partitions (keys already co-partitioned)."""
    dev = left.device
    how = {"inner": "inner", "left": "left", "leftouter": "left", "left_outer": "left", "right": "right",
           "rightouter": "right", "right_outer": "right", "outer": "full", "full": "full", "fullouter": "full",
           "full_outer": "full", "semi": "semi", "leftsemi": "semi", "left_semi": "semi", "anti": "anti",
           "leftanti": "anti", "left_anti": "anti", "cross": "cross"}[how.lower()]
    nl, nr = left.n, right.n
    if how != "cross" and _native_rows(dev, nl, nr):
        out = _join_native(left, right, lkeys, rkeys, how, drop_right_keys)
        if out is not None:
            return out
    if how == "cross":
        li = torch.arange(nl, device=dev).repeat_interleave(nr)
        ri = torch.arange(nr, device=dev).repeat(nl)
        return _assemble(left, right, li, ri, None, None, [], drop_right_keys=False)
    lk = [concat_columns([ca, cb]) for ca, cb in _join_key_columns(left, right, lkeys, rkeys)]
    gid, G = combine_codes(lk, nl + nr, dev)
    # null keys never match
    nullany = torch.zeros(nl + nr, dtype=torch.bool, device=dev)
    for c in lk:
        nullany |= ~c.valid_mask()
    lg, rg = gid[:nl], gid[nl:]
    lnull, rnull = nullany[:nl], nullany[nl:]
    rg_eff = torch.where(rnull, torch.full_like(rg, -1), rg)
    rorder = torch.argsort(rg_eff, stable=True)
    rsorted = rg_eff[rorder]
    lo = torch.searchsorted(rsorted, lg, right=False)
    hi = torch.searchsorted(rsorted, lg, right=True)
    cnt = torch.where(lnull, torch.zeros_like(hi), hi - lo)
    if how == "semi":
        return left.filter(cnt > 0)
    if how == "anti":
        return left.filter(cnt == 0)
    li = torch.arange(nl, device=dev).repeat_interleave(cnt)
    start = torch.repeat_interleave(lo, cnt)
    off = torch.arange(li.numel(), device=dev) - torch.repeat_interleave(torch.cumsum(cnt, 0) - cnt, cnt)
    ri = rorder[start + off] if li.numel() else torch.zeros(0, dtype=torch.int64, device=dev)
    lmiss = rmiss = None
    if how in ("left", "full"):
        lmiss = torch.nonzero(cnt == 0).flatten()
    if how in ("right", "full"):
        matched = torch.zeros(nr, dtype=torch.bool, device=dev)
        if ri.numel():
            matched[ri] = True
        rmiss = torch.nonzero(~matched).flatten()
    return _assemble(left, right, li, ri, lmiss, rmiss, list(zip(lkeys, rkeys)), drop_right_keys, how)


def _join_key_columns(left: Batch, right: Batch, lkeys, rkeys):
    """Key column pairs in one representation on both sides (shared string dictionary, common numeric dtype)."""
    pairs = []
    for a, b in zip(lkeys, rkeys):
        ca, cb = left.columns[a], right.columns[b]
        if isinstance(ca.dtype, T.StringType) or isinstance(cb.dtype, T.StringType):
            from .column import _cast
            ca = ca if isinstance(ca.dtype, T.StringType) else _cast(ca, T.StringType())
            cb = cb if isinstance(cb.dtype, T.StringType) else _cast(cb, T.StringType())
            ca, cb = unify_dictionaries([ca, cb])
        elif ca.values.dtype != cb.values.dtype:
            if ca.values.dtype in _INT_DT and cb.values.dtype in _INT_DT:
                ca = ColumnData(ca.values.to(torch.int64), T.LongType(), ca.valid)
                cb = ColumnData(cb.values.to(torch.int64), T.LongType(), cb.valid)
            else:
                ca = ColumnData(ca.values.to(torch.float64), T.DoubleType(), ca.valid)
                cb = ColumnData(cb.values.to(torch.float64), T.DoubleType(), cb.valid)
        pairs.append((ca, cb))
    return pairs


def _join_native(left: Batch, right: Batch, lkeys, rkeys, how: str, drop_right_keys: bool) -> Optional[Batch]:
    """K16 hash join: a table of the right input's key words (hashagg.hip join_build), probed by every left row
    (join_probe).  Output order is the portable path's: matched pairs by left row, then by right row."""
    dev = left.device
    nl, nr = left.n, right.n
    pairs = _join_key_columns(left, right, lkeys, rkeys)
    lcols = [p[0] for p in pairs]
    rcols = [p[1] for p in pairs]
    kw = _key_words([lcols, rcols])
    if kw is None:
        return None
    (lw, rw), _ = kw
    lvalid, rvalid = _all_valid(lcols), _all_valid(rcols)
    tab = K.join_table(rw, rvalid)
    ovf, maxc = torch.stack([tab.ovf[0].long(), tab.bcnt.max().long()]).cpu().tolist()
    if ovf:
        return None
    ri_all, cnt_l, slot_l = K.join_probe(lw, lvalid, tab, want_cnt=maxc > 1, want_slot=maxc > 1)
    if how == "semi":
        return left.filter(ri_all >= 0)
    if how == "anti":
        return left.filter(ri_all < 0)
    if maxc <= 1:
        li = K.compact_mask(ri_all >= 0)
        ri = ri_all[li]
        matched_l = None
    else:
        cnt = cnt_l.long()
        total = int(cnt.sum())
        li = torch.repeat_interleave(torch.arange(nl, device=dev), cnt, output_size=total)
        # build rows grouped by table slot, in row order within a slot (CSR over the slots)
        _, _, rslot = K.join_probe(rw, rvalid, tab, want_slot=True)
        rslot = torch.where(rslot < 0, torch.full_like(rslot, tab.nslots), rslot)
        order_r = torch.argsort(rslot, stable=True)
        bc = tab.bcnt.long()
        start = torch.cumsum(bc, 0) - bc
        within = torch.arange(total, device=dev) - torch.repeat_interleave(torch.cumsum(cnt, 0) - cnt, cnt,
                                                                           output_size=total)
        ri = order_r[start[slot_l[li]] + within] if total else torch.zeros(0, dtype=torch.int64, device=dev)
        matched_l = cnt > 0
    lmiss = rmiss = None
    if how in ("left", "full"):
        lmiss = K.compact_mask(ri_all < 0 if matched_l is None else ~matched_l)
    if how in ("right", "full"):
        matched = torch.zeros(nr, dtype=torch.bool, device=dev)
        if ri.numel():
            matched[ri] = True
        rmiss = K.compact_mask(~matched)
    return _assemble(left, right, li, ri, lmiss, rmiss, list(zip(lkeys, rkeys)), drop_right_keys, how)


def _assemble(left, right, li, ri, lmiss, rmiss, keypairs, drop_right_keys, how="inner"):
    dev = left.device
    cols = {}
    nmatch = li.numel()
    nlm = 0 if lmiss is None else lmiss.numel()
    nrm = 0 if rmiss is None else rmiss.numel()
    total = nmatch + nlm + nrm
    rkeys = {b: a for a, b in keypairs} if drop_right_keys else {}
    # the matched rows of each side in one multi-column gather (K19 on the GPU)
    lt = left.take(li)
    rt = Batch({k: c for k, c in right.columns.items() if k not in rkeys}, right.n, right.device).take(ri)

    for name, c in left.columns.items():
        pieces = [lt.columns[name]]
        if nlm:
            pieces.append(c.take(lmiss))
        if nrm:
            # right-only rows: left side null, but keys come from right
            rname = next((b for a, b in keypairs if a == name), None)
            if rname is not None and drop_right_keys:
                rc = right.columns[rname]
                if isinstance(c.dtype, T.StringType):
                    pieces.append(rc.take(rmiss))
                else:
                    t = rc.take(rmiss)
                    pieces.append(ColumnData(t.values.to(c.values.dtype), c.dtype, t.valid))
            else:
                pieces.append(_null_like(c, nrm))
        cols[name] = concat_columns(pieces) if len(pieces) > 1 else pieces[0]
    for name, c in right.columns.items():
        if name in rkeys:
            continue
        outname = name
        if outname in cols:
            outname = name  # Spark keeps duplicate names; we suffix to stay addressable
            k = 1
            while outname in cols:
                outname = f"{name}_{k}"
                k += 1
        pieces = [rt.columns[name]]
        if nlm:
            pieces.append(_null_like(c, nlm))
        if nrm:
            pieces.append(c.take(rmiss))
        cols[outname] = concat_columns(pieces) if len(pieces) > 1 else pieces[0]
    return Batch(cols, total, dev)


def _null_like(c: ColumnData, n: int) -> ColumnData:
    shape = (n,) + tuple(c.values.shape[1:])
    return ColumnData(torch.zeros(shape, dtype=c.values.dtype, device=c.device), c.dtype,
                      torch.zeros(n, dtype=torch.bool, device=c.device), c.dictionary, c.meta)


# ------------------------------------------------------------------- distinct
def dedup_indices(batch: Batch, keys: List[str]) -> torch.Tensor:
    gid, G = combine_codes([batch.columns[k] for k in keys], batch.n, batch.device)
    if batch.n == 0:
        return torch.zeros(0, dtype=torch.int64, device=batch.device)
    first = first_index_per_group(gid, G)
    return torch.sort(first).values


def dedup_partitions(batch: Batch, keys: List[str], nparts: int) -> Optional[List[Batch]]:
    """K16 dropDuplicates on the GPU: the first row of every key (hash table insert-if-absent, first row by
    atomicMin), split into ``nparts`` output partitions by key hash, rows in input order within a partition.
    None -> the caller takes the portable path."""
    n, dev = batch.n, batch.device
    if not keys or not _native_rows(dev, n) or not 1 <= nparts <= 255:
        return None
    kw = _key_words([[batch.columns[k] for k in keys]])
    if kw is None:
        return None
    (words,), _ = kw
    keep = K.hash_groups(words, mode=1, pout=nparts)
    if keep is None:
        return None
    idx, counts = K.bucket_compact(keep, nparts)
    b = batch.take(idx)
    bounds = [0] + torch.cumsum(counts, 0).cpu().tolist()
    return [b.slice(bounds[i], bounds[i + 1]) for i in range(nparts)]
