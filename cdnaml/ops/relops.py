"""Tensor-level entry points of the relational kernels (relational.hip, hash.hip,
hashagg.hip): column moments, partition destinations, mask compaction and gathers, dictionary / dense ids, the
partitioned hash aggregation, hash joins and grouped reductions.  Same contract as ``kernels``: device tensors go
to the gfx950 kernels, CPU tensors to a PyTorch reference of the same op."""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch

from . import _lib
from ._base import _native, _ptr, _stream, upload  # noqa: F401


# ------------------------------------------------------------ K20 / K16 (relational.hip)
def _merge_moments(part: torch.Tensor) -> torch.Tensor:
    """Chan merge of per-block moments [nb, d, 5] (count, mean, M2, min, max) -> [d, 5]."""
    cnt, mean, m2 = part[..., 0], part[..., 1], part[..., 2]
    N = cnt.sum(0)
    w = torch.where(N > 0, cnt / N.clamp_min(1), torch.zeros_like(cnt))
    mu = torch.where(cnt > 0, mean, torch.zeros_like(mean))
    M = (w * mu).sum(0)
    dev2 = torch.where(cnt > 0, cnt * (mu - M) ** 2, torch.zeros_like(mu))
    M2 = torch.where(cnt > 0, m2, torch.zeros_like(m2)).sum(0) + dev2.sum(0)
    has = cnt > 0
    inf = torch.full_like(mean, float("inf"))
    mn = torch.where(has, part[..., 3], inf).amin(0)
    mxs = torch.where(has, part[..., 4], -inf)
    mx = torch.where(torch.isnan(mxs).any(0), torch.full_like(M, float("nan")), mxs.amax(0))
    nanmean = torch.isnan(torch.where(has, mean, torch.zeros_like(mean))).any(0)
    M = torch.where(nanmean, torch.full_like(M, float("nan")), M)
    return torch.stack([N, M, M2, mn, mx], 1)


def col_moments(X: torch.Tensor, valid: Optional[torch.Tensor] = None) -> torch.Tensor:
    """K20: per-column (count, mean, M2, min, max) of X [n, d] in fp64, skipping entries with valid == 0.

    NaNs are values (mean NaN, max NaN, min ignores them) as in Spark's describe/summary."""
    n, d = X.shape
    if n == 0 or d == 0:
        out = torch.zeros((d, 5), dtype=torch.float64, device=X.device)
        out[:, 3], out[:, 4] = float("inf"), float("-inf")
        return out
    if _native(X):
        Xc = X if X.dtype in (torch.float32, torch.float64) else X.double()
        if Xc.stride(1) != 1:
            Xc = Xc.contiguous()
        v = None
        if valid is not None:
            v = valid.to(torch.uint8)
            v = v if v.stride(1) == 1 else v.contiguous()
        rpb = max(256, -(-n // 4096))
        nb = -(-n // rpb)
        part = torch.empty((nb, d, 5), dtype=torch.float64, device=X.device)
        _lib.check(_lib.lib().cdna_col_moments(0 if Xc.dtype == torch.float32 else 1, _ptr(Xc), n, d, Xc.stride(0),
                                               _ptr(v), 0 if v is None else v.stride(0), rpb, _ptr(part),
                                               _stream(X.device)), "cdna_col_moments")
        return _merge_moments(part)
    x = X.double()
    ok = torch.ones_like(x, dtype=torch.bool) if valid is None else valid.bool()
    cnt = ok.sum(0).double()
    xs = torch.where(ok, x, torch.zeros_like(x))
    mean = xs.sum(0) / cnt.clamp_min(1)
    m2 = torch.where(ok, (x - mean) ** 2, torch.zeros_like(x)).sum(0)
    mn = torch.where(ok & ~torch.isnan(x), x, torch.full_like(x, float("inf"))).amin(0)
    mx = torch.where(ok, x, torch.full_like(x, float("-inf")))
    mx = torch.where((torch.isnan(mx)).any(0), torch.full_like(mean, float("nan")), mx.nan_to_num(float("-inf")).amax(0))
    return torch.stack([cnt, mean, m2, mn, mx], 1)


def partition_dest(dest: torch.Tensor, W: int):
    """K16: stable counting sort of rows by destination bucket in [0, W).

    Returns (perm int64 [n] = stable argsort of dest, counts [W] int64)."""
    n = dest.numel()
    if n == 0:
        return torch.zeros(0, dtype=torch.int64, device=dest.device), torch.zeros(W, dtype=torch.int64,
                                                                                 device=dest.device)
    if _native(dest) and W <= 8192:
        d32 = dest.to(torch.int32).contiguous()
        rpb = max(1024, -(-n // 2048))
        nb = -(-n // rpb)
        counts = torch.empty((W, nb), dtype=torch.int32, device=dest.device)
        L = _lib.lib()
        _lib.check(L.cdna_partition_dest(1, _ptr(d32), n, W, rpb, _ptr(counts), None, None, _stream(dest.device)),
                   "cdna_partition_dest(count)")
        flat = counts.reshape(-1).long()
        offs = (torch.cumsum(flat, 0) - flat).contiguous()
        perm = torch.empty(n, dtype=torch.int64, device=dest.device)
        _lib.check(L.cdna_partition_dest(2, _ptr(d32), n, W, rpb, None, _ptr(offs), _ptr(perm),
                                         _stream(dest.device)), "cdna_partition_dest(scatter)")
        return perm, counts.long().sum(1)
    perm = torch.argsort(dest.long(), stable=True)
    return perm, torch.bincount(dest.long(), minlength=W)


def compact_mask(mask: torch.Tensor) -> torch.Tensor:
    """K19: int64 indices of the True entries of a 1-D mask, in order (== torch.nonzero(mask).flatten())."""
    n = mask.numel()
    if not _native(mask) or n == 0:
        return torch.nonzero(mask.reshape(-1), as_tuple=False).flatten()
    m8 = mask.reshape(-1).to(torch.uint8).contiguous()
    rpb = max(4096, -(-n // 4096))
    nb = -(-n // rpb)
    counts = torch.empty(nb, dtype=torch.int32, device=mask.device)
    L = _lib.lib()
    _lib.check(L.cdna_compact_mask(1, _ptr(m8), n, rpb, _ptr(counts), None, None, _stream(mask.device)),
               "cdna_compact_mask(count)")
    c64 = counts.long()
    csum = torch.cumsum(c64, 0)
    total = int(csum[-1].item())
    idx = torch.empty(total, dtype=torch.int64, device=mask.device)
    if total:
        offs = (csum - c64).contiguous()
        _lib.check(L.cdna_compact_mask(2, _ptr(m8), n, rpb, None, _ptr(offs), _ptr(idx), _stream(mask.device)),
                   "cdna_compact_mask(write)")
    return idx


GATHER_MIN = int(__import__("os").environ.get("CDNAML_GATHER_MIN", "65536"))


def gather_cols(tensors, idx: torch.Tensor):
    """K19 gather: [t[idx] for t in tensors] for 1-D contiguous device tensors of 1/2/4/8-byte elements, up to 8 per
    launch (relational.hip gather_kernel); entries that do not qualify come back as None."""
    import ctypes
    out = [None] * len(tensors)
    ok = [i for i, t in enumerate(tensors) if t is not None and t.is_cuda and t.dim() == 1 and t.is_contiguous()
          and t.element_size() in (1, 2, 4, 8)]
    m = idx.numel()
    ix = idx.to(torch.int64).contiguous()
    for c0 in range(0, len(ok), 8):
        grp = ok[c0:c0 + 8]
        src = [tensors[i] for i in grp]
        dst = [torch.empty(m, dtype=t.dtype, device=t.device) for t in src]
        eb = (ctypes.c_int * len(grp))(*[t.element_size() for t in src])
        _lib.check(_lib.lib().cdna_gather(_ptr(ix), m, min(int(t.shape[0]) for t in src), len(grp), _ptr_array(src),
                                          _ptr_array(dst), eb, _stream(ix.device)), "cdna_gather")
        for i, d in zip(grp, dst):
            out[i] = d
    return out


def bucket_compact(keep: torch.Tensor, nb: int):
    """Rows with keep = 1 + bucket (uint8, 0 = dropped) grouped by bucket, in row order within a bucket:
    (idx int64, counts per bucket int64 on the device)."""
    n = keep.numel()
    dev = keep.device
    L = _lib.lib()
    rpb = max(1024, -(-n // 16384) + 63) // 64 * 64      # rows per wave
    nw = -(-n // rpb)
    nblk = 4 * (-(-nw // 4))
    counts = torch.zeros((nb, nblk), dtype=torch.int32, device=dev)
    _lib.check(L.cdna_bucket_compact(1, _ptr(keep), n, nb, rpb, _ptr(counts), None, None, _stream(dev)),
               "cdna_bucket_compact(count)")
    flat = counts.view(-1).long()
    csum = torch.cumsum(flat, 0)
    total = int(csum[-1].item())
    idx = torch.empty(total, dtype=torch.int64, device=dev)
    if total:
        _lib.check(L.cdna_bucket_compact(2, _ptr(keep), n, nb, rpb, None, _ptr((csum - flat).contiguous()), _ptr(idx),
                                         _stream(dev)), "cdna_bucket_compact(scatter)")
    return idx, counts.long().sum(1)


# ------------------------------------------------------------------- K16 / K17
_EMPTY64 = -(1 << 63)


def _key_bits(x: torch.Tensor) -> torch.Tensor:
    """1-D values -> int64 bit patterns whose equality is value equality (-0.0 == 0.0, one NaN)."""
    if x.dtype.is_floating_point:
        x = torch.where(x == 0, torch.zeros_like(x), x)
        x = torch.where(torch.isnan(x), torch.full_like(x, float("nan")), x)
        if x.dtype == torch.float64:
            return x.contiguous().view(torch.int64)
        return x.float().contiguous().view(torch.int32).to(torch.int64) & 0xFFFFFFFF
    return x.to(torch.int64).contiguous()


def _bits_values(bits: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
    if dtype == torch.float64:
        return bits.view(torch.float64)
    if dtype.is_floating_point:
        return (bits & 0xFFFFFFFF).to(torch.int32).view(torch.float32)
    return bits


def hash_dense_ids(x: torch.Tensor):
    """K16: dense ids of the values of a 1-D device tensor, equal to ``torch.unique(x, return_inverse=True)``
    (ids are ranks of the sorted distinct values) but built with one hash-table pass instead of a sort of
    all n rows.  Returns (ids int64 [n], number of distinct values, sorted distinct values)."""
    n = x.numel()
    dev = x.device
    bits = _key_bits(x.reshape(-1))
    if n == 0:
        return torch.zeros(0, dtype=torch.int64, device=dev), 0, x.reshape(-1)[:0]
    L = _lib.lib()
    P = 1 << max(10, (2 * min(n, 1 << 20) - 1).bit_length())
    table = torch.full((P,), _EMPTY64, dtype=torch.int64, device=dev)
    slot = torch.empty(n, dtype=torch.int64, device=dev)
    ovf = torch.zeros(1, dtype=torch.int32, device=dev)
    _lib.check(L.cdna_hash_insert(_ptr(bits), n, _ptr(table), P - 1, _ptr(slot), 64, _ptr(ovf), _stream(dev)),
               "cdna_hash_insert")
    if int(ovf.item()):
        # more than ~2^20 distinct keys: a table of 2n random slots loses to the radix sort (measured on
        # dropDuplicates of 1e8 rows / 4.3e7 keys: 93 vs 78 ms), so the sort takes it from here
        vals, inv = torch.unique(_bits_values(bits, x.dtype), return_inverse=True)
        return inv, int(vals.numel()), vals.to(x.dtype)
    occ = torch.nonzero(table != _EMPTY64).flatten()
    keys = table[occ]
    special = bool((slot == P).any())
    if special:
        keys = torch.cat([keys, torch.full((1,), _EMPTY64, dtype=torch.int64, device=dev)])
    vals = _bits_values(keys, x.dtype)
    order = torch.argsort(vals, stable=True)
    G = keys.numel()
    rank = torch.empty(G, dtype=torch.int64, device=dev)
    rank[order] = torch.arange(G, device=dev)
    rank_of_slot = torch.empty(P + 1, dtype=torch.int64, device=dev)
    rank_of_slot[occ] = rank[:occ.numel()]
    if special:
        rank_of_slot[P] = rank[-1]
    return rank_of_slot[slot], G, vals[order].to(x.dtype)


HASH_MIN_ROWS = int(__import__("os").environ.get("CDNAML_HASH_MIN_ROWS", "16384"))


def dense_ids(x: torch.Tensor):
    """(ids, G): K16 hash ids on the GPU for large inputs, ``torch.unique`` otherwise (same result)."""
    if _native(x) and x.numel() >= HASH_MIN_ROWS and x.dim() == 1:
        ids, G, _ = hash_dense_ids(x)
        return ids, G
    uniq, inv = torch.unique(x, return_inverse=True)
    return inv, int(uniq.numel())


def dict_encode(arr, device):
    """K17: an Arrow string array -> (codes int32 [n] on ``device`` (-1 for nulls), valid bool tensor or None,
    sorted dictionary as a numpy object array).  Strings go to the device once (offsets + UTF-8 bytes); one
    hash-table pass finds every string's representative row (exact: equal tags are byte-compared); only the
    distinct strings come back to the host to be sorted."""
    import pyarrow as pa
    if isinstance(arr, pa.ChunkedArray):
        arr = arr.combine_chunks()
    if pa.types.is_large_string(arr.type):
        arr = arr.cast(pa.string())
    n = len(arr)
    dev = torch.device(device)
    valid_np = None if arr.null_count == 0 else np.asarray(arr.is_valid().to_numpy(zero_copy_only=False))
    bufs = arr.buffers()
    offs_np = np.frombuffer(bufs[1], dtype=np.int32, count=n + 1 + arr.offset)[arr.offset:]
    data_np = np.frombuffer(bufs[2], dtype=np.uint8) if bufs[2] is not None else np.zeros(1, np.uint8)
    offs = torch.from_numpy(offs_np.copy()).to(dev)
    data = torch.from_numpy(data_np.copy() if data_np.size else np.zeros(1, np.uint8)).to(dev)
    L = _lib.lib()
    P = 1 << max(10, (2 * n - 1).bit_length())
    table = torch.zeros(P, dtype=torch.int64, device=dev)
    rep = torch.empty(n, dtype=torch.int32, device=dev)
    ovf = torch.zeros(1, dtype=torch.int32, device=dev)
    vt = None if valid_np is None else torch.from_numpy(valid_np.astype(np.uint8)).to(dev)
    _lib.check(L.cdna_dict_encode(_ptr(offs), _ptr(data), _ptr(vt), n, _ptr(table), P - 1, _ptr(rep), 1 << 20,
                                  _ptr(ovf), _stream(dev)), "cdna_dict_encode")
    if int(ovf.item()):
        raise RuntimeError("dict_encode: hash table overflow")
    reps = torch.unique(rep[rep >= 0]) if n else rep[:0]
    reps_h = reps.cpu().numpy()
    strs = np.array([arr[int(i)].as_py() for i in reps_h], dtype=object) if len(reps_h) < 4096 else \
        np.asarray(arr.take(pa.array(reps_h)).to_numpy(zero_copy_only=False), dtype=object)
    order = np.argsort(strs, kind="stable")
    rank = np.empty(len(order), dtype=np.int32)
    rank[order] = np.arange(len(order), dtype=np.int32)
    lut = torch.full((max(n, 1),), -1, dtype=torch.int32, device=dev)
    if len(reps_h):
        lut[reps.long()] = torch.from_numpy(rank).to(dev)
    codes = torch.where(rep >= 0, lut[rep.clamp_min(0).long()], torch.full_like(rep, -1))
    valid = None if valid_np is None else torch.from_numpy(valid_np).to(dev)
    return codes, valid, strs[order]


# ----------------------------------------------------------- K16 partitioned hash operators (hashagg.hip)
HP_MAX_ACC = 4
HP_OPS = {"sum": 0, "min": 1, "max": 2, "count": 3, "last": 4}
_PACK_DT = {torch.uint8: 0, torch.bool: 0, torch.int16: 1, torch.int32: 2, torch.int64: 3, torch.int8: 4}
_VAL_DT = {torch.float64: 0, torch.float32: 1, torch.int64: 2, torch.int32: 3, torch.uint8: 4, torch.bool: 4,
           torch.int16: 5, torch.int8: 6}


def _ptr_array(ts):
    import ctypes
    arr = (ctypes.c_void_p * max(1, len(ts)))(*[_ptr(t) for t in ts])
    return arr


def pack_keys(cols, n: int, dev) -> torch.Tensor:
    """K16 key words: cols = [(values 1-D integer tensor, valid bool tensor or None, lo, radix)] -> int64 [n] with
    word = sum_j code_j * prod_{l > j} radix_l, code = value - lo + 1 (null 0): equality is tuple equality and the
    signed order is the lexicographic tuple order with nulls first.  The caller checks prod(radix) < 2^62."""
    import ctypes
    vals = [v.contiguous() if v.dtype != torch.bool else v.contiguous().view(torch.uint8) for v, _, _, _ in cols]
    valids = [None if m is None else m.contiguous().view(torch.uint8) for _, m, _, _ in cols]
    k = len(cols)
    lo = (ctypes.c_longlong * k)(*[int(c[2]) for c in cols])
    rdx = (ctypes.c_longlong * k)(*[int(c[3]) for c in cols])
    dts = (ctypes.c_int * k)(*[_PACK_DT[v.dtype] for v in vals])
    out = torch.empty(n, dtype=torch.int64, device=dev)
    _lib.check(_lib.lib().cdna_pack_keys(k, _ptr_array(vals), _ptr_array(valids), lo, rdx, dts, n, _ptr(out),
                                         _stream(torch.device(dev))), "cdna_pack_keys")
    return out


def _excl_scan_n(c: torch.Tensor, n: int) -> torch.Tensor:
    """Exclusive int64 prefix sums of c followed by the total n."""
    out = torch.empty(c.numel() + 1, dtype=torch.int64, device=c.device)
    torch.cumsum(c, 0, out=out[1:])
    out[0] = 0
    return out


def _hp_shape(n: int, na: int):
    L = _lib.lib()
    S = min(65535, L.cdna_hp_agg_lds_budget() // (16 + 8 * na) - 1)
    cap = S * 7 // 8
    # partitions: ~70 % of the table's capacity in rows per partition (so even all-distinct keys fit), <= 2^14
    pbits = 0
    while pbits < 14 and n > (cap * 7 // 10) << pbits:
        pbits += 1
    return S, cap, pbits


def hash_groups(key: torch.Tensor, values=(), accs=(), mode: int = 0, pout: int = 1):
    """K16 partitioned LDS hash aggregation / dedup over int64 key words [n] (hashagg.hip).

    values: [(tensor 1-D, valid or None)] scattered with the keys (<= 4); accs: [(op name, value index)] with op in
    sum / min / max / count (non-null count) / last (value index ignored).  mode 0: aggregate; 2: aggregate and
    also return every row's group; 1: dedup.

    mode 0 / 2 -> dict(G, pos (sparse positions of the groups, partition order), key, cnt, first, acc [na][n]
    sparse arrays, gpos (mode 2: every row's sparse group position)); mode 1 -> keep uint8 [n] (1 + output
    partition at the first row of every key, 0 elsewhere).  None when a partition overflowed its table."""
    n = key.numel()
    dev = key.device
    L = _lib.lib()
    st = _stream(dev)
    na = len(accs)
    assert na <= HP_MAX_ACC and len(values) <= HP_MAX_ACC and n < (1 << 31)
    if LOCAL_FIRST:
        r = _la_groups(key, values, accs, mode, pout)
        if r is not None:
            return r
    S, cap, pbits = _hp_shape(n, na)
    P = 1 << pbits
    rpb = max(4096, -(-n // 512))
    nblk = -(-n // rpb)
    key = key.contiguous()
    counts = torch.empty((P, nblk), dtype=torch.int32, device=dev)
    _lib.check(L.cdna_hp_hist(_ptr(key), n, pbits, rpb, _ptr(counts), st), "cdna_hp_hist")
    offs = _excl_scan_n(counts.view(-1), n)
    nv = len(values)
    vals = [v.contiguous() if v.dtype != torch.bool else v.contiguous().view(torch.uint8) for v, _ in values]
    vvalid = [None if m is None else m.contiguous().view(torch.uint8) for _, m in values]
    import ctypes
    vdt = (ctypes.c_int * max(1, nv))(*[_VAL_DT[v.dtype] for v in vals])

    def bufs():
        return (torch.empty(n, dtype=torch.int64, device=dev), torch.empty(n, dtype=torch.int32, device=dev),
                torch.empty((nv, n), dtype=torch.int64, device=dev) if nv else None)
    kout, rout, vout = bufs()
    if pbits <= 7:
        _lib.check(L.cdna_hp_part(0, n, P, 64 - pbits, rpb, nblk, 1, 1, 1, _ptr(offs), None, _ptr(key), nv,
                                  _ptr_array(vals), _ptr_array(vvalid), vdt, None, None, None, _ptr(kout), _ptr(rout),
                                  _ptr(vout), st), "cdna_hp_part")
    else:
        hi = pbits - 7
        offs_a = _excl_scan_n(counts.view(1 << hi, 128, nblk).sum(1, dtype=torch.int64).view(-1), n)
        k1, r1, v1 = bufs()
        _lib.check(L.cdna_hp_part(0, n, 1 << hi, 64 - hi, rpb, nblk, 1, 1, 1, _ptr(offs_a), None, _ptr(key), nv,
                                  _ptr_array(vals), _ptr_array(vvalid), vdt, None, None, None, _ptr(k1), _ptr(r1),
                                  _ptr(v1), st), "cdna_hp_part(0)")
        gs = 16
        _lib.check(L.cdna_hp_part(1, n, 128, 64 - pbits, rpb, nblk, gs, -(-nblk // gs), 1 << hi, _ptr(offs),
                                  _ptr(offs_a), None, nv, None, None, None, _ptr(k1), _ptr(r1), _ptr(v1), _ptr(kout),
                                  _ptr(rout), _ptr(vout), st), "cdna_hp_part(1)")
        del k1, r1, v1
    ops = (ctypes.c_int * max(1, na))(*[HP_OPS[o] for o, _ in accs])
    vcols = (ctypes.c_int * max(1, na))(*[int(j) for _, j in accs])
    ngroups = torch.empty(P, dtype=torch.int32, device=dev)
    if mode == 1:
        keep = torch.zeros(n, dtype=torch.uint8, device=dev)
        _lib.check(L.cdna_hp_agg(_ptr(kout), _ptr(rout), _ptr(vout), n, _ptr(offs), pbits, nblk, S, cap, 0, ops, vcols,
                                 1, int(pout), None, None, None, None, _ptr(ngroups), _ptr(keep), None, st),
                   "cdna_hp_agg(dedup)")
        if bool((ngroups < 0).any()):
            return None
        return keep
    gkey = torch.empty(n, dtype=torch.int64, device=dev)
    gcnt = torch.empty(n, dtype=torch.int32, device=dev)
    gfirst = torch.empty(n, dtype=torch.int32, device=dev)
    gacc = torch.empty((max(na, 1), n), dtype=torch.int64, device=dev)
    gpos = torch.empty(n, dtype=torch.int32, device=dev) if mode == 2 else None
    _lib.check(L.cdna_hp_agg(_ptr(kout), _ptr(rout), _ptr(vout), n, _ptr(offs), pbits, nblk, S, cap, na, ops, vcols,
                             int(mode), 1, _ptr(gkey), _ptr(gcnt), _ptr(gfirst), _ptr(gacc), _ptr(ngroups), None,
                             _ptr(gpos), st), "cdna_hp_agg")
    ng = ngroups.long()
    csum = torch.cumsum(ng, 0)
    ovf, G = torch.stack([(ng < 0).any().long(), csum[-1]]).cpu().tolist()
    if ovf:
        return None
    starts = offs[:-1].view(P, nblk)[:, 0]
    pos = torch.repeat_interleave(starts - (csum - ng), ng, output_size=G) + torch.arange(G, device=dev)
    return {"G": G, "pos": pos, "key": gkey, "cnt": gcnt, "first": gfirst, "acc": gacc, "gpos": gpos}


# try the low-cardinality path (per-block LDS tables over row chunks + one merge) before partitioning
LOCAL_FIRST = True


def _la_groups(key: torch.Tensor, values, accs, mode: int, pout: int):
    """hashagg.hip la_agg + la_merge: the same results as the partitioned path (dense group arrays, pos =
    0..G-1) when every row chunk and the merged table hold at most one table of distinct keys; else None."""
    import ctypes
    n = key.numel()
    dev = key.device
    L = _lib.lib()
    na, nv = len(accs), len(values)
    S, cap, _ = _hp_shape(n, na)
    nblk = max(1, min(1024, n // 16384))
    rpb = -(-n // nblk)
    nblk = -(-n // rpb)
    pcap = nblk * (cap + 2)
    pkey = torch.empty(pcap, dtype=torch.int64, device=dev)
    pcnt = torch.empty(pcap, dtype=torch.int32, device=dev)
    pfirst = torch.empty(pcap, dtype=torch.int32, device=dev)
    pacc = torch.empty((max(na, 1), pcap), dtype=torch.int64, device=dev)
    ctr = torch.zeros(2, dtype=torch.int32, device=dev)
    gkey = torch.empty(S + 1, dtype=torch.int64, device=dev)
    gcnt = torch.empty(S + 1, dtype=torch.int32, device=dev)
    gfirst = torch.empty(S + 1, dtype=torch.int32, device=dev)
    gacc = torch.empty((max(na, 1), S + 1), dtype=torch.int64, device=dev)
    ng = torch.empty(1, dtype=torch.int32, device=dev)
    keep = torch.zeros(n, dtype=torch.uint8, device=dev) if mode == 1 else None
    vals = [v.contiguous() if v.dtype != torch.bool else v.contiguous().view(torch.uint8) for v, _ in values]
    vvalid = [None if m is None else m.contiguous().view(torch.uint8) for _, m in values]
    vdt = (ctypes.c_int * max(1, nv))(*[_VAL_DT[v.dtype] for v in vals])
    ops = (ctypes.c_int * max(1, na))(*[HP_OPS[o] for o, _ in accs])
    vcols = (ctypes.c_int * max(1, na))(*[int(j) for _, j in accs])
    _lib.check(L.cdna_la_groups(_ptr(key.contiguous()), n, rpb, S, cap, na, ops, vcols, nv, _ptr_array(vals),
                                _ptr_array(vvalid), vdt, 1 if mode == 1 else 0, int(pout), _ptr(pkey), _ptr(pcnt),
                                _ptr(pfirst), _ptr(pacc), pcap, _ptr(ctr[0:1]), _ptr(ctr[1:2]), _ptr(gkey),
                                _ptr(gcnt), _ptr(gfirst), _ptr(gacc), _ptr(ng), _ptr(keep), _stream(dev)),
               "cdna_la_groups")
    G = int(ng.item())
    if G < 0:
        return None
    if mode == 1:
        return keep
    gpos = None
    if mode == 2:
        ri, _, _ = join_probe(key, None, join_table(gkey[:G], None))
        gpos = ri.to(torch.int32)
    return {"G": G, "pos": torch.arange(G, device=dev), "key": gkey, "cnt": gcnt, "first": gfirst, "acc": gacc,
            "gpos": gpos}


def ordered_to_double(u: torch.Tensor) -> torch.Tensor:
    """Inverse of hashagg.hip's ord_of (order-preserving u64 image of an fp64)."""
    neg = u >= 0                      # top bit clear (as int64: non-negative) <- a negative double
    bits = torch.where(neg, ~u, u & 0x7FFFFFFFFFFFFFFF)
    return bits.view(torch.float64)


class JoinTable:
    """K16 join build side.  kind 'dense': direct-addressed arrays over the key range [lo, lo + R) plus a presence
    bitmap; kind 'hash': open-addressing table of 2x the rows.  brow / bcnt: first build row and build rows per
    slot; nslots: slot count (slot ids of probes are < nslots); ovf: device overflow flag (hash only)."""

    def __init__(self, **kw):
        self.__dict__.update(kw)


DENSE_JOIN_MAX = 1 << 26


def join_table(keys: torch.Tensor, valid: Optional[torch.Tensor]) -> JoinTable:
    """Build side of a K16 join over int64 key words (hashagg.hip join_build / join_build_dense)."""
    n = keys.numel()
    dev = keys.device
    L = _lib.lib()
    v8 = None if valid is None else valid.contiguous().view(torch.uint8)
    keys = keys.contiguous()
    if n:
        kv = keys if valid is None else keys[valid]
        if kv.numel():
            lo, hi = (int(x) for x in torch.stack(list(torch.aminmax(kv))).cpu().tolist())
            R = hi - lo + 1
            if R <= max(1 << 22, 8 * n) and R <= DENSE_JOIN_MAX:
                brow = torch.full((R,), (1 << 63) - 1, dtype=torch.int64, device=dev)
                bcnt = torch.zeros(R, dtype=torch.int32, device=dev)
                bits = torch.zeros((R + 31) // 32, dtype=torch.int32, device=dev)
                _lib.check(L.cdna_join_build_dense(_ptr(keys), _ptr(v8), n, lo, R, _ptr(brow), _ptr(bcnt), _ptr(bits),
                                                   _stream(dev)), "cdna_join_build_dense")
                return JoinTable(kind="dense", lo=lo, R=R, brow=brow, bcnt=bcnt, bits=bits, nslots=R,
                                 ovf=torch.zeros(1, dtype=torch.int32, device=dev))
    P = 1 << max(10, (2 * max(n, 1) - 1).bit_length())
    table = torch.full((P + 1,), _EMPTY64, dtype=torch.int64, device=dev)
    brow = torch.full((P + 1,), (1 << 63) - 1, dtype=torch.int64, device=dev)
    bcnt = torch.zeros(P + 1, dtype=torch.int32, device=dev)
    ovf = torch.zeros(1, dtype=torch.int32, device=dev)
    _lib.check(L.cdna_join_build(_ptr(keys), _ptr(v8), n, _ptr(table), P - 1, _ptr(brow), _ptr(bcnt), _ptr(ovf),
                                 _stream(dev)), "cdna_join_build")
    return JoinTable(kind="hash", table=table, mask=P - 1, brow=brow, bcnt=bcnt, nslots=P + 1, ovf=ovf)


def join_probe(keys: torch.Tensor, valid: Optional[torch.Tensor], tab: JoinTable, want_cnt: bool = False,
               want_slot: bool = False):
    """K16 join probe: per probe row the first matching build row (-1: none), optionally the number of build rows
    with its key and its table slot."""
    n = keys.numel()
    dev = keys.device
    ri = torch.empty(n, dtype=torch.int64, device=dev)
    cnt = torch.empty(n, dtype=torch.int32, device=dev) if want_cnt else None
    slot = torch.empty(n, dtype=torch.int64, device=dev) if want_slot else None
    v8 = None if valid is None else valid.contiguous().view(torch.uint8)
    L = _lib.lib()
    if tab.kind == "dense":
        _lib.check(L.cdna_join_probe_dense(_ptr(keys.contiguous()), _ptr(v8), n, tab.lo, tab.R, _ptr(tab.brow),
                                           _ptr(tab.bcnt), _ptr(tab.bits), _ptr(ri), _ptr(cnt), _ptr(slot),
                                           _stream(dev)), "cdna_join_probe_dense")
    else:
        _lib.check(L.cdna_join_probe(_ptr(keys.contiguous()), _ptr(v8), n, _ptr(tab.table), tab.mask, _ptr(tab.brow),
                                     _ptr(tab.bcnt), _ptr(ri), _ptr(cnt), _ptr(slot), _stream(dev)),
                   "cdna_join_probe")
    return ri, cnt, slot


GROUPED_MAX = 8192  # groups an LDS-privatised reduction holds (64 KB of fp64)


def _grouped(op: int, vals: Optional[torch.Tensor], gid: torch.Tensor, G: int) -> Optional[torch.Tensor]:
    n = gid.numel()
    if not (_native(gid) and 0 < G <= GROUPED_MAX and n >= HASH_MIN_ROWS):
        return None
    dev = gid.device
    rpb = max(4096, -(-n // 2048))
    nblk = -(-n // rpb)
    part = torch.empty((nblk, G), dtype=torch.float64 if op == 0 else torch.int64, device=dev)
    g = gid.to(torch.int64).contiguous()
    v = None if vals is None else vals.to(torch.float64).contiguous()
    _lib.check(_lib.lib().cdna_grouped_reduce(op, _ptr(v), _ptr(g), n, G, rpb, _ptr(part), _stream(dev)),
               "cdna_grouped_reduce")
    return part.sum(0) if op == 0 else part.min(0).values


def group_sum(vals: Optional[torch.Tensor], gid: torch.Tensor, G: int) -> torch.Tensor:
    """fp64 per-group sums (vals None: row counts); LDS-privatised kernel for few groups, index_add otherwise."""
    r = _grouped(0, vals, gid, G)
    if r is not None:
        return r
    s = torch.zeros(G, dtype=torch.float64, device=gid.device)
    s.index_add_(0, gid, torch.ones(gid.numel(), dtype=torch.float64, device=gid.device) if vals is None
                 else vals.to(torch.float64))
    return s


def group_first(gid: torch.Tensor, G: int) -> torch.Tensor:
    """First row index of every group (n for empty groups)."""
    r = _grouped(1, None, gid, G)
    if r is not None:
        return r
    n = gid.numel()
    first = torch.full((G,), n, dtype=torch.int64, device=gid.device)
    first.scatter_reduce_(0, gid, torch.arange(n, device=gid.device), reduce="amin", include_self=True)
    return first


from . import tune as _tune  # noqa: E402  (CDNAML_TUNE overrides of the constants above)
_tune.apply(__import__(__name__, fromlist=["_"]))
