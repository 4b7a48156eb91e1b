"""``pyspark.sql.functions``-compatible column functions.

Elementwise functions run as device tensor ops on the partition; string
functions act on the (small) host dictionary and re-encode codes; random
columns use the counter-based Philox kernel keyed by (seed, partition, row).
"""
from __future__ import annotations

import datetime as _dt
import math
from typing import Any

import numpy as np
import torch

from ..ops import kernels as K
from . import types as T
from .batch import ColumnData, column_from_numpy, full_column, map_dictionary, unify_dictionaries
from .column import (AnalysisException, BinOp, CaseWhen, Cast, ColRef, Column, Expr, Func, IsIn, IsNaN, IsNull, Lit,
                     RowFunc, SortOrder, Star, Unary, _cast, _to_expr)


# --------------------------------------------------------------- basics
def col(name: str) -> Column:
    if name == "*":
        return Column(Star())
    return Column(ColRef(name))


column = col


def lit(value) -> Column:
    if isinstance(value, Column):
        return value
    return Column(Lit(value))


def _c(x) -> Column:
    return x if isinstance(x, Column) else col(x)


def _ce(x) -> Expr:
    return _c(x)._expr


def expr(s: str) -> Column:
    from .parser import parse_expression
    return parse_expression(s)


def when(cond, value) -> Column:
    return Column(CaseWhen([(_to_expr(cond), _to_expr(value))]))


def asc(c):
    return _c(c).asc()


def desc(c):
    return _c(c).desc()


def isnull(c):
    return Column(IsNull(_ce(c)))


def isnan(c):
    return Column(IsNaN(_ce(c)))


def broadcast(df):
    return df


# ------------------------------------------------------------ math
def _math(fname, fn, out_t=None):
    def f(c, *extra):
        def ev(b, ctx, args):
            a = args[0]
            if isinstance(a.dtype, T.StringType):
                a = _cast(a, T.DoubleType())
            v = a.values.to(torch.float64)
            r = fn(v, *extra)
            valid = a.valid
            if fname in ("log", "log10", "log2", "ln", "log1p", "sqrt"):
                bad = ~torch.isfinite(r) & torch.isfinite(v) if fname != "log1p" else v <= -1
                if fname in ("log", "log10", "log2", "ln"):
                    bad = v <= 0
                if fname == "sqrt":
                    bad = v < 0
                if bool(bad.any()):
                    valid = ~bad if valid is None else valid & ~bad
            return ColumnData(r if out_t is None else r.to(out_t.torch_dtype), out_t or T.DoubleType(), valid)
        fn_ = Func(fname, ev, [_ce(c)])
        fn_.fuse = fname if (out_t is None and not extra) else None  # K18 opcode tag (sql/fused.py)
        return Column(fn_)
    return f


log10 = _math("log10", torch.log10)
log2 = _math("log2", torch.log2)
log1p = _math("log1p", torch.log1p)
exp = _math("exp", torch.exp)
expm1 = _math("expm1", torch.expm1)
sqrt = _math("sqrt", torch.sqrt)
cbrt = _math("cbrt", lambda v: torch.sign(v) * torch.abs(v) ** (1.0 / 3))
sin = _math("sin", torch.sin)
cos = _math("cos", torch.cos)
tan = _math("tan", torch.tan)
signum = _math("signum", torch.sign)


def log(arg1, arg2=None) -> Column:
    if arg2 is None:
        return _math("ln", torch.log)(arg1)._rename("ln")
    base = float(arg1)
    return Column(Func("log", lambda b, ctx, a: _math_ev(a[0], lambda v: torch.log(v) / math.log(base)), [_ce(arg2)]))


def _math_ev(a, fn):
    v = a.values.to(torch.float64)
    bad = v <= 0
    valid = a.valid
    if bool(bad.any()):
        valid = ~bad if valid is None else valid & ~bad
    return ColumnData(fn(v), T.DoubleType(), valid)


def _rename(self, n):
    e = self._expr
    if isinstance(e, Func):
        e.fname = n
        if getattr(e, "fuse", None) is not None:
            e.fuse = n
    return self


Column._rename = _rename


def abs(c) -> Column:  # noqa: A001
    def ev(b, ctx, args):
        a = args[0]
        return ColumnData(torch.abs(a.values), a.dtype, a.valid)
    f = Func("abs", ev, [_ce(c)])
    f.fuse = "abs"
    return Column(f)


def pow(a, b) -> Column:  # noqa: A001
    return Column(BinOp("**", _to_expr(a if not isinstance(a, str) else col(a)),
                        _to_expr(b if not isinstance(b, str) else col(b))))


def round(c, scale: int = 0) -> Column:  # noqa: A001
    def ev(b, ctx, args):
        a = args[0]
        if isinstance(a.dtype, T.IntegralType) and scale >= 0:
            return a
        v = a.values.to(torch.float64)
        m = 10.0 ** scale
        r = torch.sign(v) * torch.floor(torch.abs(v) * m + 0.5) / m  # HALF_UP like Spark
        return ColumnData(r, T.DoubleType() if not isinstance(a.dtype, T.FloatType) else T.FloatType(), a.valid)
    f = Func("round", ev, [_ce(c)], display=f"round({_ce(c).name()}, {scale})")
    f.fuse = ("round", int(scale))
    return Column(f)


def bround(c, scale: int = 0) -> Column:
    def ev(b, ctx, args):
        a = args[0]
        v = a.values.to(torch.float64)
        return ColumnData(torch.round(v * 10.0 ** scale) / 10.0 ** scale, T.DoubleType(), a.valid)
    return Column(Func("bround", ev, [_ce(c)]))


def floor(c) -> Column:
    def ev(b, ctx, args):
        a = args[0]
        return ColumnData(torch.floor(a.values.to(torch.float64)).to(torch.int64), T.LongType(), a.valid)
    f = Func("FLOOR", ev, [_ce(c)])
    f.fuse = "floor"
    return Column(f)


def ceil(c) -> Column:
    def ev(b, ctx, args):
        a = args[0]
        return ColumnData(torch.ceil(a.values.to(torch.float64)).to(torch.int64), T.LongType(), a.valid)
    f = Func("CEIL", ev, [_ce(c)])
    f.fuse = "ceil"
    return Column(f)


def greatest(*cols) -> Column:
    def ev(b, ctx, args):
        v = torch.stack([a.values.to(torch.float64) for a in args]).max(0).values
        return ColumnData(v, T.DoubleType())
    return Column(Func("greatest", ev, [_ce(c) for c in cols]))


def least(*cols) -> Column:
    def ev(b, ctx, args):
        v = torch.stack([a.values.to(torch.float64) for a in args]).min(0).values
        return ColumnData(v, T.DoubleType())
    return Column(Func("least", ev, [_ce(c) for c in cols]))


def coalesce(*cols) -> Column:
    def ev(b, ctx, args):
        if any(isinstance(a.dtype, T.StringType) for a in args):
            args = unify_dictionaries([a if isinstance(a.dtype, T.StringType) else _cast(a, T.StringType())
                                       for a in args])
        out = args[-1].values.clone()
        valid = args[-1].valid_mask().clone()
        for a in reversed(args[:-1]):
            m = a.valid_mask()
            out = torch.where(m if out.dim() == 1 else m[:, None], a.values.to(out.dtype), out)
            valid = valid | m
        return ColumnData(out, args[0].dtype, None if bool(valid.all()) else valid, args[0].dictionary)
    return Column(Func("coalesce", ev, [_to_expr(c if not isinstance(c, str) else col(c)) for c in cols]))


def nanvl(c1, c2) -> Column:
    def ev(b, ctx, args):
        a, o = args
        v = a.values.to(torch.float64)
        return ColumnData(torch.where(torch.isnan(v), o.values.to(torch.float64), v), T.DoubleType(), a.valid)
    return Column(Func("nanvl", ev, [_ce(c1), _ce(c2)]))


# ------------------------------------------------------------ strings
def _strfn(fname, pyfn, c, display=None):
    def ev(b, ctx, args):
        a = args[0]
        if not isinstance(a.dtype, T.StringType):
            a = _cast(a, T.StringType())
        return map_dictionary(a, pyfn)
    return Column(Func(fname, ev, [_ce(c)], display=display))


def lower(c):
    return _strfn("lower", lambda s: s.lower(), c)


def upper(c):
    return _strfn("upper", lambda s: s.upper(), c)


def trim(c):
    return _strfn("trim", lambda s: s.strip(), c)


def ltrim(c):
    return _strfn("ltrim", lambda s: s.lstrip(), c)


def rtrim(c):
    return _strfn("rtrim", lambda s: s.rstrip(), c)


def initcap(c):
    return _strfn("initcap", lambda s: s.title(), c)


def reverse(c):
    return _strfn("reverse", lambda s: s[::-1], c)


def translate(c, matching: str, replace: str):
    table = {}
    for i, ch in enumerate(matching):
        if ord(ch) not in table:
            table[ord(ch)] = replace[i] if i < len(replace) else None
    return _strfn("translate", lambda s: s.translate(table), c,
                  display=f"translate({_ce(c).name()}, {matching}, {replace})")


def regexp_replace(c, pattern: str, replacement: str):
    import re
    rx = re.compile(pattern)
    repl = re.sub(r"\$(\d+)", r"\\\1", replacement)
    return _strfn("regexp_replace", lambda s: rx.sub(repl, s), c)


def regexp_extract(c, pattern: str, idx: int):
    import re
    rx = re.compile(pattern)

    def f(s):
        m = rx.search(s)
        return (m.group(idx) or "") if m else ""
    return _strfn("regexp_extract", f, c)


def substring(c, pos: int, length: int):
    def f(s):
        start = pos - 1 if pos > 0 else (len(s) + pos if pos < 0 else 0)
        return s[max(start, 0): max(start, 0) + length]
    return _strfn("substring", f, c, display=f"substring({_ce(c).name()}, {pos}, {length})")


def lpad(c, n, pad):
    return _strfn("lpad", lambda s: (pad * n + s)[-n:] if len(s) < n else s[:n], c)


def rpad(c, n, pad):
    return _strfn("rpad", lambda s: (s + pad * n)[:n], c)


def length(c):
    def ev(b, ctx, args):
        a = args[0]
        if not isinstance(a.dtype, T.StringType):
            a = _cast(a, T.StringType())
        d = a.dictionary if a.dictionary is not None else np.array([], dtype=object)
        lut = torch.tensor([len(s) for s in d.tolist()] + [0], dtype=torch.int32, device=a.device)
        codes = a.values.long()
        codes = torch.where(codes < 0, torch.full_like(codes, len(d)), codes)
        return ColumnData(lut[codes], T.IntegerType(), a.valid)
    return Column(Func("length", ev, [_ce(c)]))


def concat(*cols):
    def ev(b, ctx, args):
        strs = [(a if isinstance(a.dtype, T.StringType) else _cast(a, T.StringType())).to_numpy() for a in args]
        out = np.array([None if any(s[i] is None for s in strs) else "".join(s[i] for s in strs)
                        for i in range(b.n)], dtype=object)
        return column_from_numpy(out, T.StringType(), b.device)
    return Column(Func("concat", ev, [_ce(c) if isinstance(c, (str, Column)) else _to_expr(c) for c in cols]))


def concat_ws(sep, *cols):
    def ev(b, ctx, args):
        strs = [(a if isinstance(a.dtype, T.StringType) else _cast(a, T.StringType())).to_numpy() for a in args]
        out = np.array([sep.join(s[i] for s in strs if s[i] is not None) for i in range(b.n)], dtype=object)
        return column_from_numpy(out, T.StringType(), b.device)
    return Column(Func("concat_ws", ev, [_ce(c) for c in cols]))


def format_number(c, d: int):
    def ev(b, ctx, args):
        vals = args[0].to_numpy()
        out = np.array([None if v is None else f"{float(v):,.{d}f}" for v in vals], dtype=object)
        return column_from_numpy(out, T.StringType(), b.device)
    return Column(Func("format_number", ev, [_ce(c)]))


def split(c, pattern):
    import re

    def ev(b, ctx, args):
        vals = args[0].to_numpy()
        out = np.array([None if v is None else re.split(pattern, v) for v in vals], dtype=object)
        return ColumnData(torch.zeros(b.n, device=b.device), T.ArrayType(T.StringType()), meta={"_py": out})
    return Column(Func("split", ev, [_ce(c)]))


# -------------------------------------------------------------- dates
def _date_part(fname, fn):
    def f(c):
        def ev(b, ctx, args):
            a = args[0]
            if isinstance(a.dtype, T.StringType):
                a = _cast(a, T.DateType())
            days = a.values.cpu().numpy().astype(np.int64)
            if isinstance(a.dtype, T.TimestampType):
                days = days // 86_400_000_000
            dates = np.datetime64("1970-01-01") + days.astype("timedelta64[D]")
            r = fn(dates)
            return ColumnData(torch.from_numpy(np.asarray(r, np.int32)).to(b.device), T.IntegerType(), a.valid)
        return Column(Func(fname, ev, [_ce(c)]))
    return f


year = _date_part("year", lambda d: d.astype("datetime64[Y]").astype(int) + 1970)
month = _date_part("month", lambda d: d.astype("datetime64[M]").astype(int) % 12 + 1)
dayofmonth = _date_part("dayofmonth", lambda d: (d - d.astype("datetime64[M]")).astype(int) + 1)
dayofweek = _date_part("dayofweek", lambda d: ((d.astype(int) + 4) % 7) + 1)


def to_date(c, fmt=None):
    def ev(b, ctx, args):
        a = args[0]
        if isinstance(a.dtype, T.TimestampType):
            return ColumnData((a.values // 86_400_000_000).to(torch.int32), T.DateType(), a.valid)
        if isinstance(a.dtype, T.DateType):
            return a
        import pandas as pd
        vals = a.to_numpy()
        out = pd.to_datetime(pd.Series(vals), format=_py_fmt(fmt) if fmt else None, errors="coerce")
        return column_from_numpy(np.array([None if pd.isna(x) else x.date() for x in out], dtype=object),
                                 T.DateType(), b.device)
    return Column(Func("to_date", ev, [_ce(c)]))


def to_timestamp(c, fmt=None):
    def ev(b, ctx, args):
        import pandas as pd
        vals = args[0].to_numpy()
        out = pd.to_datetime(pd.Series(vals), format=_py_fmt(fmt) if fmt else None, errors="coerce")
        return column_from_numpy(out.to_numpy(), T.TimestampType(), b.device)
    return Column(Func("to_timestamp", ev, [_ce(c)]))


def _py_fmt(fmt):
    return (fmt.replace("yyyy", "%Y").replace("MM", "%m").replace("dd", "%d").replace("HH", "%H")
            .replace("mm", "%M").replace("ss", "%S"))


def current_date():
    return lit(_dt.date.today())


def current_timestamp():
    return lit(_dt.datetime.now())


def datediff(end, start):
    def ev(b, ctx, args):
        e, s = [_cast(a, T.DateType()) if isinstance(a.dtype, T.StringType) else a for a in args]
        return ColumnData((e.values.long() - s.values.long()).to(torch.int32), T.IntegerType(), None)
    return Column(Func("datediff", ev, [_ce(end), _ce(start)]))


def date_add(c, days: int):
    def ev(b, ctx, args):
        a = _cast(args[0], T.DateType()) if isinstance(args[0].dtype, T.StringType) else args[0]
        return ColumnData(a.values + int(days), T.DateType(), a.valid)
    return Column(Func("date_add", ev, [_ce(c)]))


# ------------------------------------------------------- row functions
def rand(seed: int = None) -> Column:
    """Uniform [0,1) doubles: Philox keyed by (seed, partition, row)."""
    if seed is None:
        seed = int(np.random.SeedSequence().entropy % (2 ** 63))

    def ev(b, ctx):
        off = (int(ctx.partition_index) << 40) + int(ctx.row_offset)
        u = K.uniform(b.n, seed, off, 0, device=b.device)
        return ColumnData(u, T.DoubleType())
    return Column(RowFunc("rand", ev, display=f"rand({seed})"))


def randn(seed: int = None) -> Column:
    if seed is None:
        seed = int(np.random.SeedSequence().entropy % (2 ** 63))

    def ev(b, ctx):
        off = (int(ctx.partition_index) << 40) + int(ctx.row_offset)
        u1 = K.uniform(b.n, seed, off, 1, device=b.device).clamp_min(1e-300)
        u2 = K.uniform(b.n, seed, off, 2, device=b.device)
        z = torch.sqrt(-2 * torch.log(u1)) * torch.cos(2 * math.pi * u2)
        return ColumnData(z, T.DoubleType())
    return Column(RowFunc("randn", ev, display=f"randn({seed})"))


def monotonically_increasing_id() -> Column:
    def ev(b, ctx):
        base = int(ctx.partition_index) << 33
        return ColumnData(torch.arange(b.n, dtype=torch.int64, device=b.device) + base + int(ctx.row_offset),
                          T.LongType())
    return Column(RowFunc("monotonically_increasing_id", ev))


def spark_partition_id() -> Column:
    def ev(b, ctx):
        return ColumnData(torch.full((b.n,), int(ctx.partition_index), dtype=torch.int32, device=b.device),
                          T.IntegerType())
    return Column(RowFunc("SPARK_PARTITION_ID", ev))


def _hash_column(c: ColumnData) -> torch.Tensor:
    """Deterministic 32-bit hash per row (murmur-style finaliser on device)."""
    if isinstance(c.dtype, T.StringType):
        import xxhash
        d = c.dictionary if c.dictionary is not None else np.array([], dtype=object)
        hs = [xxhash.xxh32_intdigest(s.encode("utf-8"), seed=42) for s in d.tolist()] + [42]
        lut = torch.tensor(hs, dtype=torch.int64, device=c.device)
        codes = c.values.long()
        codes = torch.where(codes < 0, torch.full_like(codes, len(d)), codes)
        h = lut[codes]
    else:
        v = c.values
        if v.dim() == 2:
            h = torch.zeros(v.shape[0], dtype=torch.int64, device=v.device)
            for j in range(v.shape[1]):
                h = _mix(h * 31 + _bits(v[:, j]))
            return h & 0xFFFFFFFF
        h = _bits(v)
    h = _mix(h)
    if c.valid is not None:
        h = torch.where(c.valid, h, torch.full_like(h, 42))
    return h & 0xFFFFFFFF


def _bits(v: torch.Tensor) -> torch.Tensor:
    if v.dtype == torch.float64:
        return v.view(torch.int64)
    if v.dtype == torch.float32:
        return v.view(torch.int32).to(torch.int64)
    return v.to(torch.int64)


def _mix(h: torch.Tensor) -> torch.Tensor:
    h = h & 0xFFFFFFFFFFFF
    h = (h ^ (h >> 16)) * 0x85EB & 0xFFFFFFFFFFFF
    h = (h ^ (h >> 13)) * 0xC2B2 & 0xFFFFFFFFFFFF
    return h ^ (h >> 16)


# ---- Spark-compatible Murmur3_x86_32 (seed 42, column hashes chained) ----
_M32 = 0xFFFFFFFF


def _rotl(x: torch.Tensor, r: int) -> torch.Tensor:
    return ((x << r) | (x >> (32 - r))) & _M32


def _mix_k1(k: torch.Tensor) -> torch.Tensor:
    k = (k * 0xCC9E2D51) & _M32
    k = _rotl(k, 15)
    return (k * 0x1B873593) & _M32


def _mix_h1(h: torch.Tensor, k: torch.Tensor) -> torch.Tensor:
    h = (h ^ k) & _M32
    h = _rotl(h, 13)
    return (h * 5 + 0xE6546B64) & _M32


def _fmix(h: torch.Tensor, length: int) -> torch.Tensor:
    h = h ^ length
    h = h ^ (h >> 16)
    h = (h * 0x85EBCA6B) & _M32
    h = h ^ (h >> 13)
    h = (h * 0xC2B2AE35) & _M32
    return h ^ (h >> 16)


def _murmur_int(v: torch.Tensor, seed: torch.Tensor) -> torch.Tensor:
    return _fmix(_mix_h1(seed, _mix_k1(v & _M32)), 4)


def _murmur_long(v: torch.Tensor, seed: torch.Tensor) -> torch.Tensor:
    lo = v & _M32
    hi = (v >> 32) & _M32
    h = _mix_h1(seed, _mix_k1(lo))
    h = _mix_h1(h, _mix_k1(hi))
    return _fmix(h, 8)


def _murmur_bytes_py(b: bytes, seed: int) -> int:
    """Spark's Murmur3_x86_32.hashUnsafeBytes (trailing bytes mixed one by one, signed)."""
    def mk(k):
        k = (k * 0xCC9E2D51) & _M32
        k = ((k << 15) | (k >> 17)) & _M32
        return (k * 0x1B873593) & _M32

    def mh(h, k):
        h ^= k
        h = ((h << 13) | (h >> 19)) & _M32
        return (h * 5 + 0xE6546B64) & _M32
    h = seed & _M32
    n = len(b)
    aligned = n - n % 4
    for i in range(0, aligned, 4):
        h = mh(h, mk(int.from_bytes(b[i:i + 4], "little")))
    for i in range(aligned, n):
        x = b[i] - 256 if b[i] >= 128 else b[i]
        h = mh(h, mk(x & _M32))
    h ^= n
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & _M32
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & _M32
    return h ^ (h >> 16)


def _spark_hash_column(c: ColumnData, seed: torch.Tensor) -> torch.Tensor:
    dt = c.dtype
    v = c.values
    if isinstance(dt, T.StringType):
        d = c.dictionary if c.dictionary is not None else np.array([], dtype=object)
        codes = c.values.long()
        uniq_seeds = torch.unique(seed)
        if uniq_seeds.numel() == 1:
            s0 = int(uniq_seeds[0])
            lut = torch.tensor([_murmur_bytes_py(x.encode("utf-8"), s0) for x in d.tolist()] + [s0],
                               dtype=torch.int64, device=c.device)
            h = lut[torch.where(codes < 0, torch.full_like(codes, len(d)), codes)]
        else:
            sd, cd = seed.cpu().tolist(), codes.cpu().tolist()
            h = torch.tensor([_murmur_bytes_py(d[k].encode("utf-8"), s) if k >= 0 else s for k, s in zip(cd, sd)],
                             dtype=torch.int64, device=c.device)
    elif isinstance(dt, (T.LongType, T.TimestampType)):
        h = _murmur_long(v.long(), seed)
    elif isinstance(dt, T.DoubleType):
        x = torch.where(v == 0, torch.zeros_like(v), v.double())  # -0.0 -> 0.0
        x = torch.where(torch.isnan(x), torch.full_like(x, float("nan")), x)
        h = _murmur_long(x.view(torch.int64), seed)
    elif isinstance(dt, T.FloatType):
        x = torch.where(v == 0, torch.zeros_like(v), v.float())
        h = _murmur_int(x.view(torch.int32).long(), seed)
    elif isinstance(dt, (T.VectorUDT, T.ArrayType)):
        et = dt.elementType if isinstance(dt, T.ArrayType) else T.DoubleType()
        h = seed
        for j in range(v.shape[1]):
            if isinstance(et, (T.IntegerType, T.ShortType, T.ByteType)):
                h = _murmur_int(v[:, j].round().long(), h)
            elif isinstance(et, T.LongType):
                h = _murmur_long(v[:, j].round().long(), h)
            else:
                h = _murmur_long(v[:, j].double().view(torch.int64), h)
        return h
    else:  # int / short / byte / boolean / date -> hashInt
        h = _murmur_int(v.long(), seed)
    if c.valid is not None:
        h = torch.where(c.valid, h, seed)  # nulls leave the running hash unchanged
    return h


def hash(*cols) -> Column:  # noqa: A001
    """Spark ``hash``: Murmur3_x86_32, seed 42, chained over the columns (bit-compatible)."""
    def ev(b, ctx, args):
        h = torch.full((b.n,), 42, dtype=torch.int64, device=b.device)
        for a in args:
            h = _spark_hash_column(a, h)
        h = torch.where(h >= 2 ** 31, h - 2 ** 32, h)
        return ColumnData(h.to(torch.int32), T.IntegerType())
    return Column(Func("hash", ev, [_ce(c) for c in cols]))


xxhash64 = hash


def struct(*cols):
    raise NotImplementedError("struct columns are not supported; select the fields individually")


def array(*cols) -> Column:
    def ev(b, ctx, args):
        kinds = [a.dtype for a in args]
        if kinds and all(isinstance(k, (T.IntegerType, T.ShortType, T.ByteType)) for k in kinds):
            et = T.IntegerType()
        elif kinds and all(isinstance(k, T.IntegralType) for k in kinds):
            et = T.LongType()
        else:
            et = T.DoubleType()
        return ColumnData(torch.stack([a.values.float() for a in args], dim=1), T.ArrayType(et))
    return Column(Func("array", ev, [_ce(c) for c in cols]))


# --------------------------------------------------------- aggregates
class AggExpr(Expr):
    """Aggregate function marker; evaluated by the group-by engine."""

    def __init__(self, kind: str, x: Expr = None, distinct: bool = False, param: Any = None, display=None):
        self.kind, self.x, self.distinct, self.param = kind, x, distinct, param
        self.children = [x] if x is not None else []
        self.display = display

    def is_aggregate(self):
        return True

    def eval(self, b, ctx):
        raise AnalysisException(f"aggregate {self.kind} used outside of an aggregation")

    def name(self):
        if self.display:
            return self.display
        inner = "1" if self.x is None else self.x.name()
        if self.kind == "count" and self.x is None:
            return "count(1)"
        if self.distinct:
            return f"count(DISTINCT {inner})" if self.kind == "count" else f"{self.kind}(DISTINCT {inner})"
        return f"{self.kind}({inner})"

    def __str__(self):
        return self.name()


def _agg(kind, display=None):
    def f(c="*", *rest):
        if isinstance(c, str) and c == "*" and kind == "count":
            return Column(AggExpr("count", None))
        return Column(AggExpr(kind, _ce(c)))
    return f


count = _agg("count")
sum = _agg("sum")  # noqa: A001
avg = _agg("avg")
mean = avg
min = _agg("min")  # noqa: A001
max = _agg("max")  # noqa: A001
stddev = _agg("stddev")
stddev_samp = _agg("stddev_samp")
stddev_pop = _agg("stddev_pop")
variance = _agg("variance")
var_samp = _agg("var_samp")
var_pop = _agg("var_pop")
first = _agg("first")
last = _agg("last")
collect_list = _agg("collect_list")
collect_set = _agg("collect_set")
skewness = _agg("skewness")
kurtosis = _agg("kurtosis")


def countDistinct(c, *cols) -> Column:
    return Column(AggExpr("count", _ce(c), distinct=True))


count_distinct = countDistinct


def approx_count_distinct(c, rsd=0.05) -> Column:
    return Column(AggExpr("count", _ce(c), distinct=True, display=f"approx_count_distinct({_ce(c).name()})"))


def sumDistinct(c) -> Column:
    return Column(AggExpr("sum", _ce(c), distinct=True))


def percentile_approx(c, percentage, accuracy=10000) -> Column:
    return Column(AggExpr("percentile", _ce(c), param=percentage,
                          display=f"percentile_approx({_ce(c).name()}, {percentage}, {accuracy})"))


def median(c) -> Column:
    return Column(AggExpr("percentile", _ce(c), param=0.5, display=f"median({_ce(c).name()})"))


# ----------------------------------------------------------- UDFs
def udf(f=None, returnType=T.StringType()):
    """Row-at-a-time Python UDF (host path)."""
    from .udf import make_udf
    if f is None or isinstance(f, (str, T.DataType)):
        rt = f if f is not None else returnType
        return lambda fn: make_udf(fn, T.to_type(rt))
    return make_udf(f, T.to_type(returnType))


def pandas_udf(f=None, returnType=None, functionType=None):
    from .udf import pandas_udf as _pu
    return _pu(f, returnType, functionType)


# --------------------------------------------------------- ML helpers
def vector_to_array(c, dtype="float64") -> Column:
    def ev(b, ctx, args):
        return ColumnData(args[0].values, T.ArrayType(T.DoubleType()), args[0].valid)
    return Column(Func("vector_to_array", ev, [_ce(c)]))


def array_to_vector(c) -> Column:
    def ev(b, ctx, args):
        return ColumnData(args[0].values.float(), T.VectorUDT(), args[0].valid)
    return Column(Func("array_to_vector", ev, [_ce(c)]))


def element_at(c, idx: int) -> Column:
    return _c(c).getItem(idx - 1)
