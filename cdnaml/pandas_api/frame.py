"""pandas-API DataFrame / Series over the engine (Koalas InternalFrame design, ML 14:41-65)."""
from __future__ import annotations

import numbers
from typing import Any, Dict, List, Optional, Sequence, Union

import numpy as np
import pandas as pd

from ..sql import functions as F
from ..sql import types as T
from ..sql.column import Column
from .config import get_option

INDEX = "__index_level_0__"


def _session():
    from ..session import SparkSession
    return SparkSession.builder.getOrCreate()


def _attach_index(sdf, index_col: Optional[Union[str, List[str]]] = None):
    """Engine frame -> (frame with an index column, index column name)."""
    if index_col is not None:
        name = index_col if isinstance(index_col, str) else index_col[0]
        return sdf, name
    kind = get_option("compute.default_index_type")
    if kind == "distributed":
        return sdf.withColumn(INDEX, F.monotonically_increasing_id()), INDEX
    return sdf._with_sequence_id(INDEX), INDEX


def from_spark(sdf, index_col=None) -> "DataFrame":
    out, idx = _attach_index(sdf, index_col)
    return DataFrame._internal(out, idx, [c for c in sdf.columns if c != idx])


def from_pandas(pdf: Union[pd.DataFrame, pd.Series]) -> Union["DataFrame", "Series"]:
    if isinstance(pdf, pd.Series):
        return from_pandas(pdf.to_frame())[pdf.name if pdf.name is not None else 0]
    p = pdf.copy()
    p.columns = [str(c) for c in p.columns]
    idx_name = p.index.name or INDEX
    p = p.reset_index().rename(columns={"index": idx_name} if p.index.name is None else {})
    sdf = _session().createDataFrame(p)
    data_cols = [c for c in p.columns if c != idx_name]
    return DataFrame._internal(sdf, idx_name, data_cols, index_label=pdf.index.name)


class DataFrame:
    """pandas-like frame; operations build engine plans, collection is explicit."""

    def __init__(self, data=None, index=None, columns=None, dtype=None, copy=False):
        from ..sql.dataframe import DataFrame as EngineDF
        if isinstance(data, DataFrame):
            self._init(data._sdf, data._idx, list(data._cols), data._index_label)
            return
        if isinstance(data, EngineDF):
            k = from_spark(data)
        else:
            pdf = data if isinstance(data, pd.DataFrame) else pd.DataFrame(data, index=index, columns=columns,
                                                                            dtype=dtype)
            k = from_pandas(pdf)
        self._init(k._sdf, k._idx, k._cols, k._index_label)

    def _init(self, sdf, idx, cols, index_label=None, order=None):
        object.__setattr__(self, "_sdf", sdf)
        object.__setattr__(self, "_idx", idx)
        object.__setattr__(self, "_cols", list(cols))
        object.__setattr__(self, "_index_label", index_label)
        object.__setattr__(self, "_order", order)  # hidden column holding the natural row order

    @classmethod
    def _internal(cls, sdf, idx, cols, index_label=None, order=None) -> "DataFrame":
        obj = cls.__new__(cls)
        obj._init(sdf, idx, cols, index_label, order)
        return obj

    def _with(self, sdf, cols=None) -> "DataFrame":
        return DataFrame._internal(sdf, self._idx, self._cols if cols is None else cols, self._index_label,
                                   self._order)

    def _keep(self):
        """Internal columns every projection must carry."""
        return [self._idx] + ([self._order] if self._order and self._order != self._idx else [])

    # --------------------------------------------------------------- metadata
    @property
    def columns(self) -> pd.Index:
        return pd.Index(self._cols)

    @columns.setter
    def columns(self, names):
        names = list(names)
        if len(names) != len(self._cols):
            raise ValueError("Length mismatch")
        sdf = self._sdf.select(*self._keep(), *[F.col(o).alias(n) for o, n in zip(self._cols, names)])
        self._init(sdf, self._idx, names, self._index_label)

    @property
    def dtypes(self) -> pd.Series:
        return pd.Series({c: _np_dtype(self._sdf.schema[c].dataType) for c in self._cols})

    @property
    def shape(self):
        return (len(self), len(self._cols))

    @property
    def size(self):
        return len(self) * len(self._cols)

    @property
    def empty(self):
        return len(self._cols) == 0 or len(self) == 0

    @property
    def ndim(self):
        return 2

    @property
    def index(self):
        return self.to_pandas().index

    def __len__(self):
        return self._sdf.count()

    def _ordered(self):
        return self._sdf.orderBy(self._order or self._idx)

    # --------------------------------------------------------------- access
    def __getitem__(self, key):
        if isinstance(key, str):
            if key not in self._cols:
                raise KeyError(key)
            return Series(self, F.col(key), key)
        if isinstance(key, Series):
            return self._with(self._sdf.filter(key._col))
        if isinstance(key, (list, tuple, pd.Index)):
            for k in key:
                if k not in self._cols:
                    raise KeyError(k)
            return self._with(self._sdf.select(*self._keep(), *key), list(key))
        if isinstance(key, slice):
            return self.iloc[key]
        raise TypeError(f"unsupported key {key!r}")

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        if name in self._cols:
            return self[name]
        raise AttributeError(f"'DataFrame' object has no attribute '{name}'")

    def __setitem__(self, key, value):
        if isinstance(value, Series):
            col = value._col
        elif isinstance(value, (list, np.ndarray, pd.Series)):
            raise ValueError("assign a pandas-API Series or a scalar (collect-free semantics)")
        else:
            col = F.lit(value)
        sdf = self._sdf.withColumn(key, col)
        cols = self._cols if key in self._cols else self._cols + [key]
        self._init(sdf, self._idx, cols, self._index_label)

    def __contains__(self, k):
        return k in self._cols

    def __iter__(self):
        return iter(self._cols)

    def keys(self):
        return self.columns

    def items(self):
        for c in self._cols:
            yield c, self[c]

    @property
    def iloc(self):
        return _ILoc(self)

    @property
    def loc(self):
        return _Loc(self)

    # --------------------------------------------------------------- conversion
    def to_pandas(self) -> pd.DataFrame:
        pdf = self._ordered().select(self._idx, *self._cols).toPandas()
        pdf = pdf.set_index(self._idx)
        pdf.index.name = self._index_label
        return pdf

    toPandas = to_pandas

    def to_spark(self, index_col: Optional[str] = None):
        cols = ([F.col(self._idx).alias(index_col)] if index_col else []) + list(self._cols)
        return self._sdf.select(*cols)

    def to_koalas(self, index_col=None):
        return self

    pandas_api = to_koalas

    def to_numpy(self):
        return self.to_pandas().to_numpy()

    @property
    def values(self):
        return self.to_numpy()

    def to_dict(self, orient="dict"):
        return self.to_pandas().to_dict(orient)

    def to_csv(self, path=None, sep=",", header=True, **kw):
        if path is None:
            return self.to_pandas().to_csv(sep=sep, header=header)
        self.to_spark().write.mode(kw.get("mode", "overwrite")).option("header", str(header).lower()) \
            .option("sep", sep).csv(path)

    def to_parquet(self, path, mode="overwrite", partition_cols=None, **kw):
        w = self.to_spark().write.mode(mode)
        if partition_cols:
            w = w.partitionBy(*([partition_cols] if isinstance(partition_cols, str) else partition_cols))
        w.parquet(path)

    def to_delta(self, path, mode="overwrite", **kw):
        self.to_spark().write.format("delta").mode(mode).save(path)

    def to_table(self, name, format="delta", mode="overwrite", **kw):  # noqa: A002
        self.to_spark().write.format(format).mode(mode).saveAsTable(name)

    # --------------------------------------------------------------- display
    def head(self, n: int = 5) -> "DataFrame":
        return self._with(self._ordered().limit(n))

    def tail(self, n: int = 5) -> "DataFrame":
        return self._with(self._sdf.orderBy(F.col(self._idx).desc()).limit(n).orderBy(self._idx))

    def __repr__(self):
        mx = get_option("display.max_rows")
        pdf = self.head(mx + 1).to_pandas()
        s = repr(pdf.head(mx))
        if len(pdf) > mx:
            s += f"\n\n[Showing only the first {mx} rows x {len(self._cols)} columns]"
        return s

    def _repr_html_(self):
        return self.head(get_option("display.max_rows")).to_pandas()._repr_html_()

    # --------------------------------------------------------------- reshaping
    def filter(self, items=None, like: Optional[str] = None, regex: Optional[str] = None, axis=None):
        if sum(x is not None for x in (items, like, regex)) != 1:
            raise TypeError("Must pass exactly one of items, like, or regex")
        import re
        if items is not None:
            keep = [c for c in items if c in self._cols]
        elif like is not None:
            keep = [c for c in self._cols if like in c]
        else:
            rx = re.compile(regex)
            keep = [c for c in self._cols if rx.search(c)]
        return self[keep]

    def drop(self, labels=None, axis=1, columns=None):
        cols = columns if columns is not None else labels
        cols = [cols] if isinstance(cols, str) else list(cols)
        keep = [c for c in self._cols if c not in cols]
        return self._with(self._sdf.select(*self._keep(), *keep), keep)

    def rename(self, columns: Optional[Dict[str, str]] = None, mapper=None, axis=None, **kw):
        m = columns or mapper or {}
        new = [m.get(c, c) for c in self._cols]
        sdf = self._sdf.select(*self._keep(), *[F.col(c).alias(m.get(c, c)) for c in self._cols])
        return self._with(sdf, new)

    def assign(self, **kw):
        out = self.copy()
        for k, v in kw.items():
            out[k] = v(out) if callable(v) else v
        return out

    def copy(self, deep=True):
        return DataFrame._internal(self._sdf, self._idx, list(self._cols), self._index_label)

    def astype(self, dtype):
        m = dtype if isinstance(dtype, dict) else {c: dtype for c in self._cols}
        sdf = self._sdf.select(*self._keep(), *[F.col(c).cast(_spark_type(m[c])).alias(c) if c in m else F.col(c)
                                            for c in self._cols])
        return self._with(sdf)

    def fillna(self, value=None, **kw):
        if isinstance(value, dict):
            return self._with(self._sdf.fillna(value))
        return self._with(self._sdf.fillna(value))

    def dropna(self, how="any", subset=None, **kw):
        return self._with(self._sdf.dropna(how=how, subset=subset or self._cols))

    def isnull(self):
        return self._with(self._sdf.select(*self._keep(), *[F.col(c).isNull().alias(c) for c in self._cols]))

    isna = isnull

    def notnull(self):
        return self._with(self._sdf.select(*self._keep(), *[F.col(c).isNotNull().alias(c) for c in self._cols]))

    notna = notnull

    def sort_values(self, by, ascending=True, **kw):
        by = [by] if isinstance(by, str) else list(by)
        asc = [ascending] * len(by) if isinstance(ascending, bool) else list(ascending)
        order = [F.col(b).asc() if a else F.col(b).desc() for b, a in zip(by, asc)]
        s = self._sdf.orderBy(*order)._with_sequence_id("__sorted_pos")
        s = s.drop(self._idx).withColumnRenamed("__sorted_pos", self._idx)
        return self._with(s)

    def sort_index(self, ascending=True, **kw):
        return self if ascending else self._with(self._sdf.orderBy(F.col(self._idx).desc()))

    def reset_index(self, drop=False, **kw):
        base = self._ordered()
        s = base._with_sequence_id("__new_idx")
        cols = list(self._cols)
        if not drop:
            name = self._index_label or "index"
            s = s.withColumnRenamed(self._idx, name)
            cols = [name] + cols
        else:
            s = s.drop(self._idx)
        s = s.withColumnRenamed("__new_idx", INDEX)
        return DataFrame._internal(s, INDEX, cols)

    def set_index(self, keys, drop=True, **kw):
        k = keys if isinstance(keys, str) else keys[0]
        cols = [c for c in self._cols if c != k or not drop]
        order = self._order or self._idx
        return DataFrame._internal(self._sdf, k, cols, index_label=k, order=order)

    def merge(self, right: "DataFrame", how="inner", on=None, left_on=None, right_on=None, suffixes=("_x", "_y")):
        on = [on] if isinstance(on, str) else on
        if on is None:
            raise ValueError("merge needs `on` (column names)")
        l_ = self.to_spark()
        r = right.to_spark()
        dup = [c for c in r.columns if c in l_.columns and c not in on]
        for c in dup:
            l_ = l_.withColumnRenamed(c, c + suffixes[0])
            r = r.withColumnRenamed(c, c + suffixes[1])
        return from_spark(l_.join(r, on=on, how=how))

    def join(self, right, on=None, how="left", lsuffix="", rsuffix=""):
        return self.merge(right, how=how, on=on, suffixes=(lsuffix, rsuffix))

    def groupby(self, by, as_index=True, dropna=True):
        by = [by] if isinstance(by, str) else [b.name if isinstance(b, Series) else b for b in by]
        return GroupBy(self, by, as_index)

    # --------------------------------------------------------------- stats
    def _numeric(self):
        return [c for c in self._cols if self._sdf.schema[c].dataType.is_numeric]

    def _reduce(self, fn, numeric_only=True) -> pd.Series:
        cols = self._numeric() if numeric_only else self._cols
        if not cols:
            return pd.Series(dtype=float)
        row = self._sdf.agg(*[fn(F.col(c)).alias(c) for c in cols]).collect()[0]
        return pd.Series({c: row[i] for i, c in enumerate(cols)})

    def count(self):
        return self._reduce(F.count, numeric_only=False).astype("int64")

    def sum(self, numeric_only=True):
        return self._reduce(F.sum)

    def mean(self, numeric_only=True):
        return self._reduce(F.avg)

    def min(self, numeric_only=True):
        return self._reduce(F.min)

    def max(self, numeric_only=True):
        return self._reduce(F.max)

    def std(self, ddof=1, numeric_only=True):
        return self._reduce(F.stddev if ddof == 1 else F.stddev_pop)

    def var(self, ddof=1, numeric_only=True):
        return self._reduce(F.variance if ddof == 1 else F.var_pop)

    def median(self, numeric_only=True):
        return self.quantile(0.5)

    def quantile(self, q=0.5, numeric_only=True):
        cols = self._numeric()
        qs = [q] if isinstance(q, numbers.Number) else list(q)
        vals = self._sdf.approxQuantile(cols, qs, 0.0)
        if isinstance(q, numbers.Number):
            return pd.Series({c: v[0] if v else np.nan for c, v in zip(cols, vals)})
        return pd.DataFrame({c: v for c, v in zip(cols, vals)}, index=qs)

    def describe(self, percentiles=None):
        cols = self._numeric()
        ps = percentiles or [0.25, 0.5, 0.75]
        stats = ["count", "mean", "stddev", "min"] + [f"{int(p * 100)}%" for p in ps] + ["max"]
        s = self._sdf.select(*cols).summary(*stats).toPandas().set_index("summary").astype(float)
        s.index = ["count", "mean", "std", "min"] + [f"{int(p * 100)}%" for p in ps] + ["max"]
        s.index.name = None
        return s

    def corr(self, method="pearson"):
        cols = self._numeric()
        out = pd.DataFrame(np.eye(len(cols)), index=cols, columns=cols)
        for i, a in enumerate(cols):
            for b in cols[i + 1:]:
                v = self._sdf.corr(a, b)
                out.loc[a, b] = out.loc[b, a] = v
        return out

    def nunique(self, dropna=True):
        row = self._sdf.agg(*[F.countDistinct(F.col(c)).alias(c) for c in self._cols]).collect()[0]
        return pd.Series({c: row[i] for i, c in enumerate(self._cols)})

    def nlargest(self, n, columns):
        return self.sort_values(columns, ascending=False).head(n)

    def nsmallest(self, n, columns):
        return self.sort_values(columns, ascending=True).head(n)

    def apply(self, func, axis=0):
        return from_pandas(self.to_pandas().apply(func, axis=axis))

    # --------------------------------------------------------------- plotting
    @property
    def plot(self):
        return _PlotAccessor(self)

    def hist(self, bins=10, **kw):
        return self.plot.hist(bins=bins, **kw)


class Series:
    """A column anchored to a pandas-API frame."""

    def __init__(self, anchor: DataFrame, col: Column, name: Optional[str]):
        self._anchor = anchor
        self._col = col
        self._name = name

    # --------------------------------------------------------------- basics
    @property
    def name(self):
        return self._name

    @name.setter
    def name(self, v):
        self._name = v

    def rename(self, name):
        return Series(self._anchor, self._col, name)

    @property
    def dtype(self):
        sdf = self._frame_sdf()
        return _np_dtype(sdf.schema[self._out_name()].dataType)

    def _out_name(self):
        return self._name if self._name is not None else "0"

    def _frame_sdf(self):
        a = self._anchor
        return a._sdf.select(*a._keep(), self._col.alias(self._out_name()))

    def to_frame(self, name=None) -> DataFrame:
        n = name or self._out_name()
        a = self._anchor
        return DataFrame._internal(a._sdf.select(*a._keep(), self._col.alias(n)), a._idx, [n], a._index_label,
                                   a._order)

    def to_pandas(self) -> pd.Series:
        s = self.to_frame().to_pandas().iloc[:, 0]
        s.name = self._name
        return s

    def to_numpy(self):
        return self.to_pandas().to_numpy()

    @property
    def values(self):
        return self.to_numpy()

    def to_list(self):
        return self.to_pandas().tolist()

    tolist = to_list

    def __len__(self):
        return len(self._anchor)

    def head(self, n=5):
        return Series(self._anchor.head(n), self._col, self._name)

    def __repr__(self):
        return repr(self.head(get_option("display.max_rows")).to_pandas())

    # --------------------------------------------------------------- arithmetic
    def _bin(self, other, op):
        o = other._col if isinstance(other, Series) else other
        return Series(self._anchor, op(self._col, o), self._name)

    def __add__(self, o): return self._bin(o, lambda a, b: a + b)  # noqa: E704
    def __radd__(self, o): return self._bin(o, lambda a, b: b + a)  # noqa: E704
    def __sub__(self, o): return self._bin(o, lambda a, b: a - b)  # noqa: E704
    def __rsub__(self, o): return self._bin(o, lambda a, b: b - a)  # noqa: E704
    def __mul__(self, o): return self._bin(o, lambda a, b: a * b)  # noqa: E704
    def __rmul__(self, o): return self._bin(o, lambda a, b: b * a)  # noqa: E704
    def __truediv__(self, o): return self._bin(o, lambda a, b: a / b)  # noqa: E704
    def __rtruediv__(self, o): return self._bin(o, lambda a, b: b / a)  # noqa: E704
    def __mod__(self, o): return self._bin(o, lambda a, b: a % b)  # noqa: E704
    def __pow__(self, o): return self._bin(o, lambda a, b: F.pow(a, b))  # noqa: E704
    def __eq__(self, o): return self._bin(o, lambda a, b: a == b)  # noqa: E704
    def __ne__(self, o): return self._bin(o, lambda a, b: a != b)  # noqa: E704
    def __lt__(self, o): return self._bin(o, lambda a, b: a < b)  # noqa: E704
    def __le__(self, o): return self._bin(o, lambda a, b: a <= b)  # noqa: E704
    def __gt__(self, o): return self._bin(o, lambda a, b: a > b)  # noqa: E704
    def __ge__(self, o): return self._bin(o, lambda a, b: a >= b)  # noqa: E704
    def __and__(self, o): return self._bin(o, lambda a, b: a & b)  # noqa: E704
    def __or__(self, o): return self._bin(o, lambda a, b: a | b)  # noqa: E704

    def __invert__(self):
        return Series(self._anchor, ~self._col, self._name)

    def __neg__(self):
        return Series(self._anchor, -self._col, self._name)

    def __abs__(self):
        return Series(self._anchor, F.abs(self._col), self._name)

    abs = __abs__

    __hash__ = object.__hash__

    def astype(self, dtype):
        return Series(self._anchor, self._col.cast(_spark_type(dtype)), self._name)

    def isnull(self):
        return Series(self._anchor, self._col.isNull(), self._name)

    isna = isnull

    def notnull(self):
        return Series(self._anchor, self._col.isNotNull(), self._name)

    notna = notnull

    def fillna(self, value):
        return Series(self._anchor, F.coalesce(self._col, F.lit(value)), self._name)

    def between(self, left, right, inclusive="both"):
        return Series(self._anchor, (self._col >= left) & (self._col <= right), self._name)

    def isin(self, values):
        return Series(self._anchor, self._col.isin(list(values)), self._name)

    def clip(self, lower=None, upper=None):
        c = self._col
        if lower is not None:
            c = F.when(c < lower, F.lit(lower)).otherwise(c)
        if upper is not None:
            c = F.when(c > upper, F.lit(upper)).otherwise(c)
        return Series(self._anchor, c, self._name)

    @property
    def str(self):
        return _StrAccessor(self)

    # --------------------------------------------------------------- reductions
    def _agg(self, fn):
        return self._frame_sdf().agg(fn(F.col(self._out_name()))).collect()[0][0]

    def count(self): return int(self._agg(F.count))  # noqa: E704
    def sum(self): return self._agg(F.sum)  # noqa: E704
    def mean(self): return self._agg(F.avg)  # noqa: E704
    def min(self): return self._agg(F.min)  # noqa: E704
    def max(self): return self._agg(F.max)  # noqa: E704
    def std(self, ddof=1): return self._agg(F.stddev if ddof == 1 else F.stddev_pop)  # noqa: E704
    def var(self, ddof=1): return self._agg(F.variance if ddof == 1 else F.var_pop)  # noqa: E704

    def median(self):
        return self.quantile(0.5)

    def quantile(self, q=0.5):
        v = self._frame_sdf().approxQuantile(self._out_name(), [q] if isinstance(q, numbers.Number) else list(q),
                                             0.0)
        return v[0] if isinstance(q, numbers.Number) else pd.Series(v, index=list(q))

    def nunique(self, dropna=True):
        return int(self._agg(F.countDistinct))

    def unique(self):
        n = self._out_name()
        return self._frame_sdf().select(n).distinct().toPandas()[n].to_numpy()

    def value_counts(self, normalize=False, sort=True, ascending=False, dropna=True) -> "Series":
        n = self._out_name()
        sdf = self._frame_sdf().select(n)
        if dropna:
            sdf = sdf.filter(F.col(n).isNotNull())
        g = sdf.groupBy(n).count()
        if normalize:
            tot = sdf.count()
            g = g.withColumn("count", F.col("count") / float(max(tot, 1)))
        if sort:
            g = g.orderBy(F.col("count").asc() if ascending else F.col("count").desc(), n)
        g = g._with_sequence_id("__vc_pos")
        k = DataFrame._internal(g, "__vc_pos", [n, "count"])
        # pandas-on-Spark value_counts: the values become the index
        out = k.set_index(n)
        return Series(out, F.col("count"), "proportion" if normalize else "count")

    # --------------------------------------------------------------- plotting
    @property
    def plot(self):
        return _PlotAccessor(self.to_frame())

    def hist(self, bins=10, **kw):
        return self.plot.hist(bins=bins, **kw)


class GroupBy:
    def __init__(self, kdf: DataFrame, by: List[str], as_index: bool):
        self._k = kdf
        self._by = by
        self._as_index = as_index

    def _finish(self, sdf, cols):
        if self._as_index:
            k = from_spark(sdf.orderBy(*self._by))
            if len(self._by) == 1:
                return k.set_index(self._by[0])
            return k
        return from_spark(sdf.orderBy(*self._by))

    def _agg_all(self, fn, name):
        vals = [c for c in self._k._cols if c not in self._by and self._k._sdf.schema[c].dataType.is_numeric]
        sdf = self._k._sdf.groupBy(*self._by).agg(*[fn(F.col(c)).alias(c) for c in vals])
        return self._finish(sdf, vals)

    def sum(self): return self._agg_all(F.sum, "sum")  # noqa: E704
    def mean(self): return self._agg_all(F.avg, "mean")  # noqa: E704
    def min(self): return self._agg_all(F.min, "min")  # noqa: E704
    def max(self): return self._agg_all(F.max, "max")  # noqa: E704
    def std(self): return self._agg_all(F.stddev, "std")  # noqa: E704

    def count(self):
        vals = [c for c in self._k._cols if c not in self._by]
        sdf = self._k._sdf.groupBy(*self._by).agg(*[F.count(F.col(c)).alias(c) for c in vals])
        return self._finish(sdf, vals)

    def size(self):
        sdf = self._k._sdf.groupBy(*self._by).count()
        k = self._finish(sdf, ["count"])
        return k["count"]

    def agg(self, spec):
        fns = {"sum": F.sum, "mean": F.avg, "avg": F.avg, "min": F.min, "max": F.max, "count": F.count,
               "std": F.stddev, "var": F.variance}
        exprs = []
        for c, f in spec.items():
            for fn in ([f] if isinstance(f, str) else f):
                exprs.append(fns[fn](F.col(c)).alias(c if isinstance(f, str) else f"{c}_{fn}"))
        sdf = self._k._sdf.groupBy(*self._by).agg(*exprs)
        return self._finish(sdf, None)

    def __getitem__(self, cols):
        cols = [cols] if isinstance(cols, str) else list(cols)
        sub = self._k[self._by + [c for c in cols if c not in self._by]]
        return GroupBy(sub, self._by, self._as_index)


class _ILoc:
    def __init__(self, k):
        self._k = k

    def __getitem__(self, key):
        rows, cols = (key, slice(None)) if not isinstance(key, tuple) else key
        k = self._k
        if isinstance(cols, slice):
            keep = k._cols[cols]
        else:
            keep = [k._cols[i] for i in ([cols] if isinstance(cols, int) else cols)]
        s = k._ordered()._with_sequence_id("__pos")
        if isinstance(rows, slice):
            start, stop, step = rows.start or 0, rows.stop, rows.step or 1
            cond = F.col("__pos") >= start
            if stop is not None:
                cond = cond & (F.col("__pos") < stop)
            if step != 1:
                cond = cond & (((F.col("__pos") - start) % step) == 0)
            s = s.filter(cond)
        elif isinstance(rows, int):
            return k._with(s.filter(F.col("__pos") == rows).drop("__pos")).to_pandas()[keep].iloc[0]
        else:
            s = s.filter(F.col("__pos").isin(list(rows)))
        return DataFrame._internal(s.drop("__pos").select(k._idx, *keep), k._idx, keep, k._index_label)


class _Loc:
    def __init__(self, k):
        self._k = k

    def __getitem__(self, key):
        rows, cols = (key, None) if not isinstance(key, tuple) else key
        k = self._k
        out = k[rows] if isinstance(rows, Series) else k
        if cols is not None and not (isinstance(cols, slice) and cols == slice(None)):
            out = out[[cols] if isinstance(cols, str) else list(cols)]
            if isinstance(cols, str):
                return out[cols]
        return out


class _StrAccessor:
    def __init__(self, s: Series):
        self._s = s

    def _w(self, c):
        return Series(self._s._anchor, c, self._s._name)

    def lower(self): return self._w(F.lower(self._s._col))  # noqa: E704
    def upper(self): return self._w(F.upper(self._s._col))  # noqa: E704
    def len(self): return self._w(F.length(self._s._col))  # noqa: E704
    def strip(self): return self._w(F.trim(self._s._col))  # noqa: E704

    def contains(self, pat, regex=True):
        return self._w(self._s._col.rlike(pat) if regex else self._s._col.contains(pat))

    def startswith(self, pat):
        return self._w(self._s._col.startswith(pat))

    def replace(self, pat, repl, regex=True):
        return self._w(F.regexp_replace(self._s._col, pat, repl))


class _PlotAccessor:
    """Plots collect at most ``plotting.max_rows`` rows (Koalas' top-n / sample
    semantics) and draw with the configured backend."""

    def __init__(self, k: DataFrame):
        self._k = k

    def _pdf(self):
        mx = get_option("plotting.max_rows")
        n = len(self._k)
        ratio = get_option("plotting.sample_ratio")
        k = self._k
        if ratio is None and n > mx:
            ratio = mx / n
        if ratio is not None and ratio < 1:
            k = k._with(k._sdf.sample(fraction=float(ratio), seed=0))
        return k.to_pandas()

    def _backend(self):
        b = get_option("plotting.backend")
        if b == "matplotlib":
            import matplotlib
            if matplotlib.get_backend().lower() not in ("agg", "module://matplotlib_inline.backend_inline"):
                try:
                    matplotlib.use("Agg")
                except Exception:  # noqa: BLE001
                    pass
        return b

    def __call__(self, kind="line", **kw):
        self._backend()
        pdf = self._pdf()
        return pdf.plot(kind=kind, **kw)

    def hist(self, bins=10, x=None, y=None, **kw):
        self._backend()
        pdf = self._pdf()
        if y is not None:
            pdf = pdf[[y] if isinstance(y, str) else list(y)]
        return pdf.plot.hist(bins=bins, **kw)

    def bar(self, x=None, y=None, **kw):
        self._backend()
        return self._pdf().plot.bar(x=x, y=y, **kw)

    def line(self, x=None, y=None, **kw):
        self._backend()
        return self._pdf().plot.line(x=x, y=y, **kw)

    def scatter(self, x, y, **kw):
        self._backend()
        return self._pdf().plot.scatter(x=x, y=y, **kw)

    def box(self, **kw):
        self._backend()
        return self._pdf().plot.box(**kw)

    def pie(self, **kw):
        self._backend()
        return self._pdf().plot.pie(**kw)

    def area(self, **kw):
        self._backend()
        return self._pdf().plot.area(**kw)

    def kde(self, **kw):
        self._backend()
        return self._pdf().plot.kde(**kw)

    density = kde


# ------------------------------------------------------------------ helpers
def _np_dtype(dt: T.DataType):
    m = {T.DoubleType: np.dtype("float64"), T.FloatType: np.dtype("float32"), T.IntegerType: np.dtype("int32"),
         T.LongType: np.dtype("int64"), T.ShortType: np.dtype("int16"), T.ByteType: np.dtype("int8"),
         T.BooleanType: np.dtype("bool"), T.TimestampType: np.dtype("datetime64[ns]")}
    for k, v in m.items():
        if isinstance(dt, k):
            return v
    return np.dtype("object")


def _spark_type(dtype) -> str:
    if isinstance(dtype, str):
        return {"float64": "double", "float": "double", "float32": "float", "int64": "bigint", "int": "bigint",
                "int32": "int", "bool": "boolean", "str": "string", "object": "string"}.get(dtype, dtype)
    d = np.dtype(dtype) if dtype not in (str, object) else np.dtype(object)
    return {"f": "double" if d.itemsize == 8 else "float", "i": "bigint" if d.itemsize == 8 else "int",
            "b": "boolean", "O": "string", "U": "string"}.get(d.kind, "string")
