"""Top-level pandas-API functions: readers, ``sql`` with ``{kdf}`` placeholders, concat."""
from __future__ import annotations

import inspect
import string
import uuid
from typing import List, Optional

from .frame import DataFrame, Series, _session, from_spark


def read_parquet(path: str, columns: Optional[List[str]] = None, index_col=None, **kw) -> DataFrame:
    sdf = _session().read.parquet(path)
    if columns:
        sdf = sdf.select(*(list(columns) + ([index_col] if isinstance(index_col, str) else list(index_col or []))))
    return from_spark(sdf, index_col)


def read_csv(path: str, sep: str = ",", header="infer", names=None, usecols=None, index_col=None,
             dtype=None, **kw) -> DataFrame:
    r = _session().read.option("header", "true" if header in ("infer", 0, True) and names is None else "false") \
        .option("sep", sep).option("inferSchema", "true")
    sdf = r.csv(path)
    if names:
        sdf = sdf.toDF(*names)
    if usecols:
        sdf = sdf.select(*usecols)
    return from_spark(sdf, index_col)


def read_json(path: str, lines: bool = True, index_col=None, **kw) -> DataFrame:
    return from_spark(_session().read.json(path), index_col)


def read_delta(path: str, version: Optional[str] = None, timestamp: Optional[str] = None, index_col=None,
               **kw) -> DataFrame:
    r = _session().read.format("delta")
    if version is not None:
        r = r.option("versionAsOf", version)
    if timestamp is not None:
        r = r.option("timestampAsOf", timestamp)
    return from_spark(r.load(path), index_col)


def read_table(name: str, index_col=None) -> DataFrame:
    return from_spark(_session().table(name), index_col)


def sql(query: str, index_col=None, **kwargs) -> DataFrame:
    """``ks.sql("select distinct(property_type) from {kdf}")`` — names in braces are
    resolved from ``kwargs`` or the caller's variables (ML 14:194)."""
    frame = inspect.currentframe().f_back
    scope = dict(frame.f_globals)
    scope.update(frame.f_locals)
    scope.update(kwargs)
    session = _session()
    views = []
    mapping = {}
    for _, field, _, _ in string.Formatter().parse(query):
        if not field or field in mapping:
            continue
        obj = scope.get(field)
        if isinstance(obj, (DataFrame, Series)):
            sdf = obj.to_spark() if isinstance(obj, DataFrame) else obj.to_frame().to_spark()
            v = f"__ks_{field}_{uuid.uuid4().hex[:8]}"
            sdf.createOrReplaceTempView(v)
            views.append(v)
            mapping[field] = v
        elif hasattr(obj, "createOrReplaceTempView"):
            v = f"__ks_{field}_{uuid.uuid4().hex[:8]}"
            obj.createOrReplaceTempView(v)
            views.append(v)
            mapping[field] = v
        elif obj is not None:
            mapping[field] = repr(obj) if isinstance(obj, str) else str(obj)
    try:
        out = session.sql(query.format(**mapping))
        return from_spark(out.cache() if hasattr(out, "cache") else out, index_col)
    finally:
        for v in views:
            pass  # temp views live until the session ends (the plan may still reference them lazily)


def concat(objs, axis=0, ignore_index=False, **kw) -> DataFrame:
    objs = list(objs)
    if axis not in (0, "index"):
        raise NotImplementedError("concat along columns is not supported")
    cols = []
    for o in objs:
        for c in o._cols:
            if c not in cols:
                cols.append(c)
    from ..feature_store import _union_by_name
    sdf = objs[0].to_spark()
    for o in objs[1:]:
        sdf = _union_by_name(sdf, o.to_spark())
    return from_spark(sdf.select(*cols))


def to_datetime(arg, format=None, **kw):  # noqa: A002
    from ..sql import functions as F
    if isinstance(arg, Series):
        c = F.to_timestamp(arg._col, format) if format else arg._col.cast("timestamp")
        return Series(arg._anchor, c, arg._name)
    import pandas as pd
    return pd.to_datetime(arg, format=format, **kw)
