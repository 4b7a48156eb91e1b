"""Python/pandas bridge: udf, pandas_udf, mapInPandas, applyInPandas (SURVEY §2.4 B2–B6).

Device partitions are cut into Arrow-sized record batches
(``spark.sql.execution.arrow.maxRecordsPerBatch``, default 10,000 —
ML 12 - Inference with Pandas UDFs.py:90,121), moved to host pandas, handed
to the user function, and the results moved back to the device.  Models of
this framework never need this path: ``Model.transform`` and
``tracking.pyfunc.spark_udf`` run the native predict kernels on device.
"""
from __future__ import annotations

import inspect
import typing
from typing import Iterator

import numpy as np
import pandas as pd
import torch

from . import types as T
from .batch import Batch, batch_from_pandas, column_from_numpy, concat_batches, empty_batch
from .column import Column, Func, _to_expr


def _max_records(session) -> int:
    try:
        return int(session.conf.get("spark.sql.execution.arrow.maxRecordsPerBatch"))
    except Exception:
        return 10000


class UserDefinedFunction:
    def __init__(self, func, returnType, kind="row"):
        self.func = func
        self.returnType = returnType
        self.evalType = kind
        self.__name__ = getattr(func, "__name__", "udf")

    def __call__(self, *cols):
        from .functions import col
        exprs = [col(c)._expr if isinstance(c, str) else _to_expr(c) for c in cols]
        udf = self

        def ev(b, ctx, args):
            return udf._run(b, ctx, args)
        return Column(Func(self.__name__, ev, exprs))

    # ---------------------------------------------------------------- exec
    def _result_column(self, values, device):
        rt = self.returnType
        if isinstance(rt, T.StructType):
            raise NotImplementedError("struct-returning UDFs are not supported")
        if isinstance(values, pd.DataFrame):
            values = values.iloc[:, 0]
        arr = values.to_numpy() if isinstance(values, pd.Series) else np.asarray(values)
        return column_from_numpy(arr, rt, device)

    def _run(self, b, ctx, args):
        if b.n == 0:
            # Spark never hands a UDF an empty batch (schema inference here runs plans on 0 rows): models such
            # as sklearn estimators raise on 0 samples
            return column_from_numpy(np.array([], dtype=object), self.returnType, b.device)
        session = ctx.session
        bs = _max_records(session) if session is not None else 10000
        if self.evalType == "row":
            hosts = [a.to_numpy() for a in args]
            out = [self.func(*vals) for vals in zip(*hosts)] if hosts else [self.func() for _ in range(b.n)]
            return column_from_numpy(np.array(out, dtype=object), self.returnType, b.device)
        series = [pd.Series(a.to_numpy()) for a in args]
        chunks = [(s0, min(b.n, s0 + bs)) for s0 in range(0, b.n, bs)]
        if self.evalType == "scalar":
            outs = [self.func(*[s.iloc[a:z].reset_index(drop=True) for s in series]) for a, z in chunks]
        elif self.evalType == "scalar_iter":
            def gen():
                for a, z in chunks:
                    parts = [s.iloc[a:z].reset_index(drop=True) for s in series]
                    yield parts[0] if len(parts) == 1 else tuple(parts)
            outs = list(self.func(gen()))
        else:
            raise ValueError(self.evalType)
        if not outs:
            return column_from_numpy(np.array([], dtype=object), self.returnType, b.device)
        res = pd.concat([o if isinstance(o, (pd.Series, pd.DataFrame)) else pd.Series(o) for o in outs],
                        ignore_index=True)
        return self._result_column(res, b.device)


def make_udf(f, returnType):
    return UserDefinedFunction(f, returnType, "row")


class PandasUDFType:
    SCALAR = 200
    SCALAR_ITER = 204
    GROUPED_MAP = 201
    GROUPED_AGG = 202


def _infer_kind(f):
    try:
        hints = typing.get_type_hints(f)
    except Exception:
        hints = getattr(f, "__annotations__", {})
    ret = hints.get("return")
    origin = typing.get_origin(ret)
    if origin in (typing.Iterator, Iterator) or (origin is not None and getattr(origin, "__name__", "") in
                                                  ("Iterator", "Iterable")):
        return "scalar_iter"
    try:
        import collections.abc as cabc
        if origin in (cabc.Iterator, cabc.Iterable):
            return "scalar_iter"
    except Exception:
        pass
    return "scalar"


def pandas_udf(f=None, returnType=None, functionType=None):
    """``@pandas_udf("double")`` (Series->Series) or Iterator[...] -> Iterator[Series]."""
    if f is not None and not callable(f):
        returnType, f = f, None
    if isinstance(returnType, int) and functionType is None:
        functionType, returnType = returnType, None

    def wrap(fn):
        rt = T.to_type(returnType) if returnType is not None else T.DoubleType()
        if isinstance(returnType, str) and ("," in returnType or " " in returnType.strip()):
            rt = T.to_schema(returnType)
        if functionType == PandasUDFType.GROUPED_MAP:
            return UserDefinedFunction(fn, rt, "grouped_map")
        kind = "scalar_iter" if functionType == PandasUDFType.SCALAR_ITER else _infer_kind(fn)
        return UserDefinedFunction(fn, rt, kind)
    if f is not None:
        return wrap(f)
    return wrap


# ----------------------------------------------------------- mapInPandas
def map_in_pandas(df, func, schema):
    from .dataframe import MapPlan
    schema = T.to_schema(schema)
    session = df._session

    def fn(b, ctx):
        bs = _max_records(session)
        if b.n == 0 and not b.names:
            return empty_batch(schema, b.device)
        pdf = b.to_pandas() if b.n else pd.DataFrame({k: pd.Series(dtype=object) for k in b.names})

        def gen():
            for s0 in range(0, max(b.n, 1), bs):
                yield pdf.iloc[s0:s0 + bs].reset_index(drop=True)
        outs = [o for o in func(gen())] if b.n else []
        outs = [o for o in outs if o is not None and len(o)]
        if not outs:
            return empty_batch(schema, b.device)
        res = pd.concat(outs, ignore_index=True)
        return batch_from_pandas(res[[c for c in schema.names]], schema, b.device)
    plan = MapPlan(df._plan, "MapInPandas", fn)
    plan._schema = schema
    from .dataframe import DataFrame
    return DataFrame(plan, session)


# -------------------------------------------------------- applyInPandas
def _apply_parallelism(session, ngroups: int) -> int:
    """Threads for applyInPandas groups: ``cdnaml.applyInPandas.parallelism`` (default: one per group, at most
    the process's CPU share, capped at 16)."""
    import os
    try:
        v = int(session.conf.get("cdnaml.applyInPandas.parallelism"))
    except Exception:
        v = 0
    if v <= 0:
        try:
            cpus = len(os.sched_getaffinity(0))
        except AttributeError:
            cpus = os.cpu_count() or 1
        v = min(16, cpus)
    return max(1, min(v, ngroups))


def apply_in_pandas(grouped, func, schema):
    from .dataframe import DataFrame, PartitionsPlan, _shuffle
    schema = T.to_schema(schema)
    df = grouped._prepared()
    keys = grouped.keys
    session = df._session
    nparams = len(inspect.signature(func).parameters)

    def run(parts):
        comm = session.comm
        P = int(session.conf.get("spark.sql.shuffle.partitions"))
        shuffled = _shuffle(session, parts, P if comm.distributed else 1, keys)
        b = concat_batches(shuffled) if shuffled else empty_batch(df.schema, session.device)
        if b.n == 0:
            return [empty_batch(schema, session.device)]
        pdf = b.to_pandas()
        groups = [(key, g.reset_index(drop=True)) for key, g in pdf.groupby(keys, sort=True, dropna=False)]

        def one(item):
            key, g = item
            if nparams == 2:
                return func(key if isinstance(key, tuple) else (key,), g)
            return func(g)
        # groups are independent: a thread pool runs them concurrently (numpy / scikit-learn / this engine's
        # kernels release the GIL; the tracking store is thread-safe, with thread-local active runs), and
        # the results are concatenated in group order, as the serial loop would
        par = _apply_parallelism(session, len(groups))
        if par > 1:
            from concurrent.futures import ThreadPoolExecutor
            with ThreadPoolExecutor(max_workers=par) as ex:
                results = list(ex.map(one, groups))
        else:
            results = [one(it) for it in groups]
        outs = [o for o in results if o is not None and len(o)]
        if not outs:
            return [empty_batch(schema, session.device)]
        res = pd.concat(outs, ignore_index=True)
        return [batch_from_pandas(res[[c for c in schema.names]], schema, session.device)]
    return DataFrame(PartitionsPlan(session, f"FlatMapGroupsInPandas({keys})", [df._plan], run, lambda s: schema),
                     session)
