"""GroupedData: distributed hash aggregation.

Rows are hash-partitioned on the group keys (RCCL all-to-all when W > 1) and
aggregated locally with segmented device reductions
(:func:`cdnaml.sql.relational.aggregate`).  ``applyInPandas`` runs a Python
function per group after the same shuffle (ML 13 - Training with Pandas
Function API.py:73-162).
"""
from __future__ import annotations

from typing import List

import torch

from . import relational as R
from . import types as T
from .batch import Batch, concat_batches, empty_batch
from .column import Alias, AnalysisException, ColRef, Column, EvalContext, Expr
from .dataframe import DataFrame, PartitionsPlan
from .functions import AggExpr


class GroupedData:
    def __init__(self, df: DataFrame, keys: List):
        self.df = df
        self.key_exprs: List[Expr] = [ColRef(k) if isinstance(k, str) else k._expr for k in keys]
        self.keys = [e.name() for e in self.key_exprs]

    def _prepared(self):
        """DataFrame with key expressions materialised as columns."""
        df = self.df
        for e, name in zip(self.key_exprs, self.keys):
            if not isinstance(e, ColRef) or e.col_name != name:
                df = df.withColumn(name, Column(e))
        return df

    def agg(self, *exprs) -> DataFrame:
        if len(exprs) == 1 and isinstance(exprs[0], dict):
            from . import functions as F
            fmap = {"avg": F.avg, "mean": F.avg, "sum": F.sum, "min": F.min, "max": F.max, "count": F.count,
                    "stddev": F.stddev, "variance": F.variance, "first": F.first}
            exprs = [fmap[v](k).alias(f"{v if v != 'mean' else 'avg'}({k})") for k, v in exprs[0].items()]
        aggs = []
        pre = []  # (tmp name, expr) for aggregates over computed inputs
        for i, c in enumerate(exprs):
            e = c._expr
            name = e.name()
            inner = e.x if isinstance(e, Alias) else e
            if not isinstance(inner, AggExpr):
                raise AnalysisException(f"expression {name} is not an aggregate function")
            aggs.append((name, inner))
        df = self._prepared()
        keys = self.keys
        session = df._session

        def run(parts):
            P = int(session.conf.get("spark.sql.shuffle.partitions"))
            comm = session.comm
            if not keys:
                b = concat_batches(parts) if parts else empty_batch(df.schema, session.device)
                if comm.distributed:
                    from ..parallel.shuffle import exchange
                    b = exchange(comm, b, torch.zeros(b.n, dtype=torch.long, device=b.device))
                    if comm.rank != 0:
                        return []
                return [R.aggregate(b, [], aggs)]
            from .dataframe import _shuffle
            shuffled = _shuffle(session, parts, P if comm.distributed else 1, keys)
            b = concat_batches(shuffled) if shuffled else empty_batch(df.schema, session.device)
            return [R.aggregate(b, keys, aggs)]

        def sfn(s):
            return R.aggregate(empty_batch(s, torch.device("cpu")), keys, aggs).schema()
        return DataFrame(PartitionsPlan(session, f"HashAggregate(keys={keys}, aggs={[a for a, _ in aggs]})",
                                        [df._plan], run, sfn), session)

    def count(self) -> DataFrame:
        from . import functions as F
        return self.agg(F.count("*").alias("count"))

    def _simple(self, fn, cols):
        from . import functions as F
        if not cols:
            cols = [f.name for f in self.df.schema.fields if f.dataType.is_numeric and f.name not in self.keys]
        name = {F.avg: "avg", F.sum: "sum", F.min: "min", F.max: "max"}[fn]
        return self.agg(*[fn(c).alias(f"{name}({c})") for c in cols])

    def avg(self, *cols):
        from . import functions as F
        return self._simple(F.avg, cols)

    mean = avg

    def sum(self, *cols):
        from . import functions as F
        return self._simple(F.sum, cols)

    def min(self, *cols):
        from . import functions as F
        return self._simple(F.min, cols)

    def max(self, *cols):
        from . import functions as F
        return self._simple(F.max, cols)

    def pivot(self, col, values=None):
        raise NotImplementedError("pivot is not supported")

    # ------------------------------------------------------------ pandas
    def applyInPandas(self, func, schema) -> DataFrame:
        from .udf import apply_in_pandas
        return apply_in_pandas(self, func, schema)

    def apply(self, udf):
        return self.applyInPandas(udf.func, udf.returnType)
