"""Lazy, distributed, device-resident DataFrame (SURVEY §1 L2, §2.3 D1–D10).

SPMD model: every rank runs the same program; a DataFrame's partitions on a
rank live in that rank's GPU memory.  Transformations build a plan (nothing
runs: ML 00b - Spark Review.py:41-45); actions execute it and combine
per-rank results with RCCL collectives (``count`` = all-reduce, ``collect``
= all-gather, shuffles = all-to-all).  ``cache()`` keeps the materialised
partitions resident in HBM (ML 00b:88-104).
"""
from __future__ import annotations

import math

import itertools
from typing import Iterator, Callable, Dict, List, Optional, Sequence, Union

import numpy as np
import pandas as pd
import torch

from . import relational as R
from . import types as T
from .batch import Batch, ColumnData, concat_batches, empty_batch
from .column import (Alias, AnalysisException, ColRef, Column, EvalContext, Expr, Lit, SortOrder, Star, _to_expr)
from . import fused as _fused

_PART_STRIDE = 1 << 20


# ===================================================================== plans
class Plan:
    """A lazily evaluated node producing this rank's partitions."""

    def __init__(self, session, name: str, children: Sequence["Plan"] = ()):
        self.session = session
        self.name = name
        self.children = list(children)
        self.cached = False
        self._result: Optional[List[Batch]] = None
        self._schema: Optional[T.StructType] = None

    def execute(self) -> List[Batch]:
        if self._result is not None:
            return self._result
        res = self._execute()
        if self.cached:
            self._result = res
        return res

    @property
    def streamable(self) -> bool:
        """True when partitions can be produced one at a time (out-of-core narrow pipelines)."""
        return False

    def iter_execute(self) -> Iterator[Batch]:
        """This rank's partitions one at a time.  Streamed sources (``SparkSession.createDataFrameFromChunks``)
        produce them lazily, so a narrow pipeline over data larger than HBM never holds more than its
        staging buffers; other plans yield their materialised partitions."""
        if self._result is not None or not self.streamable:
            yield from self.execute()
        else:
            yield from self._iter_execute()

    def _iter_execute(self) -> Iterator[Batch]:  # pragma: no cover
        yield from self._execute()

    def _execute(self) -> List[Batch]:  # pragma: no cover
        raise NotImplementedError

    def schema(self) -> T.StructType:
        if self._schema is None:
            self._schema = self._compute_schema()
        return self._schema

    def _compute_schema(self) -> T.StructType:  # pragma: no cover
        raise NotImplementedError

    def prototype(self) -> Batch:
        """An empty batch with this plan's schema (CPU), for schema inference."""
        return empty_batch(self.schema(), torch.device("cpu"))

    def tree_string(self, indent=0) -> str:
        s = "  " * indent + ("*" if self.cached else "") + self.name + "\n"
        for c in self.children:
            s += c.tree_string(indent + 1)
        return s


class SourcePlan(Plan):
    """Leaf.  ``iter_fn`` (optional) yields the partitions lazily; each yielded batch may alias a staging
    buffer that is reused once the consumer asks for the next one, so materialising such a source clones."""

    def __init__(self, session, name, fn: Optional[Callable[[], List[Batch]]], schema: T.StructType,
                 iter_fn: Optional[Callable[[], Iterator[Batch]]] = None):
        super().__init__(session, name)
        self.fn = fn
        self.iter_fn = iter_fn
        self._schema = schema

    @property
    def streamable(self) -> bool:
        return self.iter_fn is not None

    def _execute(self):
        if self.fn is None:
            return [b.clone() for b in self.iter_fn()]
        return self.fn()

    def _iter_execute(self):
        yield from self.iter_fn()

    def _compute_schema(self):
        return self._schema


class MapPlan(Plan):
    """Per-partition transformation (narrow dependency, no collectives)."""

    def __init__(self, child: Plan, name: str, fn: Callable[[Batch, EvalContext], Batch]):
        super().__init__(child.session, name, [child])
        self.fn = fn

    def _execute(self):
        out = []
        rank = self.session.comm.rank
        for i, b in enumerate(self.children[0].execute()):
            out.append(self.fn(b, EvalContext(self.session, rank * _PART_STRIDE + i, 0)))
        return out

    @property
    def streamable(self) -> bool:
        return self.children[0].streamable

    def _iter_execute(self):
        rank = self.session.comm.rank
        for i, b in enumerate(self.children[0].iter_execute()):
            yield self.fn(b, EvalContext(self.session, rank * _PART_STRIDE + i, 0))

    def _compute_schema(self):
        b = self.fn(self.children[0].prototype(), EvalContext(self.session, 0, 0))
        return b.schema()


class PartitionsPlan(Plan):
    """Whole-partition-list transformation (may use collectives)."""

    def __init__(self, session, name, children, fn, schema_fn):
        super().__init__(session, name, children)
        self.fn = fn
        self.schema_fn = schema_fn

    def _execute(self):
        return self.fn(*[c.execute() for c in self.children])

    def _compute_schema(self):
        return self.schema_fn(*[c.schema() for c in self.children])


# ================================================================== helpers
def _expr_list(cols) -> List[Expr]:
    out = []
    for c in cols:
        if isinstance(c, (list, tuple)):
            out.extend(_expr_list(c))
        elif isinstance(c, str):
            out.append(Star() if c == "*" else ColRef(c))
        elif isinstance(c, Column):
            out.append(c._expr)
        else:
            out.append(_to_expr(c))
    return out


def _project(b: Batch, exprs: List[Expr], ctx) -> Batch:
    cols: Dict[str, ColumnData] = {}
    for e in exprs:
        if isinstance(e, Star):
            for k, c in b.columns.items():
                cols[k] = c
            continue
        name = e.name()
        c = _fused.evaluate(e, b, ctx)
        if len(c) != b.n and b.n and len(c) == 1:
            c = c.take(torch.zeros(b.n, dtype=torch.long, device=b.device))
        cols[name] = c
    return Batch(cols, b.n, b.device)


def _local_partitions(parts: List[Batch]) -> List[Batch]:
    return [p for p in parts]


class DataFrameNaFunctions:
    def __init__(self, df):
        self.df = df

    def drop(self, how="any", thresh=None, subset=None):
        return self.df.dropna(how, thresh, subset)

    def fill(self, value, subset=None):
        return self.df.fillna(value, subset)

    def replace(self, to_replace, value=None, subset=None):
        return self.df.replace(to_replace, value, subset)


class DataFrameStatFunctions:
    def __init__(self, df):
        self.df = df

    def _column_moments(self, names) -> dict:
        """{name: (count, mean, M2, min, max)} over all partitions of all ranks (K20 + Chan merge)."""
        from ..ops import kernels as K
        session = self._session
        parts = self._plan.execute()
        k = len(names)
        locs = []
        for b in parts:
            if b.n == 0:
                continue
            cols = [b.columns[nm] for nm in names]
            X = torch.stack([c.values.double() for c in cols], 1)
            v = None
            if any(c.valid is not None for c in cols):
                v = torch.stack([c.valid_mask() for c in cols], 1)
            locs.append(K.col_moments(X, v))
        dev = session.device
        if locs:
            part = torch.stack(locs).to(dev)
        else:
            part = torch.zeros((1, k, 5), dtype=torch.float64, device=dev)
            part[..., 3], part[..., 4] = float("inf"), float("-inf")
        if session.comm.distributed:
            part = torch.cat(session.comm.all_gather_varlen(part.contiguous()))
        tot = K._merge_moments(part).cpu().numpy()
        return {nm: tuple(float(x) for x in tot[i]) for i, nm in enumerate(names)}

    def approxQuantile(self, col, probabilities, relativeError):
        return self.df.approxQuantile(col, probabilities, relativeError)

    def corr(self, a, b, method=None):
        return self.df.corr(a, b)

    def cov(self, a, b):
        return self.df.cov(a, b)


class _RDD:
    """The small slice of the RDD API the course touches."""

    def __init__(self, df):
        self.df = df

    def getNumPartitions(self) -> int:
        n = len(self.df._plan.execute())
        return int(self.df._session.comm.all_reduce_scalar(float(n)))

    def collect(self):
        return self.df.collect()

    def count(self):
        return self.df.count()

    def isEmpty(self):
        return self.df.count() == 0

    def map(self, f):
        return [f(r) for r in self.df.collect()]

    def flatMap(self, f):
        return [x for r in self.df.collect() for x in f(r)]

    def toDF(self, schema=None):
        return self.df


# ================================================================ DataFrame
class DataFrame:
    def __init__(self, plan: Plan, session):
        self._plan = plan
        self._session = session
        self.isStreaming = False

    # ------------------------------------------------------------ metadata
    @property
    def schema(self) -> T.StructType:
        return self._plan.schema()

    @property
    def columns(self) -> List[str]:
        return self.schema.names

    @property
    def dtypes(self):
        return [(f.name, f.dataType.simpleString()) for f in self.schema.fields]

    def printSchema(self):
        s = "root\n"
        for f in self.schema.fields:
            s += f" |-- {f.name}: {f.dataType.typeName() if not isinstance(f.dataType, T.VectorUDT) else 'vector'}" \
                 f" (nullable = {str(f.nullable).lower()})\n"
        if self._session.comm.rank == 0:
            print(s, end="")

    def explain(self, extended=False, mode=None):
        if self._session.comm.rank == 0:
            print("== Physical Plan ==\n" + self._plan.tree_string())

    @property
    def rdd(self):
        return _RDD(self)

    @property
    def na(self):
        return DataFrameNaFunctions(self)

    @property
    def stat(self):
        return DataFrameStatFunctions(self)

    @property
    def write(self):
        from .readwriter import DataFrameWriter
        return DataFrameWriter(self)

    @property
    def writeStream(self):
        from ..streaming.stream import DataStreamWriter
        return DataStreamWriter(self)

    def __getitem__(self, item):
        if isinstance(item, str):
            if item not in self.columns and item != "*":
                lower = {c.lower(): c for c in self.columns}
                if item.lower() not in lower:
                    raise AnalysisException(f"Column '{item}' does not exist. Available: {self.columns}")
            return Column(ColRef(item))
        if isinstance(item, Column):
            return self.filter(item)
        if isinstance(item, (list, tuple)):
            return self.select(*item)
        if isinstance(item, int):
            return Column(ColRef(self.columns[item]))
        raise TypeError(item)

    def __getattr__(self, item):
        if item.startswith("_"):
            raise AttributeError(item)
        if item in self.columns:
            return Column(ColRef(item))
        raise AttributeError(f"'DataFrame' object has no attribute '{item}'")

    def _new(self, plan: Plan) -> "DataFrame":
        return DataFrame(plan, self._session)

    def _map(self, name, fn) -> "DataFrame":
        return self._new(MapPlan(self._plan, name, fn))

    # --------------------------------------------------------- projections
    def select(self, *cols) -> "DataFrame":
        exprs = _expr_list(cols)
        if any(e.is_aggregate() for e in exprs):
            return self.agg(*[Column(e) for e in exprs])
        return self._map("Project [" + ", ".join(e.name() for e in exprs) + "]",
                         lambda b, ctx: _project(b, exprs, ctx))

    def selectExpr(self, *exprs) -> "DataFrame":
        from .parser import parse_expression
        return self.select(*[parse_expression(e) for e in exprs])

    def withColumn(self, name: str, col: Column) -> "DataFrame":
        e = col._expr if isinstance(col, Column) else _to_expr(col)
        if e.is_aggregate():
            raise AnalysisException("aggregate expressions are not allowed in withColumn")

        def fn(b, ctx):
            c = _fused.evaluate(e, b, ctx)
            return b.with_column(name, c)
        return self._map(f"Project [*, {e.name()} AS {name}]", fn)

    def withColumns(self, mapping: dict) -> "DataFrame":
        df = self
        for k, v in mapping.items():
            df = df.withColumn(k, v)
        return df

    def withColumnRenamed(self, old: str, new: str) -> "DataFrame":
        def fn(b, ctx):
            if old not in b.columns:
                return b
            return Batch({(new if k == old else k): c for k, c in b.columns.items()}, b.n, b.device)
        return self._map(f"Rename {old} -> {new}", fn)

    def toDF(self, *names) -> "DataFrame":
        def fn(b, ctx):
            return Batch({n: c for n, c in zip(names, b.columns.values())}, b.n, b.device)
        return self._map("ToDF", fn)

    def drop(self, *cols) -> "DataFrame":
        names = set()
        for c in cols:
            if isinstance(c, Column):
                names.add(c._expr.name())
            elif isinstance(c, (list, tuple)):
                names.update(c)
            else:
                names.add(c)

        def fn(b, ctx):
            return b.select([k for k in b.names if k not in names])
        return self._map(f"Drop {sorted(names)}", fn)

    def alias(self, name) -> "DataFrame":
        return self

    def transform(self, func, *args, **kwargs) -> "DataFrame":
        return func(self, *args, **kwargs)

    # ------------------------------------------------------------ filters
    def filter(self, cond) -> "DataFrame":
        if isinstance(cond, str):
            from .parser import parse_expression
            cond = parse_expression(cond)
        e = cond._expr

        def fn(b, ctx):
            c = _fused.evaluate(e, b, ctx)
            m = c.values.bool() & c.valid_mask() if c.valid is not None else c.values.bool()
            return b.filter(m)
        return self._map(f"Filter {e}", fn)

    where = filter

    def dropna(self, how="any", thresh=None, subset=None) -> "DataFrame":
        if isinstance(subset, str):
            subset = [subset]

        def fn(b, ctx):
            cols = subset or b.names
            ok = torch.zeros((b.n, len(cols)), dtype=torch.bool, device=b.device)
            for j, k in enumerate(cols):
                c = b.columns[k]
                v = c.valid_mask()
                if c.values.dim() == 1 and c.values.dtype.is_floating_point:
                    v = v & ~torch.isnan(c.values)
                ok[:, j] = v
            cnt = ok.sum(1)
            if thresh is not None:
                keep = cnt >= thresh
            elif how == "any":
                keep = cnt == len(cols)
            else:
                keep = cnt > 0
            return b.filter(keep)
        return self._map("DropNA", fn)

    def fillna(self, value, subset=None) -> "DataFrame":
        if isinstance(subset, str):
            subset = [subset]

        def fn(b, ctx):
            cols = dict(b.columns)
            items = value.items() if isinstance(value, dict) else [(k, value) for k in (subset or b.names)]
            for k, v in items:
                if k not in cols:
                    continue
                c = cols[k]
                isstr = isinstance(c.dtype, T.StringType)
                if isinstance(v, str) != isstr:
                    continue
                if isinstance(v, bool) != isinstance(c.dtype, T.BooleanType):
                    continue
                if isstr:
                    d = list(c.dictionary.tolist()) if c.dictionary is not None else []
                    if v not in d:
                        d.append(v)
                    uni = np.array(sorted(d), dtype=object)
                    from .batch import recode
                    c2 = recode(c, uni)
                    code = int(np.nonzero(uni == v)[0][0])
                    vals = torch.where(c2.valid_mask(), c2.values, torch.full_like(c2.values, code))
                    cols[k] = ColumnData(vals, c.dtype, None, uni, c.meta)
                    continue
                m = c.valid_mask()
                vals = c.values
                if vals.dtype.is_floating_point:
                    m = m & ~torch.isnan(vals)
                fillv = torch.full_like(vals, v if not isinstance(c.dtype, T.IntegralType) else int(v))
                cols[k] = ColumnData(torch.where(m, vals, fillv), c.dtype, None, c.dictionary, c.meta)
            return Batch(cols, b.n, b.device)
        return self._map("FillNA", fn)

    def replace(self, to_replace, value=None, subset=None) -> "DataFrame":
        mapping = to_replace if isinstance(to_replace, dict) else (
            dict(zip(to_replace, value if isinstance(value, (list, tuple)) else [value] * len(to_replace)))
            if isinstance(to_replace, (list, tuple)) else {to_replace: value})
        from .batch import map_dictionary

        def fn(b, ctx):
            cols = dict(b.columns)
            for k in (subset or b.names):
                c = cols[k]
                if isinstance(c.dtype, T.StringType):
                    smap = {a: v for a, v in mapping.items() if isinstance(a, str)}
                    if smap:
                        cols[k] = map_dictionary(c, lambda s: smap.get(s, s))
                elif c.values.dim() == 1 and not isinstance(c.dtype, T.BooleanType):
                    vals = c.values
                    for a, v in mapping.items():
                        if isinstance(a, (int, float)) and not isinstance(a, bool) and v is not None:
                            vals = torch.where(vals == a, torch.full_like(vals, v), vals)
                    cols[k] = ColumnData(vals, c.dtype, c.valid, c.dictionary, c.meta)
            return Batch(cols, b.n, b.device)
        return self._map("Replace", fn)

    # ------------------------------------------------------------ actions
    def _local(self) -> List[Batch]:
        return self._plan.execute()

    def _local_concat(self) -> Batch:
        parts = self._local()
        if not parts:
            return empty_batch(self.schema, self._session.device)
        return concat_batches(parts)

    def count(self) -> int:
        if self._plan.streamable:
            n = sum(b.n for b in self._plan.iter_execute())
        else:
            n = sum(b.n for b in self._local())
        return int(self._session.comm.all_reduce_scalar(float(n)))

    def foreachBatch(self, fn) -> None:
        """Call ``fn(batch)`` on each of this rank's device partitions, one at a time (streamed sources are
        never materialised: out-of-core batch inference writes or reduces each batch here)."""
        for b in self._plan.iter_execute():
            fn(b)

    def isEmpty(self) -> bool:
        return self.count() == 0

    def toPandas(self) -> pd.DataFrame:
        local = self._local_concat().to_pandas()
        comm = self._session.comm
        if comm.distributed:
            parts = comm.all_gather_object(local)
            local = pd.concat(parts, ignore_index=True)
        if local.shape[1] == 0 and len(self.columns):
            local = pd.DataFrame(columns=self.columns)
        return local

    def collect(self) -> List[T.Row]:
        b = self._local_concat()
        names = list(self.columns)
        cols = [b.columns[c].to_pylist() for c in names]
        if self._session.comm.distributed:
            parts = self._session.comm.all_gather_object(cols)
            cols = [sum((p[i] for p in parts), []) for i in range(len(names))]
        cols = [[v.item() if isinstance(v, np.generic) else v for v in c] for c in cols]
        return [T.Row._make(names, vals) for vals in zip(*cols)] if names else []

    @staticmethod
    def _py_column(s: pd.Series):
        out = []
        for v in s.tolist():
            if isinstance(v, float) and np.isnan(v):
                out.append(float("nan"))
            elif isinstance(v, np.generic):
                out.append(v.item())
            else:
                out.append(v)
        return out

    def toLocalIterator(self):
        return iter(self.collect())

    def take(self, n: int) -> List[T.Row]:
        return self.limit(n).collect()

    def head(self, n: Optional[int] = None):
        if n is None:
            rows = self.take(1)
            return rows[0] if rows else None
        return self.take(n)

    def first(self):
        return self.head()

    def tail(self, n: int):
        rows = self.collect()
        return rows[-n:] if n else []

    def show(self, n: int = 20, truncate: Union[bool, int] = True, vertical: bool = False):
        pdf = self.limit(n).toPandas()
        if self._session.comm.rank != 0:
            return
        width = 20 if truncate is True else (int(truncate) if truncate else 0)

        def fmt(v):
            if v is None or (isinstance(v, float) and np.isnan(v) and False):
                return "null"
            if isinstance(v, bool):
                s = "true" if v else "false"
            elif isinstance(v, float):
                s = repr(v) if v == v else "NaN"
            else:
                s = str(v)
            if width and len(s) > width:
                s = s[: width - 3] + "..."
            return s
        cols = list(pdf.columns)
        rows = [[fmt(v) for v in r] for r in pdf.itertuples(index=False)]
        ws = [max([len(c)] + [len(r[i]) for r in rows]) for i, c in enumerate(cols)]
        sep = "+" + "+".join("-" * w for w in ws) + "+"
        print(sep)
        print("|" + "|".join(c.rjust(w) for c, w in zip(cols, ws)) + "|")
        print(sep)
        for r in rows:
            print("|" + "|".join(v.rjust(w) for v, w in zip(r, ws)) + "|")
        print(sep)

    def display(self):
        self.show()

    def foreach(self, f):
        for r in self.collect():
            f(r)

    # ---------------------------------------------------------- caching
    def cache(self) -> "DataFrame":
        self._plan.cached = True
        return self

    def persist(self, storageLevel=None) -> "DataFrame":
        return self.cache()

    def unpersist(self, blocking=False) -> "DataFrame":
        self._plan.cached = False
        self._plan._result = None
        return self

    @property
    def is_cached(self):
        return self._plan.cached

    def checkpoint(self, eager=True) -> "DataFrame":
        parts = self._local()
        schema = self.schema
        return self._new(SourcePlan(self._session, "Checkpoint", lambda: parts, schema))

    localCheckpoint = checkpoint

    # ------------------------------------------------------ partitioning
    def repartition(self, numPartitions=None, *cols) -> "DataFrame":
        if isinstance(numPartitions, (str, Column)):
            cols = (numPartitions,) + cols
            numPartitions = None
        P = numPartitions or int(self._session.conf.get("spark.sql.shuffle.partitions"))
        keys = [c if isinstance(c, str) else c._expr.name() for c in cols]
        session = self._session

        def fn(parts):
            return _shuffle(session, parts, P, keys or None)
        return self._new(PartitionsPlan(session, f"Exchange RoundRobin({P})" if not keys else
                                        f"Exchange hashpartitioning({keys}, {P})", [self._plan], fn, lambda s: s))

    def coalesce(self, numPartitions: int) -> "DataFrame":
        session = self._session

        def fn(parts):
            comm = session.comm
            W = comm.world_size
            if W > 1 and numPartitions < W:
                # move everything to the first numPartitions ranks
                b = concat_batches(parts) if parts else empty_batch(self.schema, session.device)
                from ..parallel.shuffle import exchange
                dest = torch.full((b.n,), comm.rank % numPartitions, dtype=torch.long, device=b.device)
                got = exchange(comm, b, dest)
                return [got] if comm.rank < numPartitions else []
            local_target = max(1, numPartitions // W + (1 if comm.rank < numPartitions % W else 0))
            if len(parts) <= local_target:
                return parts
            groups = np.array_split(np.arange(len(parts)), local_target)
            return [concat_batches([parts[i] for i in g]) for g in groups if len(g)]
        return self._new(PartitionsPlan(session, f"Coalesce {numPartitions}", [self._plan], fn, lambda s: s))

    def sortWithinPartitions(self, *cols, **kw) -> "DataFrame":
        orders = self._sort_orders(cols, kw.get("ascending", True))

        def fn(b, ctx):
            return b.take(R.sort_indices(b, [(o.x.eval(b, ctx), o.ascending, o.nulls_first) for o in orders]))
        return self._map("SortWithinPartitions", fn)

    # -------------------------------------------------------- sampling
    def limit(self, num: int) -> "DataFrame":
        session = self._session

        def fn(parts):
            comm = session.comm
            local = sum(p.n for p in parts)
            counts = comm.all_gather_object(local) if comm.distributed else [local]
            before = sum(counts[: comm.rank])
            quota = max(0, min(local, num - before))
            out = []
            for p in parts:
                if quota <= 0:
                    break
                take = min(quota, p.n)
                out.append(p.slice(0, take))
                quota -= take
            return out
        return self._new(PartitionsPlan(session, f"GlobalLimit {num}", [self._plan], fn, lambda s: s))

    def sample(self, withReplacement=None, fraction=None, seed=None) -> "DataFrame":
        if isinstance(withReplacement, float) and fraction is None:
            withReplacement, fraction = False, withReplacement
        elif isinstance(withReplacement, float):
            withReplacement, fraction, seed = False, withReplacement, fraction
        if seed is None:
            seed = int(np.random.SeedSequence().entropy % (2 ** 62))
        from ..ops import kernels as K

        def fn(b, ctx):
            u = K.uniform(b.n, seed, (ctx.partition_index << 40), 7, device=b.device)
            if withReplacement:
                from ..ops.philox import poisson_from_uniform
                k = torch.from_numpy(poisson_from_uniform(u.cpu().numpy(), fraction)).to(b.device)
                return b.take(torch.arange(b.n, device=b.device).repeat_interleave(k))
            return b.filter(u < fraction)
        return self._map(f"Sample {fraction}", fn)

    def _with_global_uniform(self, seed: int, name: str) -> "DataFrame":
        """Attach a Philox uniform keyed by GLOBAL row id (partition-count invariant)."""
        session = self._session
        from ..ops import kernels as K

        def fn(parts):
            comm = session.comm
            local = sum(p.n for p in parts)
            counts = comm.all_gather_object(local) if comm.distributed else [local]
            off = sum(counts[: comm.rank])
            out = []
            for p in parts:
                u = K.uniform(p.n, seed, off, 11, device=p.device)
                off += p.n
                out.append(p.with_column(name, ColumnData(u, T.DoubleType())))
            return out

        def sfn(s):
            return T.StructType(s.fields + [T.StructField(name, T.DoubleType())])
        return self._new(PartitionsPlan(session, "AttachRowUniform", [self._plan], fn, sfn))

    def _with_sequence_id(self, name: str) -> "DataFrame":
        """Attach a consecutive 0..N-1 int64 id in global row order (one counts all-gather)."""
        session = self._session

        def fn(parts):
            comm = session.comm
            local = sum(p.n for p in parts)
            counts = comm.all_gather_object(local) if comm.distributed else [local]
            off = sum(counts[: comm.rank])
            out = []
            for p in parts:
                ids = torch.arange(off, off + p.n, dtype=torch.int64, device=p.device)
                off += p.n
                out.append(p.with_column(name, ColumnData(ids, T.LongType())))
            return out

        def sfn(s):
            return T.StructType(s.fields + [T.StructField(name, T.LongType(), False)])
        return self._new(PartitionsPlan(session, "AttachSequenceId", [self._plan], fn, sfn))

    def randomSplit(self, weights: List[float], seed: Optional[int] = None) -> List["DataFrame"]:
        """Split by Philox(seed, global row id): independent of the GPU count.

        (Spark's split depends on partitioning — ML 02:34-52 demonstrates this;
        we deliberately make it invariant)
        """
        if seed is None:
            seed = int(np.random.SeedSequence().entropy % (2 ** 62))
        tot = float(sum(weights))
        bounds = np.cumsum([0.0] + [w / tot for w in weights])
        base = self._with_global_uniform(seed, "__u").cache()
        outs = []
        for i in range(len(weights)):
            lo, hi = float(bounds[i]), float(bounds[i + 1])
            hi_inc = i == len(weights) - 1
            col = Column(ColRef("__u"))
            cond = (col >= lo) & ((col <= hi) if hi_inc else (col < hi))
            outs.append(base.filter(cond).drop("__u"))
        return outs

    # ---------------------------------------------------------- set ops
    def union(self, other: "DataFrame") -> "DataFrame":
        session = self._session

        def fn(a, b):
            names = self.columns
            conv = []
            for p in b:
                cols = {}
                for k_new, (k_old, c) in zip(names, p.columns.items()):
                    cols[k_new] = c
                conv.append(Batch(cols, p.n, p.device))
            return list(a) + conv
        return self._new(PartitionsPlan(session, "Union", [self._plan, other._plan], fn, lambda s1, s2: s1))

    unionAll = union

    def unionByName(self, other: "DataFrame", allowMissingColumns=False) -> "DataFrame":
        names = self.columns
        if allowMissingColumns:
            from .functions import lit
            a, b = self, other
            for c in other.columns:
                if c not in names:
                    a = a.withColumn(c, lit(None).cast(other.schema[c].dataType))
            for c in names:
                if c not in other.columns:
                    b = b.withColumn(c, lit(None).cast(self.schema[c].dataType))
            return a.union(b.select(*a.columns))
        return self.union(other.select(*names))

    def distinct(self) -> "DataFrame":
        return self.dropDuplicates()

    def dropDuplicates(self, subset: Optional[List[str]] = None) -> "DataFrame":
        session = self._session
        if isinstance(subset, str):
            subset = [subset]

        def fn(parts):
            keys = subset or (parts[0].names if parts else self.columns)
            P = int(session.conf.get("spark.sql.shuffle.partitions"))
            if session.device.type == "cuda" and parts:
                # K16: route rows as _shuffle does, then keep every key's first row in the device hash table
                comm = session.comm
                b = _route(session, concat_batches(parts), P, keys)
                nloc = len([p for p in range(P) if p % comm.world_size == comm.rank])
                out = R.dedup_partitions(b, keys, nloc)
                if out is not None:
                    return out
                from ..parallel.shuffle import hash_keys
                shuffled = _split_local(session, b, hash_keys(b, keys) % P, P)
            else:
                shuffled = _shuffle(session, parts, P, keys)
            return [p.take(R.dedup_indices(p, keys)) for p in shuffled]
        return self._new(PartitionsPlan(session, f"HashAggregate(dedup {subset})", [self._plan], fn, lambda s: s))

    drop_duplicates = dropDuplicates

    def intersect(self, other):
        return self.join(other, on=self.columns, how="semi").distinct()

    def subtract(self, other):
        return self.join(other, on=self.columns, how="anti").distinct()

    exceptAll = subtract

    # ------------------------------------------------------------ sorting
    def _sort_orders(self, cols, ascending) -> List[SortOrder]:
        flat = []
        for c in cols:
            if isinstance(c, (list, tuple)):
                flat.extend(c)
            else:
                flat.append(c)
        if isinstance(ascending, (list, tuple)):
            asc = list(ascending)
        else:
            asc = [ascending] * len(flat)
        orders = []
        for c, a in zip(flat, asc):
            e = ColRef(c) if isinstance(c, str) else c._expr
            if isinstance(e, SortOrder):
                orders.append(e)
            else:
                orders.append(SortOrder(e, bool(a)))
        return orders

    def orderBy(self, *cols, **kw) -> "DataFrame":
        orders = self._sort_orders(cols, kw.get("ascending", True))
        session = self._session

        def fn(parts):
            comm = session.comm
            b = concat_batches(parts) if parts else empty_batch(self.schema, session.device)
            ctx = EvalContext(session)
            if comm.distributed:
                b = _range_shuffle(session, b, orders[0])
            perm = R.sort_indices(b, [(o.x.eval(b, ctx), o.ascending, o.nulls_first) for o in orders])
            return [b.take(perm)]
        return self._new(PartitionsPlan(session, "Sort [" + ", ".join(map(str, orders)) + "]", [self._plan], fn,
                                        lambda s: s))

    sort = orderBy

    # ------------------------------------------------------------ grouping
    def groupBy(self, *cols):
        from .group import GroupedData
        keys = []
        for c in cols:
            if isinstance(c, (list, tuple)):
                keys.extend(c)
            else:
                keys.append(c)
        return GroupedData(self, keys)

    groupby = groupBy

    def agg(self, *exprs):
        return self.groupBy().agg(*exprs)

    def join(self, other: "DataFrame", on=None, how: str = "inner") -> "DataFrame":
        session = self._session
        how = how or "inner"
        if on is None:
            return self.crossJoin(other)
        lkeys: List[str]
        rkeys: List[str]
        cond_expr = None
        if isinstance(on, str):
            lkeys = rkeys = [on]
        elif isinstance(on, (list, tuple)) and all(isinstance(x, str) for x in on):
            lkeys = rkeys = list(on)
        else:
            conds = on if isinstance(on, (list, tuple)) else [on]
            lkeys, rkeys = [], []
            for c in conds:
                e = c._expr
                from .column import BinOp
                if isinstance(e, BinOp) and e.op == "==" and isinstance(e.l, ColRef) and isinstance(e.r, ColRef):
                    a, b = e.l.col_name, e.r.col_name
                    a = a.split(".", 1)[-1]
                    b = b.split(".", 1)[-1]
                    if a in self.columns and b in other.columns:
                        lkeys.append(a)
                        rkeys.append(b)
                    else:
                        lkeys.append(b)
                        rkeys.append(a)
                else:
                    raise AnalysisException("only equi-join conditions are supported")
            cond_expr = True
        drop_right = cond_expr is None

        def fn(lp, rp):
            P = int(session.conf.get("spark.sql.shuffle.partitions"))
            comm = session.comm
            lb = concat_batches(lp) if lp else empty_batch(self.schema, session.device)
            rb = concat_batches(rp) if rp else empty_batch(other.schema, session.device)
            if comm.distributed:
                from ..parallel.shuffle import exchange, hash_keys, unify_global_dictionaries
                lb = unify_global_dictionaries(comm, lb)
                rb = unify_global_dictionaries(comm, rb)
                lb = exchange(comm, lb, hash_keys(lb, lkeys) % comm.world_size)
                rb = exchange(comm, rb, hash_keys(rb, rkeys) % comm.world_size)
            return [R.join(lb, rb, lkeys, rkeys, how, drop_right_keys=drop_right)]

        def sfn(ls, rs):
            lb = empty_batch(ls, torch.device("cpu"))
            rb = empty_batch(rs, torch.device("cpu"))
            return R.join(lb, rb, lkeys, rkeys, how, drop_right_keys=drop_right).schema()
        return self._new(PartitionsPlan(session, f"Join {how} {lkeys}={rkeys}", [self._plan, other._plan], fn, sfn))

    def crossJoin(self, other: "DataFrame") -> "DataFrame":
        session = self._session

        def fn(lp, rp):
            lb = concat_batches(lp) if lp else empty_batch(self.schema, session.device)
            rall = other.toPandas()
            from .batch import batch_from_pandas
            rb = batch_from_pandas(rall, other.schema, session.device)
            return [R.join(lb, rb, [], [], "cross", drop_right_keys=False)]

        def sfn(ls, rs):
            return T.StructType(ls.fields + [f for f in rs.fields])
        return self._new(PartitionsPlan(session, "CartesianProduct", [self._plan, other._plan], fn, sfn))

    # ------------------------------------------------------------ statistics
    def describe(self, *cols) -> "DataFrame":
        return self._summary(["count", "mean", "stddev", "min", "max"], cols)

    def summary(self, *statistics) -> "DataFrame":
        stats = list(statistics) or ["count", "mean", "stddev", "min", "25%", "50%", "75%", "max"]
        return self._summary(stats, ())

    def _summary(self, stats, cols) -> "DataFrame":
        from . import functions as F
        flat = []
        for c in cols:
            flat.extend(c if isinstance(c, (list, tuple)) else [c])
        fields = [f for f in self.schema.fields
                  if (not flat or f.name in flat) and (f.dataType.is_numeric or isinstance(f.dataType, T.StringType))]
        rows = {s: [] for s in stats}
        # count / mean / stddev / min / max of every numeric column: one K20 pass (col_moments) per local
        # partition, per-rank partials merged with Chan's formula (one all-gather), instead of one
        # aggregation job per column
        moment_stats = {"count", "mean", "stddev", "min", "max"}
        num_fields = [f for f in fields if f.dataType.is_numeric and not isinstance(f.dataType, T.BooleanType)]
        mom = self._column_moments([f.name for f in num_fields]) if num_fields and \
            any(s in moment_stats for s in stats) else {}
        for f in fields:
            c = F.col(f.name)
            is_str = isinstance(f.dataType, T.StringType)
            aggs = []
            for s in stats:
                if f.name in mom and s in moment_stats:
                    aggs.append(None)
                elif s == "count":
                    aggs.append(F.count(c))
                elif s == "mean":
                    aggs.append(F.avg(c) if not is_str else None)
                elif s == "stddev":
                    aggs.append(F.stddev(c) if not is_str else None)
                elif s in ("min", "max"):
                    aggs.append(F.min(c) if s == "min" else F.max(c))
                elif s.endswith("%"):
                    aggs.append(F.percentile_approx(c, float(s[:-1]) / 100.0) if not is_str else None)
                else:
                    raise ValueError(s)
            live = [(i, a) for i, a in enumerate(aggs) if a is not None]
            got = self.agg(*[a.alias(f"_s{i}") for i, a in live]).collect()[0] if live else []
            vals = [None] * len(aggs)
            for (i, _), v in zip(live, got):
                vals[i] = v
            if f.name in mom:
                cnt, mean, m2, mn, mx = mom[f.name]
                integral = isinstance(f.dataType, (T.IntegerType, T.LongType, T.ShortType, T.ByteType))
                for i, s in enumerate(stats):
                    if s == "count":
                        vals[i] = int(cnt)
                    elif cnt == 0:
                        vals[i] = None
                    elif s == "mean":
                        vals[i] = mean
                    elif s == "stddev":
                        vals[i] = math.sqrt(m2 / (cnt - 1)) if cnt > 1 else float("nan")
                    elif s in ("min", "max"):
                        v = mn if s == "min" else mx
                        vals[i] = int(v) if (integral and math.isfinite(v)) else v
            for s, v in zip(stats, vals):
                rows[s].append(None if v is None else (str(int(v)) if s == "count" else _num_str(v)))
        pdf = pd.DataFrame({"summary": stats, **{f.name: [rows[s][i] for s in stats] for i, f in enumerate(fields)}})
        return self._session.createDataFrame(pdf, schema=T.StructType(
            [T.StructField("summary", T.StringType())] + [T.StructField(f.name, T.StringType()) for f in fields]))

    def _column_moments(self, names) -> dict:
        """{name: (count, mean, M2, min, max)} over all partitions of all ranks (K20 + Chan merge)."""
        from ..ops import kernels as K
        session = self._session
        parts = self._plan.execute()
        k = len(names)
        locs = []
        for b in parts:
            if b.n == 0:
                continue
            cols = [b.columns[nm] for nm in names]
            X = torch.stack([c.values.double() for c in cols], 1)
            v = None
            if any(c.valid is not None for c in cols):
                v = torch.stack([c.valid_mask() for c in cols], 1)
            locs.append(K.col_moments(X, v))
        dev = session.device
        if locs:
            part = torch.stack(locs).to(dev)
        else:
            part = torch.zeros((1, k, 5), dtype=torch.float64, device=dev)
            part[..., 3], part[..., 4] = float("inf"), float("-inf")
        if session.comm.distributed:
            part = torch.cat(session.comm.all_gather_varlen(part.contiguous()))
        tot = K._merge_moments(part).cpu().numpy()
        return {nm: tuple(float(x) for x in tot[i]) for i, nm in enumerate(names)}

    def approxQuantile(self, col, probabilities, relativeError):
        """Exact quantiles (relativeError = 0 semantics, which satisfies any bound)."""
        if isinstance(col, (list, tuple)):
            return [self.approxQuantile(c, probabilities, relativeError) for c in col]
        from . import functions as F
        if not probabilities:
            return []
        sel = self.select(F.col(col).cast("double").alias("__q")).dropna()
        v = sel.agg(F.percentile_approx(F.col("__q"), list(probabilities)).alias("q")).collect()
        q = v[0][0]
        if q is None:
            return []
        return [float(x) for x in (q.toArray() if hasattr(q, "toArray") else q)]

    def corr(self, a, b, method=None) -> float:
        from . import functions as F
        r = self.select(F.col(a).cast("double").alias("a"), F.col(b).cast("double").alias("b")).dropna()
        s = r.agg(F.avg("a"), F.avg("b"), F.stddev_pop("a"), F.stddev_pop("b"),
                  F.avg(F.col("a") * F.col("b"))).collect()[0]
        return (s[4] - s[0] * s[1]) / (s[2] * s[3])

    def cov(self, a, b) -> float:
        from . import functions as F
        r = self.select(F.col(a).cast("double").alias("a"), F.col(b).cast("double").alias("b")).dropna()
        s = r.agg(F.avg("a"), F.avg("b"), F.avg(F.col("a") * F.col("b")), F.count("a")).collect()[0]
        n = s[3]
        return (s[2] - s[0] * s[1]) * n / (n - 1)

    # ------------------------------------------------------------ SQL views
    def createOrReplaceTempView(self, name: str):
        self._session.catalog._register_temp(name, self)

    createTempView = createOrReplaceTempView
    registerTempTable = createOrReplaceTempView

    def createOrReplaceGlobalTempView(self, name: str):
        self._session.catalog._register_temp("global_temp." + name, self)

    # ------------------------------------------------------------ pandas bridge
    def mapInPandas(self, func, schema) -> "DataFrame":
        from .udf import map_in_pandas
        return map_in_pandas(self, func, schema)

    def pandas_api(self, index_col=None):
        from ..pandas_api.frame import from_spark
        return from_spark(self, index_col)

    to_pandas_on_spark = pandas_api
    to_koalas = pandas_api

    def inputFiles(self):
        return list(getattr(self._plan, "files", []))

    def __repr__(self):
        return "DataFrame[" + ", ".join(f"{n}: {t}" for n, t in self.dtypes) + "]"


def _num_str(v):
    if isinstance(v, float):
        if v == int(v) and abs(v) < 1e16:
            return str(v)
        return repr(v)
    return str(v)


# ==================================================================== shuffles
def _route(session, b: Batch, P: int, keys: List[str]) -> Batch:
    """Send every row to the rank that owns its hash partition (partition p lives on rank p % W)."""
    comm = session.comm
    if not comm.distributed:
        return b
    from ..parallel.shuffle import exchange, hash_keys, unify_global_dictionaries
    b = unify_global_dictionaries(comm, b)
    return exchange(comm, b, (hash_keys(b, keys) % P) % comm.world_size)


def _split_local(session, b: Batch, pid: torch.Tensor, P: int) -> List[Batch]:
    """This rank's partitions (p % W == rank) of rows already routed here, rows in order within a partition."""
    comm = session.comm
    W, rank = comm.world_size, comm.rank
    order = torch.argsort(pid, stable=True)
    b = b.take(order)
    pid = pid[order]
    mine = [p for p in range(P) if p % W == rank]
    bounds = torch.searchsorted(pid, torch.tensor(mine + [P], device=pid.device).clamp(max=P)).cpu().tolist()
    return [b.slice(bounds[i], bounds[i + 1]) for i in range(len(mine))]


def _shuffle(session, parts: List[Batch], P: int, keys: Optional[List[str]]) -> List[Batch]:
    """Redistribute rows into P global partitions (partition p lives on rank p % W)."""
    comm = session.comm
    W, rank = comm.world_size, comm.rank
    if not parts:
        parts = []
    b = concat_batches(parts) if parts else None
    if b is None:
        return []
    if P == 1 and not comm.distributed:
        return [b]
    if keys:
        from ..parallel.shuffle import hash_keys, unify_global_dictionaries
        if comm.distributed:
            b = unify_global_dictionaries(comm, b)
        pid = hash_keys(b, keys) % P
    else:
        # round-robin by global row id
        local = b.n
        counts = comm.all_gather_object(local) if comm.distributed else [local]
        off = sum(counts[:rank])
        pid = (torch.arange(b.n, device=b.device) + off) % P
    if comm.distributed:
        from ..parallel.shuffle import exchange
        b = b.with_column("__pid", ColumnData(pid.to(torch.int32), T.IntegerType()))
        b = exchange(comm, b, pid % W)
        pid = b.columns["__pid"].values.long()
        b = b.select([k for k in b.names if k != "__pid"])
    out = []
    order = torch.argsort(pid, stable=True)
    b = b.take(order)
    pid = pid[order]
    mine = [p for p in range(P) if p % W == rank]
    bounds = torch.searchsorted(pid, torch.tensor(mine + [P], device=pid.device).clamp(max=P))
    bounds = bounds.cpu().tolist()
    for i in range(len(mine)):
        out.append(b.slice(bounds[i], bounds[i + 1]))
    return out


def _range_shuffle(session, b: Batch, order: SortOrder) -> Batch:
    """Sample-sort range partitioning on the leading sort key."""
    comm = session.comm
    W = comm.world_size
    from ..parallel.shuffle import exchange, unify_global_dictionaries
    b = unify_global_dictionaries(comm, b)
    c = order.x.eval(b, EvalContext(session))
    key = c.values.to(torch.float64) if c.values.dim() == 1 else c.values[:, 0].double()
    key = torch.where(c.valid_mask(), key, torch.full_like(key, float("-inf") if order.nulls_first else
                                                           float("inf")))
    if not order.ascending:
        key = -key
    k = min(b.n, 256)
    samp = key[torch.randperm(b.n, device=key.device)[:k]] if b.n else key[:0]
    allsamp = torch.cat(comm.all_gather_varlen(samp)).sort().values
    if allsamp.numel() == 0:
        return b
    qs = torch.linspace(0, allsamp.numel() - 1, W + 1, device=allsamp.device)[1:-1].long()
    splitters = allsamp[qs]
    dest = torch.searchsorted(splitters, key, right=True)
    return exchange(comm, b, dest)
