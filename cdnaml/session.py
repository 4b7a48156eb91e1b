"""SparkSession-compatible entry point.

One session per process.  Under ``torchrun`` each process owns one GPU
(``cuda:LOCAL_RANK``) and the session's communicator spans all ranks over
RCCL/xGMI; standalone it is a one-GPU (or CPU) job.  Configuration keys use
Spark's dotted names (``spark.sql.shuffle.partitions``, Labs/ML 00L:79-80;
``spark.sql.execution.arrow.maxRecordsPerBatch``, ML 12:90;
``spark.databricks.delta.retentionDurationCheck.enabled``, ML 00c:235) and
can be overridden with ``CDNAML_<KEY>`` environment variables.
"""
from __future__ import annotations

import os
import threading
from typing import List, Optional

import numpy as np
import pandas as pd
import torch

from .parallel.comm import Comm, init_from_env
from .sql import types as T
from .sql.batch import Batch, batch_from_pandas, column_from_numpy, empty_batch
from .sql.dataframe import DataFrame, SourcePlan

_DEFAULT_CONF = {
    "spark.app.name": "cdnaml",
    "spark.master": "local[*]",
    "spark.sql.shuffle.partitions": "8",
    "spark.sql.execution.arrow.maxRecordsPerBatch": "10000",
    "spark.sql.execution.arrow.pyspark.enabled": "true",
    "spark.sql.adaptive.enabled": "true",
    "spark.databricks.delta.retentionDurationCheck.enabled": "true",
    "spark.default.parallelism": "0",
    "cdnaml.warehouse.dir": "spark-warehouse",
    "cdnaml.deterministic": "false",
}


_UNSET = object()


class RuntimeConfig:
    def __init__(self, initial=None):
        self._d = dict(_DEFAULT_CONF)
        for k, v in os.environ.items():
            if k.startswith("CDNAML_CONF_"):
                self._d[k[len("CDNAML_CONF_"):].lower().replace("__", ".")] = v
        if initial:
            self._d.update({k: str(v) for k, v in initial.items()})

    def set(self, key, value):
        self._d[key] = str(value).lower() if isinstance(value, bool) else str(value)

    def get(self, key, default=_UNSET):
        """Like ``spark.conf.get``: an unset key raises unless a default (``None`` included) is given."""
        if key in self._d:
            return self._d[key]
        if default is not _UNSET:
            return default
        raise KeyError(f"conf {key} is not set")

    def unset(self, key):
        self._d.pop(key, None)

    def getAll(self):
        return dict(self._d)

    def isModifiable(self, key):
        return True


class SparkContext:
    def __init__(self, session):
        self._session = session
        self.appName = session.conf.get("spark.app.name")

    @property
    def defaultParallelism(self) -> int:
        v = int(self._session.conf.get("spark.default.parallelism"))
        return v if v > 0 else max(1, self._session.comm.world_size)

    def setLogLevel(self, level):
        pass

    def setCheckpointDir(self, dirName: str) -> None:
        """Directory for iterative-fit checkpoints (GBT / XGBoost every `checkpointInterval` rounds)."""
        import os
        os.makedirs(dirName, exist_ok=True)
        self._session.conf.set("cdnaml.checkpoint.dir", dirName)

    def getCheckpointDir(self):
        return self._session.conf.getAll().get("cdnaml.checkpoint.dir")

    def parallelize(self, data, numSlices=None):
        return self._session.createDataFrame([(x,) if not isinstance(x, (tuple, list)) else x for x in data])

    def emptyRDD(self):
        return []

    @property
    def _jvm(self):
        raise RuntimeError("no JVM: cdnaml is a native engine")


class _Builder:
    def __init__(self):
        self._conf = {}

    def appName(self, name):
        self._conf["spark.app.name"] = name
        return self

    def master(self, m):
        self._conf["spark.master"] = m
        return self

    def config(self, key=None, value=None, conf=None):
        if isinstance(key, dict):
            self._conf.update(key)
        elif key is not None:
            self._conf[key] = value
        return self

    def enableHiveSupport(self):
        return self

    def getOrCreate(self) -> "SparkSession":
        with SparkSession._lock:
            s = SparkSession._active
            if s is None or s._stopped:
                s = SparkSession(self._conf)
            else:
                for k, v in self._conf.items():
                    s.conf.set(k, v)
            return s


def _freeze_startup_objects() -> None:
    """Move every object alive at session start (torch's, numpy's, the framework's own modules: hundreds of
    thousands of containers) to the collector's permanent generation.  A full collection otherwise walks all of
    them: 65-80 ms pauses inside one in four or five deep-forest fits (`scripts/deep_reg_probe.py`: 102 / 115 ms
    fits among 37 ms ones, none with the collector off).  Objects created later are collected as usual.
    CDNAML_GC_FREEZE=0 leaves the collector alone."""
    if os.environ.get("CDNAML_GC_FREEZE", "1") == "0":
        return
    import gc
    gc.collect()
    gc.freeze()


class SparkSession:
    _active: Optional["SparkSession"] = None
    _lock = threading.Lock()

    class _BuilderDescriptor:
        def __get__(self, obj, cls):
            return _Builder()

    builder = _BuilderDescriptor()

    def __init__(self, conf=None):
        self.conf = RuntimeConfig(conf)
        use_gpu = torch.cuda.is_available() and os.environ.get("CDNAML_DEVICE", "") != "cpu"
        init_from_env("cuda" if use_gpu else "cpu")
        if use_gpu:
            from .parallel.comm import rank_device_index
            self.device = torch.device("cuda", rank_device_index())
            torch.cuda.set_device(self.device)
        else:
            self.device = torch.device("cpu")
        self.comm = Comm(self.device)
        self.sparkContext = SparkContext(self)
        from .catalog import Catalog
        self.catalog = Catalog(self)
        from .streaming.stream import StreamingQueryManager
        self.streams = StreamingQueryManager(self)
        self._stopped = False
        self.version = "3.3.0-cdnaml"
        SparkSession._active = self
        _freeze_startup_objects()

    @classmethod
    def getActiveSession(cls):
        return cls._active

    @property
    def read(self):
        from .sql.readwriter import DataFrameReader
        return DataFrameReader(self)

    @property
    def readStream(self):
        from .streaming.stream import DataStreamReader
        return DataStreamReader(self)

    @property
    def udf(self):
        from .sql.functions import udf

        class _Reg:
            def register(_, name, f, returnType=None):
                u = udf(f, returnType or T.StringType())
                self.catalog._functions[name.lower()] = u
                return u
        return _Reg()

    def newSession(self):
        return self

    def stop(self):
        self._stopped = True
        if SparkSession._active is self:
            SparkSession._active = None

    # ------------------------------------------------------------ creation
    def _from_local_batches(self, name, batches_fn, schema) -> DataFrame:
        return DataFrame(SourcePlan(self, name, batches_fn, schema), self)

    def _rank_slice(self, n: int):
        W, r = self.comm.world_size, self.comm.rank
        a = n * r // W
        b = n * (r + 1) // W
        return a, b

    def range(self, start, end=None, step=1, numPartitions=None) -> DataFrame:
        if end is None:
            start, end = 0, start
        total = max(0, (end - start + (step - (1 if step > 0 else -1))) // step)
        P = numPartitions or self.sparkContext.defaultParallelism
        dev = self.device
        W, rank = self.comm.world_size, self.comm.rank

        def fn():
            out = []
            for p in range(P):
                if p % W != rank:
                    continue
                a, b = total * p // P, total * (p + 1) // P
                ids = torch.arange(a, b, dtype=torch.int64, device=dev) * step + start
                out.append(Batch({"id": _long_col(ids)}, b - a, dev))
            return out
        return self._from_local_batches(f"Range ({start}, {end}, step={step}, splits={P})", fn,
                                        T.StructType([T.StructField("id", T.LongType(), False)]))

    def createDataFrame(self, data, schema=None, samplingRatio=None, verifySchema=True) -> DataFrame:
        dev = self.device
        names = None
        if isinstance(schema, (list, tuple)) and all(isinstance(s, str) for s in schema):
            names, schema = list(schema), None
        elif isinstance(schema, str):
            schema = T.to_schema(schema) if ("," in schema or " " in schema.strip() or ":" in schema) else \
                T.StructType([T.StructField("value", T.to_type(schema))])
        if isinstance(data, DataFrame):
            return data
        if hasattr(data, "to_pandas") and not isinstance(data, pd.DataFrame):  # pyarrow / pandas-api
            data = data.to_pandas()
        if isinstance(data, pd.DataFrame):
            pdf = data.reset_index(drop=True)
            if names:
                pdf.columns = names
        else:
            rows = list(data)
            if rows and isinstance(rows[0], T.Row) and rows[0].__fields__:
                cols = names or rows[0].__fields__
                pdf = pd.DataFrame([tuple(r) for r in rows], columns=cols)
            elif rows and isinstance(rows[0], dict):
                pdf = pd.DataFrame(rows)
            elif rows and not isinstance(rows[0], (tuple, list)):
                pdf = pd.DataFrame({(names or (schema.names if schema is not None else ["value"]))[0]: rows})
            else:
                cols = names or (schema.names if schema is not None else [f"_{i + 1}" for i in
                                                                          range(len(rows[0]) if rows else 0)])
                pdf = pd.DataFrame([tuple(r) for r in rows], columns=cols)
        if schema is None:
            probe = batch_from_pandas(pdf.head(0) if len(pdf) == 0 else pdf.iloc[:min(len(pdf), 1000)], None,
                                      torch.device("cpu"))
            schema = probe.schema()
            # infer on the whole frame for object columns with leading nulls
            fields = []
            for f in schema.fields:
                s = pdf[f.name]
                if s.dtype == object:
                    from .sql.batch import _infer_numpy_type
                    fields.append(T.StructField(f.name, _infer_numpy_type(s.to_numpy())))
                else:
                    fields.append(f)
            schema = T.StructType(fields)
        a, b = self._rank_slice(len(pdf))
        part = pdf.iloc[a:b].reset_index(drop=True)
        cached = {}

        def fn():
            if "b" not in cached:
                cached["b"] = batch_from_pandas(part, schema, dev)
            return [cached["b"]]
        return self._from_local_batches("LocalTableScan", fn, schema)

    def createDataFrameFromLocalTensors(self, columns: dict, schema=None) -> DataFrame:
        """Wrap THIS rank's shard of device tensors as a DataFrame (zero copy).

        ``columns``: name -> tensor ([n] scalar or [n, d] vector).  Each rank
        passes its own rows (SPMD); tensors already on the session device are
        used in place, so data generated in HBM never round-trips the host.
        """
        from .sql.batch import ColumnData
        cols = {}
        for k, t in columns.items():
            t = t.to(self.device) if t.device != self.device else t
            if t.dim() == 2:
                cols[k] = ColumnData(t if t.dtype == torch.float32 else t.float(), T.VectorUDT())
            else:
                cols[k] = ColumnData(t, T.from_torch(t.dtype))
        n = len(next(iter(cols.values()))) if cols else 0
        b = Batch(cols, n, self.device)
        sch = b.schema()
        return self._from_local_batches("DeviceTensorScan", lambda: [b], sch)

    def createDataFrameFromChunks(self, chunks, max_rows: int, schema=None) -> DataFrame:
        """A DataFrame STREAMED from host chunks (inputs larger than HBM).

        ``chunks``: a callable returning an iterator of ``{column: numpy array | cpu tensor}`` of at most
        ``max_rows`` rows each (this rank's rows, in order).  Chunks pass through pinned double buffers and a
        copy stream, so the H2D copy of chunk i + 1 overlaps the compute on chunk i.  Narrow pipelines
        (``model.transform``, ``select``, ``withColumn``) then run chunk by chunk; consume them with
        ``foreachBatch`` / ``count`` (batches are transient views of the staging buffers)."""
        from .models.inference import chunked_dataframe
        return chunked_dataframe(self, chunks, max_rows, schema)

    def table(self, name) -> DataFrame:
        return self.catalog._lookup(name)

    def sql(self, query: str) -> DataFrame:
        from .sql.parser import run_sql
        return run_sql(self, query)

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.stop()


def _long_col(ids):
    from .sql.batch import ColumnData
    return ColumnData(ids, T.LongType())
