"""Structured-streaming micro-batches.

File source → per-trigger device batch → the same lazy plan (e.g. a fitted
``PipelineModel.transform``) → sink.  Mirrors MLE 00 - MLlib Deployment
Options.py:46-117: ``readStream.schema(s).option("maxFilesPerTrigger", 1)
.parquet(dir)``, ``writeStream.format("memory").option("checkpointLocation",
…).outputMode("append").queryName(…).start()``, ``spark.streams.active``,
``stop``/``awaitTermination``/``recentProgress``.  Offsets and commits are
logged under the checkpoint directory so a restarted query resumes after the
last committed file.
"""
from __future__ import annotations

import json
import os
import threading
import time
import uuid
from typing import List, Optional

from ..sql import types as T
from ..sql.batch import Batch, concat_batches, empty_batch
from ..sql.dataframe import DataFrame, SourcePlan


class StreamingQueryException(Exception):
    pass


class _FileStreamSource:
    def __init__(self, session, path, fmt, schema, options):
        self.session = session
        self.path = path
        self.fmt = fmt
        self.schema = schema
        self.options = options
        self.max_files = int(options.get("maxfilespertrigger", "1000"))
        self.current: List[str] = []

    def list_files(self) -> List[str]:
        from ..sql.readwriter import _data_files
        ext = {"parquet": ".parquet", "csv": ".csv", "json": ".json"}.get(self.fmt)
        if self.fmt == "delta":
            from ..storage.delta import Snapshot, _versions
            vs = _versions(self.path)
            if not vs:
                return []
            return [os.path.join(self.path, p) for p in sorted(Snapshot(self.path, vs[-1]).files)]
        return _data_files(self.path, ext) if os.path.exists(self.path) else []

    def read_current(self) -> List[Batch]:
        if not self.current:
            return []
        r = self.session.read
        if self.fmt in ("parquet", "delta"):
            from ..sql.readwriter import scan_parquet_files
            df = scan_parquet_files(self.session, self.current, [self.path] * len(self.current), self.schema)
        else:
            df = r.format(self.fmt).schema(self.schema).options(**self.options).load(self.current)
        return df._plan.execute()


class DataStreamReader:
    def __init__(self, session):
        self._session = session
        self._schema = None
        self._options = {}
        self._format = "parquet"

    def schema(self, s):
        self._schema = T.to_schema(s)
        return self

    def option(self, k, v):
        self._options[k.lower()] = str(v)
        return self

    def options(self, **kw):
        for k, v in kw.items():
            self.option(k, v)
        return self

    def format(self, f):
        self._format = f.lower()
        return self

    def load(self, path=None):
        from ..sql.readwriter import _strip_dbfs
        path = _strip_dbfs(path)
        if self._schema is None:
            if self._format == "delta":
                from ..storage.delta import Snapshot, _versions
                self._schema = Snapshot(path, _versions(path)[-1]).schema
            else:
                raise StreamingQueryException(
                    "Schema must be specified when creating a streaming source DataFrame. (MLE 00:48)")
        src = _FileStreamSource(self._session, path, self._format, self._schema, self._options)
        plan = SourcePlan(self._session, f"StreamingRelation {self._format} {path}", src.read_current,
                          self._schema)
        df = DataFrame(plan, self._session)
        df.isStreaming = True
        plan.stream_source = src
        return df

    def parquet(self, path):
        self._format = "parquet"
        return self.load(path)

    def csv(self, path):
        self._format = "csv"
        return self.load(path)

    def json(self, path):
        self._format = "json"
        return self.load(path)

    def table(self, name):
        info = self._session.catalog._table_info(name)
        self._format = info.get("format", "parquet")
        return self.load(info["location"])


def _find_source(plan):
    if hasattr(plan, "stream_source"):
        return plan.stream_source
    for c in plan.children:
        s = _find_source(c)
        if s is not None:
            return s
    return None


class DataStreamWriter:
    def __init__(self, df: DataFrame):
        self._df = df
        self._format = "memory"
        self._options = {}
        self._mode = "append"
        self._name = None
        self._trigger_once = False
        self._interval = 0.0

    def format(self, f):
        self._format = f.lower()
        return self

    def option(self, k, v):
        self._options[k.lower()] = str(v)
        return self

    def options(self, **kw):
        for k, v in kw.items():
            self.option(k, v)
        return self

    def outputMode(self, m):
        self._mode = m.lower()
        return self

    def queryName(self, n):
        self._name = n
        return self

    def trigger(self, processingTime=None, once=None, availableNow=None):
        if once or availableNow:
            self._trigger_once = True
        if processingTime:
            self._interval = float(str(processingTime).split()[0])
        return self

    def start(self, path=None, format=None, outputMode=None, queryName=None):
        if format:
            self._format = format.lower()
        if outputMode:
            self._mode = outputMode.lower()
        if queryName:
            self._name = queryName
        src = _find_source(self._df._plan)
        if src is None:
            raise StreamingQueryException("DataFrame is not a streaming DataFrame")
        q = StreamingQuery(self._df, src, self._format, path, self._options, self._name, self._trigger_once,
                           self._interval)
        self._df._session.streams._add(q)
        q._start()
        return q

    def toTable(self, name):
        info = self._df._session.catalog
        loc = info._table_location(name)
        info._register_table(name, loc, "delta", managed=True)
        self._format = "delta"
        return self.start(loc)


class StreamingQuery:
    def __init__(self, df, src, fmt, path, options, name, once, interval):
        self._df = df
        self._src = src
        self._fmt = fmt
        self._path = path
        self._options = options
        self.name = name
        self.id = str(uuid.uuid4())
        self.runId = str(uuid.uuid4())
        self._once = once
        self._interval = interval
        self._session = df._session
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self.recentProgress: List[dict] = []
        self._batches: List[Batch] = []
        self._exc: Optional[BaseException] = None
        self._batch_id = 0
        self._ckpt = options.get("checkpointlocation")
        from ..sql.readwriter import _strip_dbfs
        if self._ckpt:
            self._ckpt = _strip_dbfs(self._ckpt)
        self._done_files = set()
        self._load_checkpoint()
        if fmt == "memory":
            if not name:
                raise StreamingQueryException("queryName must be specified for memory sink")
            self._register_memory_table()

    # ---------------------------------------------------------- checkpoint
    def _load_checkpoint(self):
        if not self._ckpt:
            return
        cdir = os.path.join(self._ckpt, "commits")
        odir = os.path.join(self._ckpt, "offsets")
        if not os.path.isdir(odir):
            return
        committed = set(int(f) for f in os.listdir(cdir) if f.isdigit()) if os.path.isdir(cdir) else set()
        for f in sorted(os.listdir(odir), key=lambda x: int(x) if x.isdigit() else -1):
            if f.isdigit() and int(f) in committed:
                with open(os.path.join(odir, f)) as fh:
                    self._done_files.update(json.load(fh)["files"])
                self._batch_id = max(self._batch_id, int(f) + 1)

    def _log(self, kind, bid, payload):
        if not self._ckpt or self._session.comm.rank != 0:
            return
        d = os.path.join(self._ckpt, kind)
        os.makedirs(d, exist_ok=True)
        tmp = os.path.join(d, f".{bid}.tmp")
        with open(tmp, "w") as fh:
            json.dump(payload, fh)
        os.replace(tmp, os.path.join(d, str(bid)))

    # ---------------------------------------------------------- sinks
    def _register_memory_table(self):
        q = self
        schema = self._df.schema

        def fn():
            return list(q._batches)
        table = DataFrame(SourcePlan(self._session, f"MemorySink {self.name}", fn, schema), self._session)
        self._session.catalog._register_temp(self.name, table)

    def _emit(self, parts: List[Batch]):
        if self._fmt == "memory":
            self._batches.extend(p for p in parts if p.n)
        elif self._fmt == "console":
            for p in parts:
                if self._session.comm.rank == 0:
                    print(f"-------------------------------------------\nBatch: {self._batch_id}\n"
                          f"-------------------------------------------")
                    print(p.to_pandas().head(20).to_string())
        elif self._fmt in ("parquet", "delta"):
            src = SourcePlan(self._session, "MicroBatch", lambda: parts, self._df.schema)
            mdf = DataFrame(src, self._session)
            if self._fmt == "delta":
                from ..storage.delta import write_delta
                write_delta(mdf, self._path, "append", {}, [], operation="STREAMING UPDATE")
            else:
                from ..sql.readwriter import write_files
                write_files(mdf, self._path, "parquet", "append", {}, [])
        elif self._fmt == "noop":
            pass
        else:
            raise StreamingQueryException(f"unsupported sink {self._fmt}")

    # ---------------------------------------------------------- loop
    def _run_one(self) -> bool:
        files = [f for f in self._src.list_files() if f not in self._done_files]
        if not files:
            return False
        chunk = files[: self._src.max_files]
        t0 = time.time()
        self._log("offsets", self._batch_id, {"files": chunk})
        self._src.current = chunk
        try:
            parts = self._df._plan.execute()
        finally:
            self._src.current = []
        n = sum(p.n for p in parts)
        self._emit(parts)
        self._log("commits", self._batch_id, {"batchId": self._batch_id})
        self._done_files.update(chunk)
        dt = max(time.time() - t0, 1e-9)
        self.recentProgress.append({"id": self.id, "runId": self.runId, "name": self.name,
                                    "batchId": self._batch_id, "numInputRows": n,
                                    "inputRowsPerSecond": n / dt, "processedRowsPerSecond": n / dt,
                                    "timestamp": time.strftime("%Y-%m-%dT%H:%M:%S"),
                                    "sources": [{"description": f"FileStreamSource[{self._src.path}]",
                                                 "numInputRows": n}],
                                    "sink": {"description": self._fmt}})
        self.recentProgress = self.recentProgress[-100:]
        self._batch_id += 1
        return True

    def _loop(self):
        try:
            while not self._stop.is_set():
                progressed = self._run_one()
                if self._once and not progressed:
                    break
                if not progressed:
                    self._stop.wait(max(self._interval, 0.05))
                elif self._interval:
                    self._stop.wait(self._interval)
        except BaseException as e:  # surfaced through exception()/awaitTermination
            self._exc = e
        finally:
            self._stop.set()

    def _start(self):
        if self._session.comm.distributed or self._once:
            # collectives must run in lock-step on the main thread of every rank
            while self._run_one():
                pass
            if self._once:
                self._stop.set()
            return
        self._thread = threading.Thread(target=self._loop, name=f"stream-{self.name}", daemon=True)
        self._thread.start()

    # ---------------------------------------------------------- API
    @property
    def isActive(self) -> bool:
        return not self._stop.is_set()

    @property
    def lastProgress(self):
        return self.recentProgress[-1] if self.recentProgress else None

    @property
    def status(self):
        return {"message": "Waiting for data to arrive" if self.isActive else "Stopped",
                "isDataAvailable": False, "isTriggerActive": False}

    def processAllAvailable(self):
        if self._thread is None:
            while self._run_one():
                pass
            return
        while self.isActive:
            pending = [f for f in self._src.list_files() if f not in self._done_files]
            if not pending:
                return
            time.sleep(0.05)

    def awaitTermination(self, timeout=None):
        if self._thread is not None:
            self._thread.join(timeout)
        if self._exc is not None:
            raise StreamingQueryException(str(self._exc)) from self._exc
        return not self.isActive

    def stop(self):
        self._stop.set()
        if self._thread is not None:
            self._thread.join(30)
        self._session.streams._remove(self)

    def exception(self):
        return self._exc

    def explain(self):
        self._df.explain()


class StreamingQueryManager:
    def __init__(self, session):
        self._session = session
        self._queries: List[StreamingQuery] = []

    def _add(self, q):
        self._queries.append(q)

    def _remove(self, q):
        if q in self._queries:
            self._queries.remove(q)

    @property
    def active(self) -> List[StreamingQuery]:
        return [q for q in self._queries if q.isActive]

    def get(self, qid):
        return next((q for q in self._queries if q.id == qid), None)

    def awaitAnyTermination(self, timeout=None):
        t0 = time.time()
        while self.active:
            if timeout is not None and time.time() - t0 > timeout:
                return False
            time.sleep(0.05)
        return True

    def resetTerminated(self):
        pass
