"""DataFrameReader / DataFrameWriter (SURVEY §2.2 S1–S6).

Host IO goes through pyarrow (CSV/Parquet/JSON); decoded columns move to the
rank's GPU once.  Files are assigned to ranks round-robin; a single large
file is row-sliced across ranks.  Writers produce one Parquet part file per
partition (the dedup lab requires exactly 8 part files after a shuffle with
``spark.sql.shuffle.partitions=8`` — Labs/ML 00L:35,79-80,139) and Hive-style
``col=value`` directories for ``partitionBy`` (ML 00c:99-121).
"""
from __future__ import annotations

import glob
import json
import os
import shutil
import uuid
from typing import Dict, List, Optional

import numpy as np
import pandas as pd
import pyarrow as pa
import pyarrow.csv as pacsv
import pyarrow.parquet as pq
import torch

from . import types as T
from .batch import Batch, ColumnData, batch_from_pandas, column_from_numpy, concat_batches, empty_batch
from .dataframe import DataFrame, SourcePlan


# ------------------------------------------------------------ arrow <-> batch
def arrow_to_spark_type(t: pa.DataType, meta: Optional[dict] = None) -> T.DataType:
    if meta and meta.get(b"cdnaml.type") == b"vector":
        return T.VectorUDT()
    if pa.types.is_boolean(t):
        return T.BooleanType()
    if pa.types.is_int8(t):
        return T.ByteType()
    if pa.types.is_int16(t):
        return T.ShortType()
    if pa.types.is_int32(t) or pa.types.is_uint16(t) or pa.types.is_uint8(t):
        return T.IntegerType()
    if pa.types.is_integer(t):
        return T.LongType()
    if pa.types.is_float32(t):
        return T.FloatType()
    if pa.types.is_floating(t) or pa.types.is_decimal(t):
        return T.DoubleType()
    if pa.types.is_string(t) or pa.types.is_large_string(t) or pa.types.is_dictionary(t):
        return T.StringType()
    if pa.types.is_date(t):
        return T.DateType()
    if pa.types.is_timestamp(t):
        return T.TimestampType()
    if pa.types.is_fixed_size_list(t) or pa.types.is_list(t):
        return T.ArrayType(T.DoubleType())
    if pa.types.is_null(t):
        return T.StringType()
    return T.StringType()


def table_to_batch(tbl: pa.Table, schema: Optional[T.StructType], device) -> Batch:
    cols = {}
    fields = schema.fields if schema is not None else None
    for i, name in enumerate(tbl.column_names):
        arr = tbl.column(i)
        f = tbl.schema.field(i)
        dt = None
        if fields is not None:
            match = [x for x in fields if x.name == name]
            dt = match[0].dataType if match else None
        if dt is None:
            dt = arrow_to_spark_type(f.type, f.metadata)
        cols[name] = arrow_column(arr, dt, device, f.metadata)
    if schema is not None:
        ordered = {}
        for fld in schema.fields:
            if fld.name in cols:
                ordered[fld.name] = cols[fld.name]
            else:
                from .batch import full_column
                ordered[fld.name] = full_column(None, fld.dataType, tbl.num_rows, device)
        cols = ordered
    return Batch(cols, tbl.num_rows, device)


def arrow_column(arr, dt: T.DataType, device, meta=None) -> ColumnData:
    if isinstance(arr, pa.ChunkedArray):
        arr = arr.combine_chunks() if arr.num_chunks != 1 else arr.chunk(0)
    n = len(arr)
    valid = None
    if arr.null_count:
        valid = torch.from_numpy(np.asarray(arr.is_valid().to_numpy(zero_copy_only=False), dtype=bool)).to(device)
    cmeta = {}
    if meta and b"cdnaml.meta" in meta:
        cmeta = json.loads(meta[b"cdnaml.meta"].decode())
    if isinstance(dt, T.StringType):
        if not (pa.types.is_string(arr.type) or pa.types.is_large_string(arr.type) or
                pa.types.is_dictionary(arr.type)):
            arr = arr.cast(pa.string())
        if not pa.types.is_dictionary(arr.type):
            arr = arr.dictionary_encode()
        d = np.asarray(arr.dictionary.to_pylist(), dtype=object)
        codes = arr.indices.fill_null(-1).to_numpy(zero_copy_only=False).astype(np.int32)
        # sort dictionary so code order == lexicographic order
        order = np.argsort(d.astype(str), kind="stable") if len(d) else np.zeros(0, np.int64)
        inv = np.empty(len(order), np.int32)
        inv[order] = np.arange(len(order), dtype=np.int32)
        codes = np.where(codes >= 0, inv[np.maximum(codes, 0)] if len(inv) else codes, -1).astype(np.int32)
        d = d[order]
        # dedupe (dictionary_encode of chunks can repeat)
        uni, remap = np.unique(d.astype(str), return_inverse=True) if len(d) else (d, np.zeros(0, np.int64))
        if len(uni) != len(d):
            codes = np.where(codes >= 0, remap[np.maximum(codes, 0)], -1).astype(np.int32)
            d = np.asarray(uni, dtype=object)
        return ColumnData(torch.from_numpy(codes).to(device), dt, valid, np.asarray(d, dtype=object), cmeta)
    if isinstance(dt, (T.VectorUDT, T.ArrayType)):
        if pa.types.is_fixed_size_list(arr.type):
            w = arr.type.list_size
            flat = arr.flatten().to_numpy(zero_copy_only=False).astype(np.float32)
            mat = flat.reshape(-1, w) if w else np.zeros((n, 0), np.float32)
            if len(mat) != n:  # nulls drop their slots
                full = np.zeros((n, w), np.float32)
                full[np.asarray(arr.is_valid())] = mat
                mat = full
        else:
            rows = arr.to_pylist()
            w = max((len(r) for r in rows if r is not None), default=0)
            mat = np.zeros((n, w), np.float32)
            for i, r in enumerate(rows):
                if r is not None:
                    mat[i, :len(r)] = r
        return ColumnData(torch.from_numpy(np.ascontiguousarray(mat)).to(device), dt, valid, meta=cmeta)
    if isinstance(dt, T.DateType):
        a = arr.cast(pa.int32()).fill_null(0).to_numpy(zero_copy_only=False) if pa.types.is_date(arr.type) \
            else None
        if a is None:
            return column_from_numpy(np.asarray(arr.to_pylist(), dtype=object), dt, device)
        return ColumnData(torch.from_numpy(a.astype(np.int32)).to(device), dt, valid, meta=cmeta)
    if isinstance(dt, T.TimestampType):
        a = arr.cast(pa.timestamp("us")).cast(pa.int64()).fill_null(0).to_numpy(zero_copy_only=False)
        return ColumnData(torch.from_numpy(a.astype(np.int64)).to(device), dt, valid, meta=cmeta)
    if pa.types.is_string(arr.type) or pa.types.is_large_string(arr.type):
        c = arrow_column(arr, T.StringType(), device)
        from .column import _cast
        return _cast(c, dt)
    npdt = np.dtype(str(dt.torch_dtype).replace("torch.", ""))
    if pa.types.is_boolean(arr.type):
        a = arr.fill_null(False).to_numpy(zero_copy_only=False)
    else:
        a = arr.fill_null(0).to_numpy(zero_copy_only=False)
    return ColumnData(torch.from_numpy(np.ascontiguousarray(a.astype(npdt))).to(device), dt, valid, meta=cmeta)


def batch_to_table(b: Batch) -> pa.Table:
    arrays, fields = [], []
    for name, c in b.columns.items():
        mask = None if c.valid is None else ~c.valid.cpu().numpy()
        meta = {}
        if c.meta:
            meta[b"cdnaml.meta"] = json.dumps(c.meta, default=str).encode()
        dt = c.dtype
        if isinstance(dt, T.StringType):
            codes = c.values.cpu().numpy().astype(np.int32)
            d = c.dictionary if c.dictionary is not None else np.array([], dtype=object)
            m = (codes < 0) if mask is None else (mask | (codes < 0))
            idx = pa.array(np.where(m, 0, codes), type=pa.int32(), mask=m)
            darr = pa.DictionaryArray.from_arrays(idx, pa.array(d.tolist() if len(d) else [""], type=pa.string()))
            arr = darr.cast(pa.string())
            ft = pa.string()
        elif isinstance(dt, (T.VectorUDT, T.ArrayType)):
            mat = c.values.detach().cpu().numpy()
            w = mat.shape[1] if mat.ndim == 2 else 1
            et = pa.float32() if isinstance(dt, T.VectorUDT) else pa.float64()
            flat = pa.array(mat.reshape(-1).astype(np.float32 if isinstance(dt, T.VectorUDT) else np.float64),
                            type=et)
            arr = pa.FixedSizeListArray.from_arrays(flat, w)
            if mask is not None:
                arr = pa.array(arr.to_pylist(), type=pa.list_(et, w), mask=mask) if mask.any() else arr
            ft = arr.type
            if isinstance(dt, T.VectorUDT):
                meta[b"cdnaml.type"] = b"vector"
        elif isinstance(dt, T.DateType):
            arr = pa.array(c.values.cpu().numpy().astype(np.int32), type=pa.int32(), mask=mask).cast(pa.date32())
            ft = pa.date32()
        elif isinstance(dt, T.TimestampType):
            arr = pa.array(c.values.cpu().numpy().astype(np.int64), type=pa.int64(), mask=mask).cast(
                pa.timestamp("us"))
            ft = pa.timestamp("us")
        else:
            a = c.values.detach().cpu().numpy()
            arr = pa.array(a, mask=mask)
            ft = arr.type
            if isinstance(dt, T.IntegerType):
                arr = arr.cast(pa.int32())
                ft = pa.int32()
        arrays.append(arr)
        fields.append(pa.field(name, ft, True, meta or None))
    return pa.Table.from_arrays(arrays, schema=pa.schema(fields))


def spark_to_arrow_schema(schema: T.StructType) -> pa.Schema:
    return batch_to_table(empty_batch(schema, torch.device("cpu"))).schema


# --------------------------------------------------------------- discovery
def _data_files(path: str, ext: Optional[str]) -> List[str]:
    if any(ch in path for ch in "*?["):
        files = sorted(glob.glob(path))
        out = []
        for f in files:
            out.extend(_data_files(f, ext) if os.path.isdir(f) else [f])
        return out
    if os.path.isfile(path):
        return [path]
    out = []
    for root, dirs, files in os.walk(path):
        dirs[:] = sorted(d for d in dirs if not d.startswith(("_", ".")))
        for f in sorted(files):
            if f.startswith(("_", ".")) or f.endswith(".crc"):
                continue
            if ext and not (f.endswith(ext) or ext == ".csv" or ext == ".json"):
                continue
            out.append(os.path.join(root, f))
    return out


def _partition_values(path: str, base: str) -> Dict[str, str]:
    rel = os.path.relpath(os.path.dirname(path), base)
    out = {}
    if rel in (".", ""):
        return out
    for part in rel.split(os.sep):
        if "=" in part:
            k, v = part.split("=", 1)
            out[k] = v
    return out


def _infer_partition_type(values: List[str]) -> T.DataType:
    try:
        ints = [int(v) for v in values if v != "__HIVE_DEFAULT_PARTITION__"]
        return T.IntegerType() if all(-2 ** 31 <= x < 2 ** 31 for x in ints) else T.LongType()
    except ValueError:
        pass
    try:
        [float(v) for v in values if v != "__HIVE_DEFAULT_PARTITION__"]
        return T.DoubleType()
    except ValueError:
        return T.StringType()


# ================================================================== reader
class DataFrameReader:
    def __init__(self, session):
        self._session = session
        self._format = "parquet"
        self._options: Dict[str, str] = {}
        self._schema: Optional[T.StructType] = None

    def format(self, source: str):
        self._format = source.lower()
        return self

    def option(self, key, value):
        self._options[key.lower()] = str(value) if not isinstance(value, bool) else str(value).lower()
        return self

    def options(self, **opts):
        for k, v in opts.items():
            self.option(k, v)
        return self

    def schema(self, schema):
        self._schema = T.to_schema(schema)
        return self

    def load(self, path=None, format=None, schema=None, **options):
        if format:
            self._format = format.lower()
        if schema is not None:
            self.schema(schema)
        self.options(**options)
        fmt = self._format
        if fmt == "delta":
            from ..storage.delta import read_delta
            return read_delta(self._session, path, self._options)
        if fmt == "csv":
            return self.csv(path)
        if fmt == "json":
            return self.json(path)
        if fmt in ("parquet", "orc"):
            return self.parquet(path)
        if fmt == "text":
            return self.text(path)
        raise ValueError(f"unsupported format {fmt}")

    def table(self, name):
        return self._session.table(name)

    # -------------------------------------------------------------- parquet
    def parquet(self, *paths, **options) -> DataFrame:
        self.options(**options)
        files = []
        bases = []
        for p in paths:
            p = _strip_dbfs(p)
            fs = _data_files(p, ".parquet")
            files.extend(fs)
            bases.extend([p] * len(fs))
        if not files:
            raise FileNotFoundError(f"Path does not exist or has no data files: {paths}")
        return scan_parquet_files(self._session, files, bases, self._schema)

    # ------------------------------------------------------------------ csv
    def csv(self, path, schema=None, sep=None, header=None, inferSchema=None, **kw) -> DataFrame:
        if schema is not None:
            self.schema(schema)
        for k, v in dict(sep=sep, header=header, inferSchema=inferSchema, **kw).items():
            if v is not None:
                self.option(k, v)
        o = self._options
        header_ = o.get("header", "false") == "true"
        infer = o.get("inferschema", "false") == "true"
        delim = o.get("sep", o.get("delimiter", ","))
        quote = o.get("quote", '"')
        escape = o.get("escape", "\\")
        multiline = o.get("multiline", "false") == "true"
        nullv = o.get("nullvalue", "")
        paths = path if isinstance(path, (list, tuple)) else [path]
        files = []
        for p in paths:
            files.extend(_data_files(_strip_dbfs(p), ".csv"))
        if not files:
            raise FileNotFoundError(f"Path does not exist: {path}")
        schema = self._schema
        tables = []
        for f in files:
            ro = pacsv.ReadOptions(autogenerate_column_names=not header_, block_size=1 << 26)
            po = pacsv.ParseOptions(delimiter=delim, quote_char=quote or False,
                                    escape_char=(escape if escape and escape != quote else False),
                                    double_quote=True, newlines_in_values=multiline)
            if schema is not None:
                names = schema.names
                if not header_:
                    ro = pacsv.ReadOptions(column_names=names, block_size=1 << 26)
                co = pacsv.ConvertOptions(column_types={n: pa.string() for n in names}, null_values=[nullv],
                                          strings_can_be_null=True)
            elif infer:
                co = pacsv.ConvertOptions(null_values=[nullv, "null", "NULL"], strings_can_be_null=True)
            else:
                co = pacsv.ConvertOptions(null_values=[nullv], strings_can_be_null=True,
                                          column_types=None, auto_dict_encode=False)
            t = pacsv.read_csv(f, read_options=ro, parse_options=po, convert_options=co)
            if not header_ and schema is None:
                t = t.rename_columns([f"_c{i}" for i in range(t.num_columns)])
            if schema is None and not infer:
                t = pa.Table.from_arrays([c.cast(pa.string()) for c in t.columns], names=t.column_names)
            tables.append(t)
        tbl = pa.concat_tables(tables, promote_options="default") if len(tables) > 1 else tables[0]
        if schema is None:
            fields = []
            for fld in tbl.schema:
                st = arrow_to_spark_type(fld.type)
                if isinstance(st, T.LongType):
                    col = tbl.column(fld.name)
                    import pyarrow.compute as pc
                    mn, mx = pc.min(col).as_py(), pc.max(col).as_py()
                    if mn is None or (-2 ** 31 <= mn and mx < 2 ** 31):
                        st = T.IntegerType()
                fields.append(T.StructField(fld.name, st))
            schema = T.StructType(fields)
        return _table_df(self._session, tbl, schema, f"FileScan csv {paths}")

    # ----------------------------------------------------------------- json
    def json(self, path, schema=None, **kw) -> DataFrame:
        if schema is not None:
            self.schema(schema)
        paths = path if isinstance(path, (list, tuple)) else [path]
        files = []
        for p in paths:
            files.extend(_data_files(_strip_dbfs(p), ".json"))
        rows = []
        for f in files:
            with open(f) as fh:
                for line in fh:
                    line = line.strip()
                    if line:
                        rows.append(json.loads(line))
        pdf = pd.json_normalize(rows, max_level=0) if rows else pd.DataFrame()
        for c in pdf.columns:
            if pdf[c].map(lambda v: isinstance(v, (dict, list))).any():
                pdf[c] = pdf[c].map(lambda v: None if v is None or (isinstance(v, float) and np.isnan(v))
                                    else json.dumps(v))
        return self._session.createDataFrame(pdf, schema=self._schema)

    def text(self, path) -> DataFrame:
        files = _data_files(_strip_dbfs(path), None)
        lines = []
        for f in files:
            with open(f) as fh:
                lines.extend(l.rstrip("\n") for l in fh)
        return self._session.createDataFrame(pd.DataFrame({"value": lines}))


def _strip_dbfs(p: str) -> str:
    """Every ``spark.read`` / ``write`` / Delta / stream / catalog path goes through
    the one DBFS resolver (``utils.dbutils.to_local``), so ``dbfs:/x``, ``/dbfs/x`` and
    ``file:/dbfs/x`` name the same file as ``dbutils.fs`` and pandas see."""
    from ..utils.dbutils import to_local
    return to_local(p)


def _table_df(session, tbl: pa.Table, schema: T.StructType, name: str) -> DataFrame:
    """Row-slice one host table across ranks (single-file sources)."""
    a, b = session._rank_slice(tbl.num_rows)
    part = tbl.slice(a, b - a)
    dev = session.device
    cache = {}

    def fn():
        if "b" not in cache:
            cache["b"] = table_to_batch(part, schema, dev)
        return [cache["b"]]
    return DataFrame(SourcePlan(session, name, fn, schema), session)


def scan_parquet_files(session, files: List[str], bases: List[str], schema: Optional[T.StructType],
                       name: str = "FileScan parquet") -> DataFrame:
    dev = session.device
    W, rank = session.comm.world_size, session.comm.rank
    pvals = [_partition_values(f, b) for f, b in zip(files, bases)]
    pkeys = []
    for pv in pvals:
        for k in pv:
            if k not in pkeys:
                pkeys.append(k)
    ptypes = {k: _infer_partition_type([pv.get(k, "") for pv in pvals]) for k in pkeys}
    if schema is None:
        s0 = pq.read_schema(files[0])
        fields = [T.StructField(f.name, arrow_to_spark_type(f.type, f.metadata)) for f in s0 if
                  f.name not in ptypes]
        # union with other files' columns (schema evolution)
        seen = {f.name for f in fields}
        for f in files[1:]:
            for fld in pq.read_schema(f):
                if fld.name not in seen and fld.name not in ptypes:
                    fields.append(T.StructField(fld.name, arrow_to_spark_type(fld.type, fld.metadata)))
                    seen.add(fld.name)
        fields += [T.StructField(k, ptypes[k]) for k in pkeys]
        schema = T.StructType(fields)
    data_schema = T.StructType([f for f in schema.fields if f.name not in ptypes])

    def read_one(f, pv):
        tbl = pq.read_table(f)
        b = table_to_batch(tbl, data_schema, dev)
        cols = dict(b.columns)
        for k in pkeys:
            from .batch import full_column
            v = pv.get(k)
            dt = ptypes[k]
            if v is None or v == "__HIVE_DEFAULT_PARTITION__":
                cols[k] = full_column(None, dt, b.n, dev)
            else:
                cols[k] = full_column(int(v) if isinstance(dt, T.IntegralType) else
                                      (float(v) if isinstance(dt, T.DoubleType) else v), dt, b.n, dev)
        return Batch({fl.name: cols[fl.name] for fl in schema.fields}, b.n, dev)

    if len(files) >= W:
        mine = [i for i in range(len(files)) if i % W == rank]

        def fn():
            return [read_one(files[i], pvals[i]) for i in mine]
    else:
        def fn():
            parts = [read_one(f, pv) for f, pv in zip(files, pvals)]
            b = concat_batches(parts) if parts else empty_batch(schema, dev)
            a, z = session._rank_slice(b.n)
            return [b.slice(a, z)]
    df = DataFrame(SourcePlan(session, f"{name} [{len(files)} files]", fn, schema), session)
    df._plan.files = files
    return df


# ================================================================== writer
class DataFrameWriter:
    def __init__(self, df: DataFrame):
        self._df = df
        self._mode = "errorifexists"
        self._format = "parquet"
        self._options: Dict[str, str] = {}
        self._partition_by: List[str] = []

    def mode(self, m):
        self._mode = (m or "errorifexists").lower()
        return self

    def format(self, f):
        self._format = f.lower()
        return self

    def option(self, k, v):
        self._options[k.lower()] = str(v).lower() if isinstance(v, bool) else str(v)
        return self

    def options(self, **kw):
        for k, v in kw.items():
            self.option(k, v)
        return self

    def partitionBy(self, *cols):
        self._partition_by = [c for cc in cols for c in (cc if isinstance(cc, (list, tuple)) else [cc])]
        return self

    def bucketBy(self, *a, **k):
        return self

    def sortBy(self, *a, **k):
        return self

    def save(self, path=None, format=None, mode=None, partitionBy=None, **options):
        if format:
            self._format = format.lower()
        if mode:
            self.mode(mode)
        if partitionBy:
            self.partitionBy(partitionBy)
        self.options(**options)
        if self._format == "delta":
            from ..storage.delta import write_delta
            return write_delta(self._df, _strip_dbfs(path), self._mode, self._options, self._partition_by)
        return write_files(self._df, _strip_dbfs(path), self._format, self._mode, self._options,
                           self._partition_by)

    def parquet(self, path, mode=None, partitionBy=None, compression=None):
        self._format = "parquet"
        if compression:
            self.option("compression", compression)
        return self.save(path, mode=mode, partitionBy=partitionBy)

    def csv(self, path, mode=None, header=None, sep=None, **kw):
        self._format = "csv"
        if header is not None:
            self.option("header", header)
        if sep is not None:
            self.option("sep", sep)
        return self.save(path, mode=mode)

    def json(self, path, mode=None):
        self._format = "json"
        return self.save(path, mode=mode)

    def saveAsTable(self, name, format=None, mode=None, partitionBy=None, **options):
        if format:
            self._format = format.lower()
        if mode:
            self.mode(mode)
        if partitionBy:
            self.partitionBy(partitionBy)
        session = self._df._session
        cat = session.catalog
        info = cat._table_info(name)
        loc = info["location"] if info else cat._table_location(name)
        if info and self._mode in ("error", "errorifexists"):
            raise RuntimeError(f"Table {name} already exists")
        if info and self._mode == "ignore":
            return
        fmt = self._format if self._format != "parquet" or info is None else info.get("format", "parquet")
        self._format = fmt
        self.save(loc)
        cat._register_table(name, loc, fmt, managed=True)

    def insertInto(self, name, overwrite=False):
        info = self._df._session.catalog._table_info(name)
        self._format = info.get("format", "parquet")
        self.mode("overwrite" if overwrite else "append").save(info["location"])


def write_files(df: DataFrame, path: str, fmt: str, mode: str, options: dict, partition_by: List[str]):
    session = df._session
    comm = session.comm
    exists = os.path.exists(path) and any(not n.startswith(".") for n in os.listdir(path)) \
        if os.path.isdir(path) else os.path.exists(path)
    if exists:
        if mode in ("error", "errorifexists", "default"):
            raise FileExistsError(f"path {path} already exists.")
        if mode == "ignore":
            return
    parts = df._plan.execute()
    counts = comm.all_gather_object(len(parts)) if comm.distributed else [len(parts)]
    base_idx = sum(counts[: comm.rank])
    comm.barrier()
    if comm.rank == 0:
        if exists and mode == "overwrite":
            shutil.rmtree(path, ignore_errors=True) if os.path.isdir(path) else os.remove(path)
        os.makedirs(path, exist_ok=True)
    comm.barrier()
    job = uuid.uuid4().hex[:8] if comm.rank == 0 else None
    job = comm.broadcast_object(job)
    written = []
    for i, b in enumerate(parts):
        idx = base_idx + i
        written.extend(_write_partition(b, path, fmt, options, partition_by, idx, job))
    comm.barrier()
    if comm.rank == 0:
        open(os.path.join(path, "_SUCCESS"), "w").close()
    return written


def _write_partition(b: Batch, path, fmt, options, partition_by, idx, job) -> List[str]:
    out = []
    if partition_by:
        from .relational import combine_codes
        gid, G = combine_codes([b.columns[k] for k in partition_by], b.n, b.device)
        for g in range(G):
            sub = b.filter(gid == g)
            if sub.n == 0:
                continue
            vals = [sub.columns[k].slice(0, 1).to_pylist()[0] for k in partition_by]
            d = os.path.join(path, *[f"{k}={'__HIVE_DEFAULT_PARTITION__' if v is None else v}"
                                     for k, v in zip(partition_by, vals)])
            os.makedirs(d, exist_ok=True)
            rest = sub.select([k for k in sub.names if k not in partition_by])
            out.append(_write_one(rest, d, fmt, options, idx, job))
        return out
    return [_write_one(b, path, fmt, options, idx, job)]


def _write_one(b: Batch, d, fmt, options, idx, job) -> str:
    if fmt == "parquet":
        comp = options.get("compression", "snappy")
        name = f"part-{idx:05d}-{job}-c000.{comp}.parquet" if comp != "none" else f"part-{idx:05d}-{job}-c000.parquet"
        fp = os.path.join(d, name)
        pq.write_table(batch_to_table(b), fp, compression=None if comp == "none" else comp)
    elif fmt == "csv":
        fp = os.path.join(d, f"part-{idx:05d}-{job}-c000.csv")
        pdf = b.to_pandas()
        pdf.to_csv(fp, index=False, header=options.get("header", "false") == "true", sep=options.get("sep", ","))
    elif fmt == "json":
        fp = os.path.join(d, f"part-{idx:05d}-{job}-c000.json")
        b.to_pandas().to_json(fp, orient="records", lines=True)
    else:
        raise ValueError(f"unsupported format {fmt}")
    return fp
