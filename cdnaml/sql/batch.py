"""Device-resident columnar partitions.

A ``Batch`` is one partition: an ordered set of ``ColumnData`` that all live
on the rank's GPU (or CPU in CPU-only runs).  Numeric columns are torch
tensors, strings are dictionary codes + a host dictionary (so string
predicates, lower()/translate() and group keys run as integer ops on the
GPU), vectors are dense ``[n, d]`` matrices (fp64 = Spark's Double at course scale, fp32 for large ones).  Nulls are a separate
validity mask (``None`` = no nulls).
"""
from __future__ import annotations

import datetime as _dt
from typing import Dict, List, Optional, Sequence

import numpy as np
import pandas as pd
import torch

from . import types as T

_EPOCH = _dt.date(1970, 1, 1)


def _gather_min() -> int:
    from ..ops import relops as R
    return R.GATHER_MIN


class ColumnData:
    __slots__ = ("values", "valid", "dtype", "dictionary", "meta")

    def __init__(self, values: torch.Tensor, dtype: T.DataType, valid: Optional[torch.Tensor] = None,
                 dictionary: Optional[np.ndarray] = None, meta: Optional[dict] = None):
        self.values = values
        self.dtype = dtype
        self.valid = valid
        self.dictionary = dictionary
        self.meta = meta or {}

    # ------------------------------------------------------------ basics
    def __len__(self):
        return int(self.values.shape[0])

    @property
    def device(self):
        return self.values.device

    def with_meta(self, meta):
        return ColumnData(self.values, self.dtype, self.valid, self.dictionary, meta)

    def clone(self) -> "ColumnData":
        return ColumnData(self.values.clone(), self.dtype, None if self.valid is None else self.valid.clone(),
                          self.dictionary, self.meta)

    def valid_mask(self) -> torch.Tensor:
        if self.valid is None:
            return torch.ones(len(self), dtype=torch.bool, device=self.device)
        return self.valid

    def has_nulls(self) -> bool:
        return self.valid is not None and not bool(self.valid.all())

    def _py_meta(self, sel):
        """meta with the host-object payload (``_py``: one Python value per row -- collect_list arrays, struct
        rows) re-indexed like the rows."""
        py = self.meta.get("_py")
        if py is None:
            return self.meta
        return dict(self.meta, _py=[py[i] for i in sel])

    def take(self, idx: torch.Tensor) -> "ColumnData":
        meta = self._py_meta(idx.reshape(-1).cpu().tolist()) if "_py" in self.meta else self.meta
        return ColumnData(self.values[idx], self.dtype, None if self.valid is None else self.valid[idx],
                          self.dictionary, meta)

    def slice(self, a: int, b: int) -> "ColumnData":
        meta = self._py_meta(range(len(self.meta["_py"]))[a:b]) if "_py" in self.meta else self.meta
        return ColumnData(self.values[a:b], self.dtype, None if self.valid is None else self.valid[a:b],
                          self.dictionary, meta)

    def to(self, device) -> "ColumnData":
        return ColumnData(self.values.to(device), self.dtype, None if self.valid is None else self.valid.to(device),
                          self.dictionary, self.meta)

    # ------------------------------------------------------------ host
    def to_numpy(self, nulls_as_nan: bool = False):
        """Host values as a numpy/pandas-friendly array (object for strings/vectors).

        ``nulls_as_nan``: numeric nulls become NaN in a float64 array (what Spark's
        Arrow ``toPandas`` produces); otherwise they are ``None`` in an object array.
        """
        py = self.meta.get("_py")
        if py is not None:  # host objects (collect_list arrays, struct rows), one per row
            out = np.empty(len(py), dtype=object)
            for i, x in enumerate(py):
                out[i] = x
            if self.valid is not None:
                out[~self.valid.cpu().numpy()] = None
            return out
        v = self.values.detach().cpu()
        valid = None if self.valid is None else self.valid.cpu().numpy()
        dt = self.dtype
        if isinstance(dt, T.StringType):
            codes = v.numpy()
            d = self.dictionary if self.dictionary is not None else np.array([], dtype=object)
            out = np.empty(len(codes), dtype=object)
            ok = codes >= 0
            if valid is not None:
                ok &= valid
            out[ok] = d[codes[ok]]
            out[~ok] = None
            return out
        if isinstance(dt, (T.VectorUDT, T.ArrayType)):
            from ..models.linalg import DenseVector
            a = v.numpy().astype(np.float64)
            out = np.empty(len(a), dtype=object)
            for i in range(len(a)):
                out[i] = DenseVector(a[i]) if isinstance(dt, T.VectorUDT) else list(a[i])
            if valid is not None:
                out[~valid] = None
            return out
        if isinstance(dt, T.DateType):
            a = v.numpy()
            out = np.empty(len(a), dtype=object)
            for i, x in enumerate(a):
                out[i] = _EPOCH + _dt.timedelta(days=int(x))
            if valid is not None:
                out[~valid] = None
            return out
        if isinstance(dt, T.TimestampType):
            a = v.numpy().astype("datetime64[us]")
            if valid is not None:
                a = a.astype(object)
                a[~valid] = None
            return a
        a = v.numpy()
        if valid is not None and not valid.all():
            if nulls_as_nan and not isinstance(dt, T.BooleanType):
                a = a.astype(np.float64)
                a[~valid] = np.nan
                return a
            if isinstance(dt, (T.FloatType, T.DoubleType)):
                a = a.astype(np.float64)
                a[~valid] = np.nan
                o = a.astype(object)
                o[~valid] = None
                return o
            o = a.astype(object)
            o[~valid] = None
            return o
        return a

    def to_pylist(self):
        a = self.to_numpy()
        if a.dtype == object:
            return list(a)
        if isinstance(self.dtype, T.BooleanType):
            return [bool(x) for x in a]
        if a.dtype.kind in "iu":
            return [int(x) for x in a]
        if a.dtype.kind == "f":
            return [float(x) for x in a]
        return list(a)


def empty_column(dt: T.DataType, device, width: int = 0, meta=None) -> ColumnData:
    if isinstance(dt, (T.VectorUDT, T.ArrayType)):
        return ColumnData(torch.zeros((0, width), dtype=torch.float32, device=device), dt, meta=meta)
    if isinstance(dt, T.StringType):
        return ColumnData(torch.zeros(0, dtype=torch.int32, device=device), dt,
                          dictionary=np.array([], dtype=object), meta=meta)
    return ColumnData(torch.zeros(0, dtype=dt.torch_dtype or torch.float64, device=device), dt, meta=meta)


def full_column(value, dt: T.DataType, n: int, device) -> ColumnData:
    """Broadcast a python literal to a column of n rows."""
    if value is None:
        c = empty_column(dt if not isinstance(dt, T.NullType) else T.DoubleType(), device)
        if isinstance(dt, T.StringType):
            return ColumnData(torch.full((n,), -1, dtype=torch.int32, device=device), dt,
                              torch.zeros(n, dtype=torch.bool, device=device), np.array([], dtype=object))
        vals = torch.zeros((n,) + tuple(c.values.shape[1:]), dtype=c.values.dtype, device=device)
        return ColumnData(vals, c.dtype, torch.zeros(n, dtype=torch.bool, device=device))
    if isinstance(dt, T.StringType):
        return ColumnData(torch.zeros(n, dtype=torch.int32, device=device), dt,
                          dictionary=np.array([str(value)], dtype=object))
    if isinstance(dt, T.VectorUDT):
        arr = torch.as_tensor(np.asarray(value.toArray() if hasattr(value, "toArray") else value, np.float64))
        return ColumnData(arr.to(device)[None, :].expand(n, -1).contiguous(), dt)
    if isinstance(dt, T.DateType) and isinstance(value, _dt.date):
        value = (value - _EPOCH).days
    return ColumnData(torch.full((n,), value, dtype=dt.torch_dtype, device=device), dt)


def infer_literal_type(v) -> T.DataType:
    if v is None:
        return T.NullType()
    if isinstance(v, bool):
        return T.BooleanType()
    if isinstance(v, (int, np.integer)):
        return T.IntegerType() if -2 ** 31 <= int(v) < 2 ** 31 else T.LongType()
    if isinstance(v, (float, np.floating)):
        return T.DoubleType()
    if isinstance(v, str):
        return T.StringType()
    if isinstance(v, _dt.datetime):
        return T.TimestampType()
    if isinstance(v, _dt.date):
        return T.DateType()
    if hasattr(v, "toArray"):
        return T.VectorUDT()
    raise TypeError(f"unsupported literal {v!r}")


class Batch:
    """One partition: ordered columns of equal length."""

    __slots__ = ("columns", "n", "device")

    def __init__(self, columns: Dict[str, ColumnData], n: Optional[int] = None, device=None):
        self.columns = dict(columns)
        if n is None:
            n = len(next(iter(self.columns.values()))) if self.columns else 0
        self.n = int(n)
        if device is None:
            device = next(iter(self.columns.values())).device if self.columns else torch.device("cpu")
        self.device = device

    def __len__(self):
        return self.n

    @property
    def names(self) -> List[str]:
        return list(self.columns.keys())

    def __getitem__(self, name) -> ColumnData:
        return self.columns[name]

    def schema(self) -> T.StructType:
        return T.StructType([T.StructField(k, c.dtype, True, c.meta) for k, c in self.columns.items()])

    def clone(self) -> "Batch":
        """Deep copy of the device tensors (a streamed batch aliases a reused staging buffer)."""
        return Batch({k: c.clone() for k, c in self.columns.items()}, self.n, self.device)

    def select(self, names: Sequence[str]) -> "Batch":
        return Batch({k: self.columns[k] for k in names}, self.n, self.device)

    def with_column(self, name: str, col: ColumnData) -> "Batch":
        cols = dict(self.columns)
        cols[name] = col
        return Batch(cols, self.n, self.device)

    def take(self, idx: torch.Tensor) -> "Batch":
        if idx.dtype != torch.bool and idx.is_cuda and idx.numel() >= _gather_min():
            return self._take_native(idx)
        return Batch({k: c.take(idx) for k, c in self.columns.items()}, int(idx.shape[0]) if idx.dtype != torch.bool
                     else int(idx.sum()), self.device)

    def _take_native(self, idx: torch.Tensor) -> "Batch":
        """Every 1-D column (values and null masks) gathered by K19 gather kernels, 8 arrays per launch."""
        from ..ops import kernels as K
        names = list(self.columns)
        arrs = []
        for k in names:
            c = self.columns[k]
            arrs.append(c.values)
            arrs.append(None if c.valid is None else c.valid.view(torch.uint8) if c.valid.dtype == torch.bool
                        else c.valid)
        got = K.gather_cols(arrs, idx)
        cols = {}
        for j, k in enumerate(names):
            c = self.columns[k]
            v = got[2 * j] if got[2 * j] is not None else c.values[idx]
            m = None
            if c.valid is not None:
                m = got[2 * j + 1]
                m = c.valid[idx] if m is None else (m.view(torch.bool) if c.valid.dtype == torch.bool else m)
            cols[k] = ColumnData(v, c.dtype, m, c.dictionary, c.meta)
        return Batch(cols, int(idx.shape[0]), self.device)

    def filter(self, mask: torch.Tensor) -> "Batch":
        from ..ops import kernels as K
        idx = K.compact_mask(mask)  # K19 stream compaction (HIP on the GPU)
        return self.take(idx)

    def slice(self, a: int, b: int) -> "Batch":
        a, b = max(0, a), min(self.n, b)
        return Batch({k: c.slice(a, b) for k, c in self.columns.items()}, max(0, b - a), self.device)

    def to(self, device) -> "Batch":
        return Batch({k: c.to(device) for k, c in self.columns.items()}, self.n, device)

    def empty_like(self) -> "Batch":
        return self.slice(0, 0)

    # ------------------------------------------------------------- pandas
    def to_pandas(self) -> pd.DataFrame:
        data = {}
        for k, c in self.columns.items():
            data[k] = c.to_numpy(nulls_as_nan=True)
        return pd.DataFrame(data, columns=self.names)


# ---------------------------------------------------------------- strings
def unify_dictionaries(cols: List[ColumnData]) -> List[ColumnData]:
    """Re-encode string columns against one shared (sorted) dictionary."""
    dicts = [c.dictionary if c.dictionary is not None else np.array([], dtype=object) for c in cols]
    if all(len(d) == len(dicts[0]) and (d is dicts[0] or np.array_equal(d, dicts[0])) for d in dicts):
        return cols
    allv = np.concatenate([np.asarray(d, dtype=object) for d in dicts]) if dicts else np.array([], dtype=object)
    uni = np.array(sorted(set(allv.tolist())), dtype=object)
    return [recode(c, uni) for c in cols]


def recode(c: ColumnData, new_dict: np.ndarray) -> ColumnData:
    """Map codes of ``c`` into ``new_dict`` (must contain every used value; missing -> -1)."""
    old = c.dictionary if c.dictionary is not None else np.array([], dtype=object)
    pos = {v: i for i, v in enumerate(new_dict.tolist())}
    lut = np.array([pos.get(v, -1) for v in old.tolist()] + [-1], dtype=np.int32)
    lut_t = torch.from_numpy(lut).to(c.device)
    codes = c.values.long()
    codes = torch.where(codes < 0, torch.full_like(codes, len(old)), codes)
    return ColumnData(lut_t[codes].to(torch.int32), c.dtype, c.valid, new_dict, c.meta)


def map_dictionary(c: ColumnData, fn) -> ColumnData:
    """Apply a python str->str function to the dictionary (then dedupe)."""
    old = c.dictionary if c.dictionary is not None else np.array([], dtype=object)
    mapped = [fn(v) for v in old.tolist()]
    uni = sorted(set(m for m in mapped if m is not None))
    pos = {v: i for i, v in enumerate(uni)}
    lut = np.array([pos[m] if m is not None else -1 for m in mapped] + [-1], dtype=np.int32)
    lut_t = torch.from_numpy(lut).to(c.device)
    codes = c.values.long()
    codes = torch.where(codes < 0, torch.full_like(codes, len(old)), codes)
    new = lut_t[codes].to(torch.int32)
    valid = c.valid
    if any(m is None for m in mapped):
        valid = new >= 0 if valid is None else valid & (new >= 0)
    return ColumnData(new, c.dtype, valid, np.array(uni, dtype=object), c.meta)


def concat_columns(cols: List[ColumnData]) -> ColumnData:
    if len(cols) == 1:
        return cols[0]
    dt = cols[0].dtype
    if isinstance(dt, T.StringType):
        cols = unify_dictionaries(cols)
    vals = torch.cat([c.values for c in cols])
    valid = None
    if any(c.valid is not None for c in cols):
        valid = torch.cat([c.valid_mask() for c in cols])
    return ColumnData(vals, dt, valid, cols[0].dictionary, cols[0].meta)


def concat_batches(batches: List[Batch]) -> Batch:
    batches = [b for b in batches if b is not None]
    if not batches:
        raise ValueError("no batches")
    nonempty = [b for b in batches if b.n > 0]
    if len(nonempty) == 1:
        return nonempty[0]
    if not nonempty:
        return batches[0]
    names = nonempty[0].names
    cols = {k: concat_columns([b.columns[k] for b in nonempty]) for k in names}
    return Batch(cols, sum(b.n for b in nonempty), nonempty[0].device)


# ------------------------------------------------------------ conversions
DICT_ENCODE_MIN_ROWS = 50_000


def column_from_numpy(arr, dt: Optional[T.DataType], device) -> ColumnData:
    """Build a device column from host values (numpy / pandas / list)."""
    if isinstance(arr, pd.Series):
        if isinstance(arr.dtype, pd.CategoricalDtype):
            arr = arr.astype(object)
        arr = arr.to_numpy()
    arr = np.asarray(arr) if not isinstance(arr, np.ndarray) else arr
    n = len(arr)
    if dt is None:
        dt = _infer_numpy_type(arr)
    if isinstance(dt, T.StringType):
        vals = np.asarray(arr, dtype=object)
        if n >= DICT_ENCODE_MIN_ROWS and torch.device(device).type == "cuda":
            # K17: Arrow strings -> device hash dictionary encode (no per-row Python, no object sort)
            try:
                import pyarrow as pa
                pa_arr = pa.array(vals, type=pa.string(), from_pandas=True)
            except (pa.ArrowInvalid, pa.ArrowTypeError):
                pa_arr = None
            if pa_arr is not None:
                from ..ops import kernels as K
                codes, valid, uni = K.dict_encode(pa_arr, device)
                return ColumnData(codes, dt, valid, uni)
        isnull = np.array([v is None or (isinstance(v, float) and np.isnan(v)) for v in vals], dtype=bool) \
            if vals.dtype == object else np.zeros(n, bool)
        sv = np.where(isnull, "", vals.astype(str) if vals.dtype != object else vals).astype(object)
        if n:
            sv = np.array([str(v) for v in sv], dtype=object)
            uni, codes = np.unique(sv[~isnull], return_inverse=True) if (~isnull).any() else (np.array([], object),
                                                                                                np.array([], int))
            full = np.full(n, -1, dtype=np.int32)
            full[~isnull] = codes
        else:
            uni, full = np.array([], dtype=object), np.zeros(0, np.int32)
        valid = None if not isnull.any() else torch.from_numpy(~isnull).to(device)
        return ColumnData(torch.from_numpy(full.astype(np.int32)).to(device), dt, valid, np.asarray(uni, object))
    if isinstance(dt, (T.VectorUDT, T.ArrayType)):
        rows = []
        isnull = np.zeros(n, bool)
        width = None
        for i, v in enumerate(arr):
            if v is None:
                isnull[i] = True
                rows.append(None)
                continue
            a = np.asarray(v.toArray() if hasattr(v, "toArray") else v, dtype=np.float64)
            width = len(a)
            rows.append(a)
        width = width or 0
        # Spark's vectors hold Doubles: kept fp64 at course scale (models.util.VECTOR_F64_MAX elements)
        from ..models.util import VECTOR_F64_MAX
        mat = np.zeros((n, width), np.float64 if n * width <= VECTOR_F64_MAX else np.float32)
        for i, r in enumerate(rows):
            if r is not None:
                mat[i] = r
        valid = None if not isnull.any() else torch.from_numpy(~isnull).to(device)
        return ColumnData(torch.from_numpy(mat).to(device), dt, valid)
    if isinstance(dt, T.DateType):
        out = np.zeros(n, np.int32)
        isnull = np.zeros(n, bool)
        for i, v in enumerate(arr):
            if v is None or (isinstance(v, float) and np.isnan(v)) or v is pd.NaT:
                isnull[i] = True
            elif isinstance(v, (np.datetime64, pd.Timestamp)):
                out[i] = int(pd.Timestamp(v).normalize().value // 86400_000_000_000)
            elif isinstance(v, _dt.date):
                out[i] = (v if not isinstance(v, _dt.datetime) else v.date()).toordinal() - _EPOCH.toordinal()
            else:
                out[i] = (pd.Timestamp(v).date() - _EPOCH).days
        valid = None if not isnull.any() else torch.from_numpy(~isnull).to(device)
        return ColumnData(torch.from_numpy(out).to(device), dt, valid)
    if isinstance(dt, T.TimestampType):
        s = pd.to_datetime(pd.Series(arr))
        isnull = s.isna().to_numpy()
        us = s.astype("int64").to_numpy() // 1000 if not isnull.all() else np.zeros(n, np.int64)
        us = np.where(isnull, 0, us)
        valid = None if not isnull.any() else torch.from_numpy(~isnull).to(device)
        return ColumnData(torch.from_numpy(us.astype(np.int64)).to(device), dt, valid)
    # numeric / boolean
    if arr.dtype == object:
        isnull = np.array([v is None or (isinstance(v, float) and np.isnan(v)) for v in arr], dtype=bool)
        fill = np.array([0 if m else v for v, m in zip(arr, isnull)])
        vals = fill.astype(np.dtype(str(dt.torch_dtype).replace("torch.", "")))
    else:
        isnull = np.zeros(n, bool)
        if arr.dtype.kind == "f" and isinstance(dt, T.IntegralType):
            isnull = np.isnan(arr)
            arr = np.where(isnull, 0, arr)
        if arr.dtype.kind == "f" and isinstance(dt, T.FractionalType) and pd.isna(arr).any():
            # pandas NaN from a missing value -> Spark null
            isnull = np.isnan(arr)
        vals = arr.astype(np.dtype(str(dt.torch_dtype).replace("torch.", "")))
    valid = None if not isnull.any() else torch.from_numpy(~isnull).to(device)
    return ColumnData(torch.from_numpy(np.ascontiguousarray(vals)).to(device), dt, valid)


def _infer_numpy_type(arr: np.ndarray) -> T.DataType:
    k = arr.dtype.kind
    if k == "b":
        return T.BooleanType()
    if k in "iu":
        return T.LongType() if arr.dtype.itemsize >= 8 else T.IntegerType()
    if k == "f":
        return T.DoubleType() if arr.dtype.itemsize >= 8 else T.FloatType()
    if k == "M":
        return T.TimestampType()
    if k in "US":
        return T.StringType()
    # object: sniff first non-null
    for v in arr:
        if v is None or (isinstance(v, float) and np.isnan(v)):
            continue
        if isinstance(v, bool):
            return T.BooleanType()
        if isinstance(v, (int, np.integer)):
            return T.LongType()
        if isinstance(v, (float, np.floating)):
            return T.DoubleType()
        if isinstance(v, str):
            return T.StringType()
        if isinstance(v, _dt.datetime):
            return T.TimestampType()
        if isinstance(v, _dt.date):
            return T.DateType()
        if hasattr(v, "toArray"):
            return T.VectorUDT()
        if isinstance(v, (list, tuple, np.ndarray)):
            return T.ArrayType(T.DoubleType())
        return T.StringType()
    return T.StringType() if len(arr) == 0 else T.DoubleType()


def pandas_dtype_to_spark(s: pd.Series) -> T.DataType:
    k = s.dtype.kind
    if k == "b":
        return T.BooleanType()
    if k in "iu":
        return T.LongType()
    if k == "f":
        return T.DoubleType()
    if k == "M":
        return T.TimestampType()
    return _infer_numpy_type(s.to_numpy())


def batch_from_pandas(pdf: pd.DataFrame, schema: Optional[T.StructType], device) -> Batch:
    cols = {}
    names = list(pdf.columns) if schema is None else schema.names
    for i, name in enumerate(names):
        src = pdf[pdf.columns[i]] if schema is not None and name not in pdf.columns else pdf[name]
        dt = schema[name].dataType if schema is not None else pandas_dtype_to_spark(src)
        cols[name] = column_from_numpy(src, dt, device)
    return Batch(cols, len(pdf), device)


def empty_batch(schema: T.StructType, device, widths: Optional[dict] = None) -> Batch:
    widths = widths or {}

    def width(f):
        if f.name in widths:
            return widths[f.name]
        ma = (f.metadata or {}).get("ml_attr") or {}
        return int(ma.get("num_attrs") or 0)

    cols = {f.name: empty_column(f.dataType, device, width(f), f.metadata) for f in schema.fields}
    return Batch(cols, 0, device)
