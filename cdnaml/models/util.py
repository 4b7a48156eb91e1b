"""Shared helpers for estimators: device matrices, ML attributes, errors."""
from __future__ import annotations

import os
from typing import List, Optional, Tuple

import numpy as np
import torch

from ..sql import types as T
from ..sql.batch import Batch, ColumnData, concat_batches
from ..sql.dataframe import MapPlan


class IllegalArgumentException(ValueError):
    pass


_VECTOR_SQL = "struct<type:tinyint,size:int,indices:array<int>,values:array<double>>"


def require_vector(df, col: str):
    f = df.schema[col] if col in df.columns else None
    if f is None:
        raise IllegalArgumentException(f"Field \"{col}\" does not exist.\nAvailable fields: {', '.join(df.columns)}")
    if not isinstance(f.dataType, (T.VectorUDT, T.ArrayType)):
        raise IllegalArgumentException(
            f"requirement failed: Column {col} must be of type {_VECTOR_SQL} but was actually "
            f"{f.dataType.simpleString()}.")


def require_numeric(df, col: str):
    f = df.schema[col]
    if not (f.dataType.is_numeric or isinstance(f.dataType, T.BooleanType)):
        raise IllegalArgumentException(
            f"requirement failed: Column {col} must be of type numeric but was actually of type "
            f"{f.dataType.simpleString()}.")


def local_batch(df, cols: List[str]) -> Batch:
    parts = df.select(*cols)._plan.execute()
    if not parts:
        from ..sql.batch import empty_batch
        return empty_batch(df.select(*cols).schema, df._session.device)
    return concat_batches(parts)


# Spark's VectorUDT holds Doubles.  A Double feature matrix of at most this many elements per rank (2^27: 1 GiB of
# fp64; the course's Airbnb / iris / MovieLens designs are 1e3-1e6) is consumed in fp64 by the linear-algebra
# estimators that opt in (linear / logistic regression, k-means, scalers, statistics); larger ones, and every fp32
# matrix (the 1e8 x 100 benchmark shapes), take the fp32 HBM-bound kernels.  CDNAML_VECTOR_F64_MAX=0 disables.
VECTOR_F64_MAX = int(os.environ.get("CDNAML_VECTOR_F64_MAX", str(1 << 27)))


def feature_dtype(X: torch.Tensor) -> torch.dtype:
    """The compute dtype of a feature matrix: fp64 for course-sized Double vectors, else fp32."""
    return torch.float64 if X.dtype == torch.float64 and X.numel() <= VECTOR_F64_MAX else torch.float32


def local_xyw(df, features_col: str, label_col: Optional[str] = None, weight_col: Optional[str] = None,
              drop_null_label: bool = True, keep_f64: bool = False
              ) -> Tuple[torch.Tensor, Optional[torch.Tensor], Optional[torch.Tensor]]:
    """This rank's rows as device tensors: X [n, d] (f32, or f64 when ``keep_f64`` and the column holds a
    course-sized Double matrix: ``feature_dtype``), y f64 [n], w f64 [n]."""
    require_vector(df, features_col)
    cols = [features_col] + ([label_col] if label_col else []) + ([weight_col] if weight_col else [])
    b = local_batch(df, cols)
    X = b.columns[features_col].values
    want = feature_dtype(X) if keep_f64 else torch.float32
    if X.dtype != want:
        X = X.to(want)
    y = w = None
    keep = None
    if label_col:
        yc = b.columns[label_col]
        y = yc.values.to(torch.float64)
        if yc.valid is not None and drop_null_label:
            keep = yc.valid
    if weight_col:
        w = b.columns[weight_col].values.to(torch.float64)
    if keep is not None and not bool(keep.all()):
        X = X[keep]
        y = y[keep]
        w = None if w is None else w[keep]
    return X, y, w


# out-of-core fits: a training frame over a streamed source (createDataFrameFromChunks /
# device_chunks) is never materialised -- its label / weight columns are collected, its features read chunk by chunk
OOC_FIT = __import__("os").environ.get("CDNAML_OOC_FIT", "1") != "0"


def streamed_columns(df, features_col: str, cols: List[str], head_rows: int = 0):
    """For a streamable training frame: ``(ChunkedRows over the features, {col: ColumnData}, feature metadata)``
    after one pass that collects the other (small) columns and counts the rows; None when the frame is not
    streamed (the caller materialises it) or a collected column has nulls.  ``head_rows``: the dict also holds
    ``"__head__"``, a copy of the first rows' features (at most that many)."""
    from .tree.binning import ChunkedRows
    if not OOC_FIT:
        return None
    sel = df.select(features_col, *cols)
    if not sel._plan.streamable:
        return None
    parts = {c: [] for c in cols}
    n, d = 0, None
    head = []
    ok = True
    # a host-chunk source read directly: the collection pass copies only the small columns, and the quantile
    # sample gathers its rows from the host chunks (the features cross PCIe once, in the binning pass)
    base = df._plan
    host_fn = getattr(base, "host_chunks_fn", None)
    if host_fn is not None and getattr(base, "iter_cols_fn", None) is not None:
        got = 0
        for ch in host_fn():  # the width (and the head rows) from the first host chunks
            Xh = torch.as_tensor(ch[features_col])
            d = int(Xh.shape[1])
            if got >= head_rows:
                break
            head.append(Xh[:head_rows - got].float().to(df._session.device))
            got += head[-1].shape[0]
        it = base.iter_cols_fn(list(cols))
        head_rows_left = 0
    else:
        host_fn = None
        it = sel._plan.iter_execute()
        head_rows_left = head_rows
    for b in it:
        if n < head_rows_left:
            head.append(b.columns[features_col].values[:head_rows_left - n].float().clone())
        for c in cols:
            cd = b.columns[c]
            if cd.valid is not None and not bool(cd.valid.all()):
                ok = False  # null labels / weights: the materialised path drops those rows
                break
            parts[c].append(cd.values.clone())  # the source reuses its chunk buffers
        if not ok:
            break
        if host_fn is None:
            d = int(b.columns[features_col].values.shape[1])
        n += b.n
    # the streamed and materialised paths issue different collectives, so every rank takes the same one: any
    # rank with nulls sends all of them to the materialised path; a rank with no chunks streams an empty shard
    # of the width the other ranks saw
    comm = df._session.comm
    if comm.distributed:
        ok = comm.all_reduce_scalar(1.0 if ok else 0.0, "min") > 0.5
        d = int(comm.all_reduce_scalar(float(-1 if d is None else d), "max"))
        d = None if d < 0 else d
    if not ok or d is None:
        return None
    dev = df._session.device
    out = {}
    for c in cols:
        f = sel.schema[c]
        v = torch.cat(parts[c]) if parts[c] else torch.zeros(0, device=dev)
        out[c] = ColumnData(v.to(dev), f.dataType)
    if head_rows:
        out["__head__"] = torch.cat(head).to(dev) if head else torch.zeros((0, d), device=dev)

    def chunks():
        r0 = 0
        for b in (sel._plan.iter_execute() if host_fn is None else base.iter_cols_fn([features_col])):
            X = b.columns[features_col].values
            yield r0, (X if X.dtype == torch.float32 else X.float())
            r0 += b.n

    def host_chunks():
        r0 = 0
        for ch in host_fn():
            X = torch.as_tensor(ch[features_col])
            yield r0, X
            r0 += X.shape[0]
    return (ChunkedRows(chunks, n, d, dev, host_it_fn=host_chunks if host_fn is not None else None), out,
            sel.schema[features_col].metadata)


GRAM_FP64_MAX_WORK = float(__import__("os").environ.get("CDNAML_GRAM_FP64_MAX_WORK", "4e9"))


def gram_fp64_auto(n: int, d: int) -> bool:
    """Course-sized Gram matrices (at most GRAM_FP64_MAX_WORK multiply-adds, n (d + 2)^2; d = 100: ~4e5 rows) take
    an fp64 library GEMM of the augmented fp32 rows -- Spark forms these statistics in Double and one-hot designs
    are ill-conditioned -- larger ones the K1 kernel (fp32 MFMA, HBM-bound)."""
    return float(n) * (d + 2) ** 2 <= GRAM_FP64_MAX_WORK


def centered_gram(X: torch.Tensor, comm, lead: int = 1024):
    """(n, mean[d], C[d, d]) over all ranks, C = sum (x - mean)(x - mean)^T, all fp64 (the Gram in fp64 arithmetic
    at course sizes: ``gram_fp64_auto``, so a feature standardisation equals the host's to rounding).

    The Gram kernel runs on features shifted by a common mean estimate (every rank's leading rows, averaged over
    the ranks that have any), so the second moments are formed about a point near the mean: E[x^2] - mean^2 of
    the raw fp32 columns cancels catastrophically for narrow, far-from-zero features (latitude: sd 0.02 about 37.8).
    """
    from ..ops import kernels as K
    n_loc, d = X.shape
    k = min(n_loc, lead)
    sh = X[:k].double().mean(0) if k else torch.zeros(d, dtype=torch.float64, device=X.device)
    if comm.distributed:
        cnt = torch.full((1,), 1.0 if k else 0.0, dtype=torch.float64, device=X.device)
        comm.all_reduce_many([sh, cnt])
        sh = sh / cnt.clamp_min(1.0)
    sh = sh.float()
    G = K.gram(X, shift=sh, fp64=X.dtype == torch.float64 or gram_fp64_auto(n_loc, d)) if n_loc else \
        torch.zeros((d + 2, d + 2), dtype=torch.float64, device=X.device)
    comm.all_reduce(G)
    n = float(G[d, d])
    s = G[:d, d]
    C = G[:d, :d] - torch.outer(s, s) / max(n, 1.0)
    return n, sh.double() + s / max(n, 1.0), C


def vector_attrs(meta: dict, width: int, name: str) -> List[dict]:
    """Per-slot attributes of a vector column (names, nominal arity)."""
    ma = (meta or {}).get("ml_attr")
    if ma and "attrs" in ma:
        attrs = list(ma["attrs"])
        if len(attrs) == width:
            return attrs
    return [{"idx": i, "name": f"{name}_{i}", "type": "numeric"} for i in range(width)]


def scalar_attr(meta: dict, name: str) -> dict:
    ma = (meta or {}).get("ml_attr")
    if ma and "type" in ma:
        a = dict(ma)
        a.setdefault("name", name)
        return a
    return {"name": name, "type": "numeric"}


def with_prediction(df, name: str, fn, out_type: T.DataType = None, meta_fn=None):
    """Append a column computed per partition by ``fn(batch) -> ColumnData``."""
    def per(b: Batch, ctx):
        c = fn(b)
        return b.with_column(name, c)
    return df._new(MapPlan(df._plan, f"Transform -> {name}", per))


def categorical_info(meta: dict, width: int, name: str) -> dict:
    """{feature index: arity} for nominal/binary vector slots (Spark categoricalFeaturesInfo)."""
    out = {}
    for i, a in enumerate(vector_attrs(meta, width, name)):
        t = a.get("type")
        if t == "nominal":
            k = a.get("num_vals") or (len(a["vals"]) if "vals" in a else None)
            if k:
                out[i] = int(k)
        elif t == "binary":
            out[i] = 2
    return out


def global_count(session, n_local: int) -> int:
    return int(session.comm.all_reduce_scalar(float(n_local)))


def global_offset(session, n_local: int) -> int:
    comm = session.comm
    if not comm.distributed:
        return 0
    counts = comm.all_gather_object(int(n_local))
    return int(sum(counts[: comm.rank]))
