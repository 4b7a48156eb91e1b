"""``pyspark.ml.stat``: Correlation and Summarizer over device feature matrices."""
import numpy as np
import pandas as pd
import torch

from ..models.linalg import DenseMatrix, DenseVector
from ..ops import kernels as K


class Correlation:
    @staticmethod
    def corr(dataset, column, method="pearson"):
        from ..models.util import local_xyw
        X, _, _ = local_xyw(dataset, column, keep_f64=True)
        if method == "spearman":
            X = torch.argsort(torch.argsort(X, 0), 0).float()
        from ..models.util import centered_gram
        _, _, C = centered_gram(X, dataset._session.comm)
        sd = torch.sqrt(torch.diagonal(C).clamp_min(1e-300))
        R = (C / torch.outer(sd, sd)).cpu().numpy()
        return _MatrixFrame(R, method, column)


class _MatrixFrame:
    """Tiny stand-in for the 1x1 DataFrame of a Matrix (head()[0] is the matrix)."""

    def __init__(self, R, method, column):
        self._m = DenseMatrix(R.shape[0], R.shape[1], R.T.reshape(-1))
        self.columns = [f"{method}({column})"]

    def head(self):
        return [self._m]

    def collect(self):
        return [[self._m]]


_METRICS = ("mean", "sum", "variance", "std", "count", "numNonZeros", "max", "min", "normL2", "normL1", "weightSum")


def _col_expr(col):
    from ..sql.column import ColRef, Column
    if isinstance(col, Column):
        return col._expr
    return ColRef(col)


class SummaryBuilder:
    """``Summarizer.metrics(...)``: ``summary(featuresCol, weightCol=None)`` is an aggregate Column whose value
    is a struct (Row) with one field per requested metric, in the requested order."""

    def __init__(self, names):
        bad = [m for m in names if m not in _METRICS]
        if bad or not names:
            raise ValueError(f"Summarizer metrics must be among {list(_METRICS)}, got {list(names)}")
        self.names = list(names)

    def summary(self, featuresCol, weightCol=None):
        from ..sql.column import Column
        from ..sql.functions import AggExpr
        x = _col_expr(featuresCol)
        w = None if weightCol is None else _col_expr(weightCol)
        disp = f"aggregate_metrics({x.name()}, {'1.0' if w is None else w.name()})"
        return Column(AggExpr("summarizer", x, param={"metrics": self.names, "weight": w, "single": False},
                              display=disp))


class Summarizer:
    """``pyspark.ml.stat.Summarizer``: vector-column statistics as aggregate expressions (usable in ``select``
    and ``groupBy().agg``).  Weighted semantics follow Spark's SummarizerBuffer: rows of weight 0 are skipped;
    ``count`` / ``numNonZeros`` count rows / non-zero entries, ``sum`` / ``mean`` / ``normL1`` / ``normL2`` are
    weighted, ``variance`` is the unbiased weighted variance (denominator W - sum(w^2) / W).  On the GPU the
    unweighted per-column moments come from K20 (``col_moments``: count, mean, M2, min, max in fp64)."""

    @staticmethod
    def metrics(*names):
        return SummaryBuilder(names)

    @staticmethod
    def _single(metric, col, weightCol=None):
        from ..sql.column import Column
        from ..sql.functions import AggExpr
        x = _col_expr(col)
        w = None if weightCol is None else _col_expr(weightCol)
        return Column(AggExpr("summarizer", x, param={"metrics": [metric], "weight": w, "single": True},
                              display=f"{metric}({x.name()})"))


for _m in _METRICS:
    setattr(Summarizer, _m, staticmethod(lambda col, weightCol=None, _m=_m: Summarizer._single(_m, col, weightCol)))


def _metric_values(X: torch.Tensor, w, metrics):
    """{metric: value} for one group's rows X [n, d] (fp64) and weights w [n] or None."""
    n, d = X.shape
    if w is not None:
        keep = w != 0
        X, w = X[keep], w[keep]
        n = X.shape[0]
    out = {}
    need_mom = any(m in metrics for m in ("mean", "variance", "std", "max", "min")) and w is None
    mom = K.col_moments(X) if need_mom else None  # K20 (count, mean, M2, min, max)
    W = float(n) if w is None else float(w.sum())
    for m in metrics:
        if m == "count":
            out[m] = int(n)
        elif m == "weightSum":
            out[m] = W
        elif m == "numNonZeros":
            out[m] = DenseVector((X != 0).sum(0).double().cpu().numpy())
        elif m in ("max", "min"):
            if n == 0:
                v = np.full(d, -np.inf if m == "max" else np.inf)
            elif mom is not None:
                v = mom[:, 4 if m == "max" else 3].cpu().numpy()
            else:
                v = (X.amax(0) if m == "max" else X.amin(0)).cpu().numpy()
            out[m] = DenseVector(v)
        elif m in ("sum", "mean", "normL1", "normL2"):
            ww = torch.ones(n, dtype=torch.float64, device=X.device) if w is None else w
            if m == "sum":
                v = (ww[:, None] * X).sum(0)
            elif m == "mean":
                v = mom[:, 1] if mom is not None else (ww[:, None] * X).sum(0) / (W if W > 0 else float("nan"))
            elif m == "normL1":
                v = (ww[:, None] * X.abs()).sum(0)
            else:
                v = torch.sqrt((ww[:, None] * X * X).sum(0))
            out[m] = DenseVector(v.cpu().numpy() if n else np.zeros(d))
        else:  # variance / std
            if w is None:
                v = (mom[:, 2] / (n - 1)) if n > 1 else torch.zeros(d, dtype=torch.float64)
            else:
                den = W - float((w * w).sum()) / W if W > 0 else 0.0
                mu = (w[:, None] * X).sum(0) / W if W > 0 else torch.zeros(d, dtype=torch.float64, device=X.device)
                v = (w[:, None] * (X - mu) ** 2).sum(0) / den if den > 0 else torch.zeros(d, dtype=torch.float64)
            v = v.clamp_min(0.0)
            out[m] = DenseVector((torch.sqrt(v) if m == "std" else v).cpu().numpy())
    return out


def summarize_groups(c, wcol, gid: torch.Tensor, G: int, param):
    """Group engine hook (relational._agg_one, kind "summarizer"): one struct Row (or, for a single metric, a
    vector / count column) per group."""
    from ..sql import types as T
    from ..sql.batch import ColumnData
    from ..sql.types import Row
    X = c.values
    if X.dim() == 1:
        X = X[:, None]
    X = X.to(torch.float64)
    if c.valid is not None:
        gid = gid[c.valid]
        X = X[c.valid]
    w = None if wcol is None else wcol.values.to(torch.float64)
    if w is not None and c.valid is not None:
        w = w[c.valid]
    metrics = param["metrics"]
    order = torch.argsort(gid, stable=True)
    counts = torch.bincount(gid, minlength=G).cpu().tolist() if gid.numel() else [0] * G
    Xs, ws = X[order], None if w is None else w[order]
    rows, r0 = [], 0
    for g in range(G):
        r1 = r0 + counts[g]
        rows.append(_metric_values(Xs[r0:r1], None if ws is None else ws[r0:r1], metrics))
        r0 = r1
    dev = c.values.device
    if param.get("single"):
        m = metrics[0]
        if m == "count":
            return ColumnData(torch.tensor([r[m] for r in rows], dtype=torch.int64, device=dev), T.LongType())
        if m == "weightSum":
            return ColumnData(torch.tensor([r[m] for r in rows], dtype=torch.float64, device=dev), T.DoubleType())
        d = X.shape[1]
        V = np.stack([r[m].toArray() for r in rows]) if rows else np.zeros((0, d))
        return ColumnData(torch.from_numpy(V).to(dev), T.VectorUDT())
    fields = [T.StructField(m, T.LongType() if m == "count" else T.DoubleType() if m == "weightSum"
                            else T.VectorUDT(), True) for m in metrics]
    structs = [Row(**{m: r[m] for m in metrics}) for r in rows]
    return ColumnData(torch.zeros(G, device=dev), T.StructType(fields), meta={"_py": structs})
