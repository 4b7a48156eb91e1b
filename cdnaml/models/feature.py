"""Feature transformers (SURVEY §2.5.2 F1–F5 and friends).

All transforms run per partition on device tensors.  String indexing works
on the dictionary codes of device string columns: the global label
frequencies are an all-gather of per-rank (value, count) maps (tiny), the
transform itself is a gather through a lookup table on the GPU.
"""
from __future__ import annotations

import math
import re
from typing import Dict, List, Optional

import numpy as np
import torch

from ..sql import types as T
from ..sql.batch import Batch, ColumnData
from ..sql.column import _cast
from ..sql.dataframe import MapPlan
from .base import Estimator, Model, Transformer
from .param import NO_DEFAULT, TypeConverters as TC, keyword_init
from .util import VECTOR_F64_MAX, IllegalArgumentException, local_batch, require_vector, scalar_attr, vector_attrs


class SparkException(RuntimeError):
    pass


def _in_out(self, single_in="inputCol", multi_in="inputCols", single_out="outputCol", multi_out="outputCols"):
    if self.isSet(multi_in):
        ins = list(self.getOrDefault(multi_in))
        outs = list(self.getOrDefault(multi_out)) if self.isSet(multi_out) else [f"{c}_out" for c in ins]
    else:
        ins = [self.getOrDefault(single_in)]
        outs = [self.getOrDefault(single_out)] if self.isDefined(single_out) else [f"{ins[0]}_out"]
    return ins, outs


# =========================================================== VectorAssembler
class VectorAssembler(Transformer):
    """Concatenate numeric / vector columns into one device feature matrix (ML 02:103-107)."""
    _params = {
        "inputCols": ("input column names", NO_DEFAULT, TC.toListString),
        "outputCol": ("output column name", "features", TC.toString),
        "handleInvalid": ("how to handle invalid data (NULL and NaN values): 'error', 'skip' or 'keep'",
                          "error", TC.toString),
    }

    def __init__(self, inputCols=None, outputCol=None, handleInvalid=None):
        super().__init__()
        keyword_init(self, dict(inputCols=inputCols, outputCol=outputCol, handleInvalid=handleInvalid))

    def _transform(self, dataset):
        ins = self.getInputCols()
        out = self.getOutputCol()
        hi = self.getHandleInvalid()
        for c in ins:
            if c not in dataset.columns:
                raise IllegalArgumentException(f"Field \"{c}\" does not exist.")
            dt = dataset.schema[c].dataType
            if isinstance(dt, T.StringType):
                raise IllegalArgumentException(
                    f"Data type string of column {c} is not supported.")

        prec = str(dataset._session.conf.get("cdnaml.ml.vectorPrecision", "auto")).lower()

        def out_dtype(b: Batch):
            """Spark's VectorUDT is Double: "auto" assembles fp64 unless an input is an fp32 matrix of real values
            (the benchmark's fp32 features, an fp32 stage's output: kept fp32, no 2x copy) or the batch exceeds
            ``util.VECTOR_F64_MAX`` elements (HBM-bound fp32 kernels from there on).  One-hot (binary) fp32 vectors
            are exact in either width.  conf ``cdnaml.ml.vectorPrecision``: auto | fp64 | fp32."""
            if prec in ("fp32", "float", "float32"):
                return torch.float32
            if prec in ("fp64", "double", "float64"):
                return torch.float64
            width = 0
            for c in ins:
                v = b.columns[c].values
                width += v.shape[1] if v.dim() == 2 else 1
                if v.dim() == 2 and v.dtype != torch.float64:
                    attrs_ = ((b.columns[c].meta or {}).get("ml_attr") or {}).get("attrs") or []
                    if not attrs_ or any(a.get("type") != "binary" for a in attrs_):
                        return torch.float32
            return torch.float64 if b.n * max(width, 1) <= VECTOR_F64_MAX else torch.float32

        def fn(b: Batch, ctx):
            mats, attrs = [], []
            bad = torch.zeros(b.n, dtype=torch.bool, device=b.device)
            vdt = out_dtype(b)
            for c in ins:
                col = b.columns[c]
                if col.values.dim() == 2:
                    m = col.values.to(vdt)
                    w = m.shape[1]
                    ma = (col.meta or {}).get("ml_attr", {})
                    if w == 0 and ma.get("num_attrs"):
                        w = int(ma["num_attrs"])
                        m = torch.zeros((b.n, w), dtype=vdt, device=b.device)
                    for a in vector_attrs(col.meta, w, c):
                        a = dict(a)
                        a["name"] = f"{c}_{a['name']}" if not str(a.get("name", "")).startswith(c) else a["name"]
                        attrs.append(a)
                else:
                    m = col.values.to(vdt)[:, None]
                    a = scalar_attr(col.meta, c)
                    a["name"] = c
                    attrs.append(a)
                if col.valid is not None:
                    bad |= ~col.valid
                if m.numel():
                    bad |= torch.isnan(m).any(1)
                mats.append(m)
            X = torch.cat(mats, 1) if mats else torch.zeros((b.n, 0), dtype=vdt, device=b.device)
            for i, a in enumerate(attrs):
                a["idx"] = i
            meta = {"ml_attr": {"attrs": attrs, "num_attrs": len(attrs)}}
            nb = b
            if bool(bad.any()):
                if hi == "error":
                    raise SparkException(
                        "Encountered null while assembling a row with handleInvalid = \"error\". Consider removing "
                        "nulls from dataset or using handleInvalid = \"keep\" or \"skip\".")
                if hi == "skip":
                    keep = ~bad
                    nb = b.filter(keep)
                    X = X[keep]
                else:
                    X = torch.where(torch.isnan(X), X, X)
            return nb.with_column(out, ColumnData(X.contiguous(), T.VectorUDT(), None, meta=meta))
        return dataset._new(MapPlan(dataset._plan, f"VectorAssembler -> {out}", fn))


# ============================================================= StringIndexer
def _label_counts(df, col) -> Dict[str, int]:
    b = local_batch(df, [col])
    c = b.columns[col]
    if not isinstance(c.dtype, T.StringType):
        c = _cast(c, T.StringType())
    d = c.dictionary if c.dictionary is not None else np.array([], dtype=object)
    codes = c.values.long()
    ok = codes >= 0
    if c.valid is not None:
        ok &= c.valid
    cnt = torch.bincount(codes[ok], minlength=len(d)).cpu().numpy() if len(d) else np.zeros(0, np.int64)
    local = {str(v): int(n) for v, n in zip(d.tolist(), cnt.tolist()) if n > 0}
    comm = df._session.comm
    if comm.distributed:
        merged: Dict[str, int] = {}
        for m in comm.all_gather_object(local):
            for k, v in m.items():
                merged[k] = merged.get(k, 0) + v
        return merged
    return local


def _order_labels(counts: Dict[str, int], order: str) -> List[str]:
    items = list(counts.items())
    if order == "frequencyDesc":
        items.sort(key=lambda kv: (-kv[1], kv[0]))
    elif order == "frequencyAsc":
        items.sort(key=lambda kv: (kv[1], kv[0]))
    elif order == "alphabetDesc":
        items.sort(key=lambda kv: kv[0], reverse=True)
    elif order == "alphabetAsc":
        items.sort(key=lambda kv: kv[0])
    else:
        raise IllegalArgumentException(f"unknown stringOrderType {order}")
    return [k for k, _ in items]


class StringIndexer(Estimator):
    """Label -> index by frequency (ML 03:60; handleInvalid="skip" drops rows)."""
    _params = {
        "inputCol": ("input column name", NO_DEFAULT, TC.toString),
        "outputCol": ("output column name", NO_DEFAULT, TC.toString),
        "inputCols": ("input column names", NO_DEFAULT, TC.toListString),
        "outputCols": ("output column names", NO_DEFAULT, TC.toListString),
        "handleInvalid": ("how to handle invalid data (unseen or NULL values): 'skip', 'error' or 'keep'",
                          "error", TC.toString),
        "stringOrderType": ("how to order labels: frequencyDesc, frequencyAsc, alphabetDesc, alphabetAsc",
                            "frequencyDesc", TC.toString),
    }

    def __init__(self, inputCol=None, outputCol=None, inputCols=None, outputCols=None, handleInvalid=None,
                 stringOrderType=None):
        super().__init__()
        keyword_init(self, dict(inputCol=inputCol, outputCol=outputCol, inputCols=inputCols,
                                outputCols=outputCols, handleInvalid=handleInvalid,
                                stringOrderType=stringOrderType))

    def _fit(self, dataset):
        ins, outs = _in_out(self)
        labels = [_order_labels(_label_counts(dataset, c), self.getStringOrderType()) for c in ins]
        m = StringIndexerModel(labelsArray=labels)
        return m


class StringIndexerModel(Model):
    _params = StringIndexer._params

    def __init__(self, labelsArray=None, labels=None):
        super().__init__()
        self.labelsArray = labelsArray or ([labels] if labels is not None else [])

    @classmethod
    def from_labels(cls, labels, inputCol, outputCol=None, handleInvalid=None):
        m = cls(labels=list(labels))
        m.set("inputCol", inputCol)
        m.set("outputCol", outputCol or f"{inputCol}_index")
        if handleInvalid:
            m.set("handleInvalid", handleInvalid)
        return m

    @property
    def labels(self):
        return self.labelsArray[0]

    def _transform(self, dataset):
        ins, outs = _in_out(self)
        hi = self.getHandleInvalid()
        labels_arr = self.labelsArray

        def fn(b: Batch, ctx):
            drop = torch.zeros(b.n, dtype=torch.bool, device=b.device)
            newcols = {}
            for c, o, labels in zip(ins, outs, labels_arr):
                col = b.columns[c]
                if not isinstance(col.dtype, T.StringType):
                    col = _cast(col, T.StringType())
                d = col.dictionary if col.dictionary is not None else np.array([], dtype=object)
                pos = {v: i for i, v in enumerate(labels)}
                lut = np.array([pos.get(v, -1) for v in d.tolist()] + [-1], dtype=np.float64)
                lut_t = torch.from_numpy(lut).to(b.device)
                codes = col.values.long()
                codes = torch.where(codes < 0, torch.full_like(codes, len(d)), codes)
                idx = lut_t[codes]
                invalid = idx < 0
                if col.valid is not None:
                    invalid |= ~col.valid
                if bool(invalid.any()):
                    if hi == "error":
                        bad = col.take(torch.nonzero(invalid).flatten()[:1]).to_pylist()[0]
                        if bad is None:
                            raise SparkException(f"Failed to execute user defined function(StringIndexerModel): "
                                                 f"StringIndexer encountered NULL value. To handle or skip NULLS, "
                                                 f"try setting StringIndexer.handleInvalid.")
                        raise SparkException(f"Unseen label: {bad}. To handle unseen labels, set Param "
                                             f"handleInvalid to keep.")
                    if hi == "skip":
                        drop |= invalid
                    else:
                        idx = torch.where(invalid, torch.full_like(idx, float(len(labels))), idx)
                vals = list(labels) + (["__unknown"] if hi == "keep" else [])
                meta = {"ml_attr": {"type": "nominal", "name": o, "vals": vals, "num_vals": len(vals)}}
                newcols[o] = ColumnData(idx, T.DoubleType(), None, meta=meta)
            nb = b
            for o, cd in newcols.items():
                nb = nb.with_column(o, cd)
            if bool(drop.any()):
                nb = nb.filter(~drop)
            return nb
        return dataset._new(MapPlan(dataset._plan, f"StringIndexerModel {ins}->{outs}", fn))

    def _save_state(self):
        return {"labelsArray": self.labelsArray}, {}

    def _load_state(self, extra, tensors, stages):
        self.labelsArray = extra["labelsArray"]


class IndexToString(Transformer):
    _params = {
        "inputCol": ("input column name", NO_DEFAULT, TC.toString),
        "outputCol": ("output column name", NO_DEFAULT, TC.toString),
        "labels": ("ordered labels", None, None),
    }

    def __init__(self, inputCol=None, outputCol=None, labels=None):
        super().__init__()
        keyword_init(self, dict(inputCol=inputCol, outputCol=outputCol, labels=labels))

    def _transform(self, dataset):
        ic, oc = self.getInputCol(), self.getOutputCol()
        labels = self.getLabels()

        def fn(b, ctx):
            col = b.columns[ic]
            labs = labels or (col.meta.get("ml_attr", {}).get("vals") if col.meta else None)
            if labs is None:
                raise IllegalArgumentException("IndexToString needs labels (param or nominal metadata)")
            idx = col.values.long().clamp(0, len(labs) - 1)
            return b.with_column(oc, ColumnData(idx.to(torch.int32), T.StringType(), col.valid,
                                                np.asarray(labs, dtype=object)))
        return dataset._new(MapPlan(dataset._plan, "IndexToString", fn))


# ============================================================ OneHotEncoder
class OneHotEncoder(Estimator):
    """Index -> one-hot vector, last category dropped by default (ML 03:50-61)."""
    _params = {
        "inputCol": ("input column name", NO_DEFAULT, TC.toString),
        "outputCol": ("output column name", NO_DEFAULT, TC.toString),
        "inputCols": ("input column names", NO_DEFAULT, TC.toListString),
        "outputCols": ("output column names", NO_DEFAULT, TC.toListString),
        "dropLast": ("whether to drop the last category", True, TC.toBoolean),
        "handleInvalid": ("how to handle invalid data: 'keep' or 'error'", "error", TC.toString),
    }

    def __init__(self, inputCols=None, outputCols=None, inputCol=None, outputCol=None, dropLast=None,
                 handleInvalid=None):
        super().__init__()
        keyword_init(self, dict(inputCols=inputCols, outputCols=outputCols, inputCol=inputCol,
                                outputCol=outputCol, dropLast=dropLast, handleInvalid=handleInvalid))

    def _fit(self, dataset):
        ins, outs = _in_out(self)
        sizes, labels = [], []
        sch = dataset.schema
        need = []
        for c in ins:
            if not (sch[c].dataType.is_numeric):
                raise IllegalArgumentException(f"requirement failed: Column {c} must be of type numeric but "
                                               f"was actually of type {sch[c].dataType.simpleString()}.")
            ma = (sch[c].metadata or {}).get("ml_attr", {})
            if ma.get("type") == "nominal" and ma.get("num_vals"):
                sizes.append(int(ma["num_vals"]))
                labels.append(list(ma.get("vals", [])))
            else:
                sizes.append(None)
                labels.append(None)
                need.append(c)
        if need:
            from ..sql import functions as F
            mx = dataset.agg(*[F.max(F.col(c)).alias(c) for c in need]).collect()[0]
            for i, c in enumerate(ins):
                if sizes[i] is None:
                    v = mx[c]
                    sizes[i] = int(v) + 1 if v is not None else 0
        m = OneHotEncoderModel(categorySizes=sizes, labels=labels)
        return m


class OneHotEncoderModel(Model):
    _params = OneHotEncoder._params

    def __init__(self, categorySizes=None, labels=None):
        super().__init__()
        self.categorySizes = list(categorySizes or [])
        self._labels = labels or [None] * len(self.categorySizes)

    def _out_meta(self, c, size, labels, keep, drop_last):
        k = size + (1 if keep else 0) - (1 if drop_last else 0)
        names = []
        for j in range(k):
            if labels and j < len(labels):
                names.append(f"{labels[j]}")
            elif keep and j == size:
                names.append("__unknown")
            else:
                names.append(str(j))
        attrs = [{"idx": j, "name": f"{c}_{n}", "type": "binary"} for j, n in enumerate(names)]
        return {"ml_attr": {"attrs": attrs, "num_attrs": k}}

    def _transform(self, dataset):
        ins, outs = _in_out(self)
        drop_last = self.getDropLast()
        keep = self.getHandleInvalid() == "keep"
        sizes = self.categorySizes
        labels = self._labels

        def fn(b: Batch, ctx):
            nb = b
            for c, o, size, labs in zip(ins, outs, sizes, labels):
                col = b.columns[c]
                v = col.values.to(torch.float64)
                k = size + (1 if keep else 0) - (1 if drop_last else 0)
                idx = v.long()
                invalid = (v != idx.double()) | (idx < 0) | (idx >= size)
                if col.valid is not None:
                    invalid |= ~col.valid
                if bool(invalid.any()):
                    if not keep:
                        raise SparkException(f"Invalid values found in column {c}: one-hot encoding expects "
                                             f"indices in [0, {size}). Set handleInvalid to 'keep'.")
                    idx = torch.where(invalid, torch.full_like(idx, size), idx)
                M = torch.zeros((b.n, max(k, 0)), dtype=torch.float32, device=b.device)
                ok = idx < k
                if b.n and k > 0:
                    rows = torch.arange(b.n, device=b.device)[ok]
                    M[rows, idx[ok]] = 1.0
                nb = nb.with_column(o, ColumnData(M, T.VectorUDT(), None,
                                                  meta=self._out_meta(c, size, labs, keep, drop_last)))
            return nb
        return dataset._new(MapPlan(dataset._plan, f"OneHotEncoderModel {ins}->{outs}", fn))

    def _save_state(self):
        return {"categorySizes": self.categorySizes, "labels": self._labels}, {}

    def _load_state(self, extra, tensors, stages):
        self.categorySizes = extra["categorySizes"]
        self._labels = extra.get("labels") or [None] * len(self.categorySizes)


# ================================================================== Imputer
class Imputer(Estimator):
    """Fill missing numeric values with mean/median/mode (ML 01:194-256)."""
    _params = {
        "inputCol": ("input column name", NO_DEFAULT, TC.toString),
        "outputCol": ("output column name", NO_DEFAULT, TC.toString),
        "inputCols": ("input column names", NO_DEFAULT, TC.toListString),
        "outputCols": ("output column names", NO_DEFAULT, TC.toListString),
        "strategy": ("strategy for imputation: mean, median or mode", "mean", TC.toString),
        "missingValue": ("placeholder for the missing values", float("nan"), TC.toFloat),
        "relativeError": ("relative error for approximate median", 0.001, TC.toFloat),
    }

    def __init__(self, strategy=None, missingValue=None, inputCols=None, outputCols=None, inputCol=None,
                 outputCol=None, relativeError=None):
        super().__init__()
        keyword_init(self, dict(strategy=strategy, missingValue=missingValue, inputCols=inputCols,
                                outputCols=outputCols, inputCol=inputCol, outputCol=outputCol,
                                relativeError=relativeError))

    def _fit(self, dataset):
        from ..sql import functions as F
        ins, outs = _in_out(self)
        mv = self.getMissingValue()
        strat = self.getStrategy()
        for c in ins:
            dt = dataset.schema[c].dataType
            if not dt.is_numeric:
                raise IllegalArgumentException(f"requirement failed: Column {c} must be of type numeric but "
                                               f"was actually of type {dt.simpleString()}.")
        surrogates = {}
        for c in ins:
            v_ = F.col("__v")
            cond = v_.isNotNull() & ~F.isnan(v_)
            if not math.isnan(mv):
                cond = cond & (v_ != mv)
            sel = dataset.select(F.col(c).cast("double").alias("__v")).filter(cond)
            if strat == "mean":
                v = sel.agg(F.avg("__v")).collect()[0][0]
            elif strat == "median":
                q = sel.approxQuantile("__v", [0.5], self.getRelativeError())
                v = q[0] if q else None
            elif strat == "mode":
                r = sel.groupBy("__v").count().orderBy(F.col("count").desc(), F.col("__v")).limit(1).collect()
                v = r[0][0] if r else None
            else:
                raise IllegalArgumentException(f"unknown strategy {strat}")
            if v is None:
                raise SparkException(f"surrogate cannot be computed. All the values in {c} are Null, Nan or "
                                     f"missingValue({mv})")
            surrogates[c] = float(v)
        return ImputerModel(surrogates=surrogates)


class ImputerModel(Model):
    _params = Imputer._params

    def __init__(self, surrogates=None):
        super().__init__()
        self.surrogates = dict(surrogates or {})

    @property
    def surrogateDF(self):
        from ..session import SparkSession
        import pandas as pd
        s = SparkSession.getActiveSession()
        return s.createDataFrame(pd.DataFrame({k: [v] for k, v in self.surrogates.items()}))

    def _transform(self, dataset):
        ins, outs = _in_out(self)
        mv = self.getMissingValue()
        sur = self.surrogates

        def fn(b, ctx):
            nb = b
            for c, o in zip(ins, outs):
                col = b.columns[c]
                v = col.values.to(torch.float64)
                miss = torch.isnan(v) if math.isnan(mv) else (v == mv) | torch.isnan(v)
                if col.valid is not None:
                    miss |= ~col.valid
                out = torch.where(miss, torch.full_like(v, sur[c]), v)
                if isinstance(col.dtype, T.FloatType):
                    nb = nb.with_column(o, ColumnData(out.float(), T.FloatType(), None, meta=col.meta))
                elif isinstance(col.dtype, T.IntegralType):
                    nb = nb.with_column(o, ColumnData(out.to(col.values.dtype), col.dtype, None, meta=col.meta))
                else:
                    nb = nb.with_column(o, ColumnData(out, T.DoubleType(), None, meta=col.meta))
            return nb
        return dataset._new(MapPlan(dataset._plan, "ImputerModel", fn))

    def _save_state(self):
        return {"surrogates": self.surrogates}, {}

    def _load_state(self, extra, tensors, stages):
        self.surrogates = extra["surrogates"]


# ================================================================= RFormula
class RFormula(Estimator):
    """R model formula -> features/label (Labs/ML 03L:35-37; ML 04:114)."""
    _params = {
        "formula": ("R model formula", NO_DEFAULT, TC.toString),
        "featuresCol": ("features column name", "features", TC.toString),
        "labelCol": ("label column name", "label", TC.toString),
        "forceIndexLabel": ("force to index label whether it is numeric or string", False, TC.toBoolean),
        "handleInvalid": ("how to handle invalid data: 'skip', 'error' or 'keep'", "error", TC.toString),
        "stringIndexerOrderType": ("string order type", "frequencyDesc", TC.toString),
    }

    def __init__(self, formula=None, featuresCol=None, labelCol=None, forceIndexLabel=None, handleInvalid=None,
                 stringIndexerOrderType=None):
        super().__init__()
        keyword_init(self, dict(formula=formula, featuresCol=featuresCol, labelCol=labelCol,
                                forceIndexLabel=forceIndexLabel, handleInvalid=handleInvalid,
                                stringIndexerOrderType=stringIndexerOrderType))

    @staticmethod
    def parse(formula: str, columns: List[str]):
        if "~" not in formula:
            raise IllegalArgumentException(f"Invalid formula: {formula}")
        lhs, rhs = [s.strip() for s in formula.split("~", 1)]
        terms: List[str] = []
        removed = set()
        tokens = re.findall(r"[+-]?\s*[^+-]+", rhs)
        for tok in tokens:
            tok = tok.strip()
            sign = "-" if tok.startswith("-") else "+"
            name = tok.lstrip("+-").strip()
            if name in ("1", "0"):
                continue
            if name == ".":
                names = [c for c in columns if c != lhs]
            else:
                names = [name]
            for n in names:
                if sign == "-":
                    removed.add(n)
                elif n not in terms:
                    terms.append(n)
        return lhs, [t for t in terms if t not in removed]

    def _fit(self, dataset):
        from .pipeline import Pipeline
        label, terms = self.parse(self.getFormula(), dataset.columns)
        sch = dataset.schema
        hi = self.getHandleInvalid()
        stages, assembled = [], []
        str_terms = [t for t in terms if isinstance(sch[t].dataType, T.StringType)]
        if str_terms:
            idx_out = [f"{t}_idx_{self.uid[-6:]}" for t in str_terms]
            ohe_out = [f"{t}_ohe_{self.uid[-6:]}" for t in str_terms]
            stages.append(StringIndexer(inputCols=str_terms, outputCols=idx_out,
                                        handleInvalid="keep" if hi == "keep" else hi,
                                        stringOrderType=self.getStringIndexerOrderType()))
            stages.append(OneHotEncoder(inputCols=idx_out, outputCols=ohe_out, dropLast=True,
                                        handleInvalid="keep" if hi == "keep" else "error"))
        for t in terms:
            if t in str_terms:
                assembled.append(f"{t}_ohe_{self.uid[-6:]}")
            else:
                assembled.append(t)
        stages.append(VectorAssembler(inputCols=assembled, outputCol=self.getFeaturesCol(),
                                      handleInvalid=hi if hi != "error" else "error"))
        label_indexer = None
        if label in dataset.columns and (isinstance(sch[label].dataType, T.StringType) or
                                         self.getForceIndexLabel()):
            label_indexer = StringIndexer(inputCol=label, outputCol=self.getLabelCol(), handleInvalid=hi)
            stages.insert(0, label_indexer)
        pm = Pipeline(stages=stages).fit(dataset)
        m = RFormulaModel(pipelineModel=pm, label=label, terms=terms,
                          tmp_cols=[c for t in str_terms for c in (f"{t}_idx_{self.uid[-6:]}",
                                                                   f"{t}_ohe_{self.uid[-6:]}")],
                          label_indexed=label_indexer is not None)
        return m


class RFormulaModel(Model):
    _params = RFormula._params

    def __init__(self, pipelineModel=None, label=None, terms=None, tmp_cols=None, label_indexed=False):
        super().__init__()
        self.pipelineModel = pipelineModel
        self.label = label
        self.terms = terms or []
        self.tmp_cols = tmp_cols or []
        self.label_indexed = label_indexed

    def _transform(self, dataset):
        df = dataset
        stages = self.pipelineModel.stages
        has_label = self.label in dataset.columns
        for s in stages:
            if isinstance(s, StringIndexerModel) and s.isSet("inputCol") and s.getInputCol() == self.label and \
                    not has_label:
                continue
            df = s.transform(df)
        if has_label and not self.label_indexed and self.getLabelCol() != self.label:
            from ..sql import functions as F
            df = df.withColumn(self.getLabelCol(), F.col(self.label).cast("double"))
        elif has_label and not self.label_indexed:
            from ..sql import functions as F
            if not isinstance(df.schema[self.label].dataType, T.DoubleType):
                df = df.withColumn(self.label, F.col(self.label).cast("double"))
        if self.tmp_cols:
            df = df.drop(*self.tmp_cols)
        return df

    def _sub_stages(self):
        return [self.pipelineModel]

    def _save_state(self):
        return {"label": self.label, "terms": self.terms, "tmp_cols": self.tmp_cols,
                "label_indexed": self.label_indexed}, {}

    def _load_state(self, extra, tensors, stages):
        self.pipelineModel = stages[0]
        self.label = extra["label"]
        self.terms = extra["terms"]
        self.tmp_cols = extra["tmp_cols"]
        self.label_indexed = extra["label_indexed"]


# ============================================================ scalers etc.
class StandardScaler(Estimator):
    _params = {
        "inputCol": ("input column name", NO_DEFAULT, TC.toString),
        "outputCol": ("output column name", NO_DEFAULT, TC.toString),
        "withMean": ("center data with mean", False, TC.toBoolean),
        "withStd": ("scale to unit standard deviation", True, TC.toBoolean),
    }

    def __init__(self, withMean=None, withStd=None, inputCol=None, outputCol=None):
        super().__init__()
        keyword_init(self, dict(withMean=withMean, withStd=withStd, inputCol=inputCol, outputCol=outputCol))

    def _fit(self, dataset):
        from .util import centered_gram, local_xyw
        X, _, _ = local_xyw(dataset, self.getInputCol(), keep_f64=True)
        n, mean, C = centered_gram(X, dataset._session.comm)
        var = torch.diagonal(C) / max(n - 1, 1)
        return StandardScalerModel(mean=mean.cpu().numpy(), std=torch.sqrt(var.clamp_min(0)).cpu().numpy())


class StandardScalerModel(Model):
    _params = StandardScaler._params

    def __init__(self, mean=None, std=None):
        super().__init__()
        self._mean = np.asarray(mean if mean is not None else [], dtype=np.float64)
        self._std = np.asarray(std if std is not None else [], dtype=np.float64)

    @property
    def mean(self):
        from .linalg import DenseVector
        return DenseVector(self._mean)

    @property
    def std(self):
        from .linalg import DenseVector
        return DenseVector(self._std)

    def _transform(self, dataset):
        ic, oc = self.getInputCol(), self.getOutputCol()
        wm, ws = self.getWithMean(), self.getWithStd()
        mu = torch.tensor(self._mean, dtype=torch.float64)
        sd = torch.tensor(np.where(self._std > 0, self._std, 1.0), dtype=torch.float64)
        zero = torch.tensor(self._std == 0)

        def fn(b, ctx):
            X = b.columns[ic].values
            X = X if X.dtype == torch.float64 else X.float()   # Double vectors stay Double
            if X.shape[0] == 0:
                X = X.new_zeros((0, len(mu)))
            Y = X
            if wm:
                Y = Y - mu.to(b.device, X.dtype)
            if ws:
                Y = Y / sd.to(b.device, X.dtype)
                Y = torch.where(zero.to(b.device)[None, :], torch.zeros_like(Y), Y)
            return b.with_column(oc, ColumnData(Y, T.VectorUDT(), b.columns[ic].valid, meta=b.columns[ic].meta))
        return dataset._new(MapPlan(dataset._plan, "StandardScalerModel", fn))

    def _save_state(self):
        return {}, {"mean": torch.tensor(self._mean), "std": torch.tensor(self._std)}

    def _load_state(self, extra, tensors, stages):
        self._mean = tensors["mean"].numpy()
        self._std = tensors["std"].numpy()


class MinMaxScaler(Estimator):
    _params = {
        "inputCol": ("input column name", NO_DEFAULT, TC.toString),
        "outputCol": ("output column name", NO_DEFAULT, TC.toString),
        "min": ("lower bound of output", 0.0, TC.toFloat),
        "max": ("upper bound of output", 1.0, TC.toFloat),
    }

    def __init__(self, min=None, max=None, inputCol=None, outputCol=None):  # noqa: A002
        super().__init__()
        keyword_init(self, dict(min=min, max=max, inputCol=inputCol, outputCol=outputCol))

    def _fit(self, dataset):
        from .util import local_xyw
        X, _, _ = local_xyw(dataset, self.getInputCol(), keep_f64=True)
        comm = dataset._session.comm
        lo = X.min(0).values.double() if X.shape[0] else torch.full((X.shape[1],), float("inf"), device=X.device,
                                                                    dtype=torch.float64)
        hi = X.max(0).values.double() if X.shape[0] else torch.full((X.shape[1],), float("-inf"), device=X.device,
                                                                    dtype=torch.float64)
        comm.all_reduce(lo, "min")
        comm.all_reduce(hi, "max")
        return MinMaxScalerModel(lo.cpu().numpy(), hi.cpu().numpy())


class MinMaxScalerModel(Model):
    _params = MinMaxScaler._params

    def __init__(self, originalMin=None, originalMax=None):
        super().__init__()
        self._lo = np.asarray(originalMin if originalMin is not None else [], np.float64)
        self._hi = np.asarray(originalMax if originalMax is not None else [], np.float64)

    @property
    def originalMin(self):
        from .linalg import DenseVector
        return DenseVector(self._lo)

    @property
    def originalMax(self):
        from .linalg import DenseVector
        return DenseVector(self._hi)

    def _transform(self, dataset):
        ic, oc = self.getInputCol(), self.getOutputCol()
        a, z = self.getMin(), self.getMax()
        lo = torch.tensor(self._lo, dtype=torch.float64)
        rng = torch.tensor(self._hi - self._lo, dtype=torch.float64)

        def fn(b, ctx):
            X = b.columns[ic].values
            X = X if X.dtype == torch.float64 else X.float()
            r = rng.to(b.device, X.dtype)
            scaled = torch.where(r[None, :] != 0, (X - lo.to(b.device, X.dtype)) / torch.where(r != 0, r, torch.ones_like(r)),
                                 torch.full_like(X, 0.5))
            return b.with_column(oc, ColumnData(scaled * (z - a) + a, T.VectorUDT()))
        return dataset._new(MapPlan(dataset._plan, "MinMaxScalerModel", fn))

    def _save_state(self):
        return {}, {"lo": torch.tensor(self._lo), "hi": torch.tensor(self._hi)}

    def _load_state(self, extra, tensors, stages):
        self._lo, self._hi = tensors["lo"].numpy(), tensors["hi"].numpy()


class Bucketizer(Transformer):
    _params = {
        "splits": ("split points", NO_DEFAULT, TC.toListFloat),
        "inputCol": ("input column name", NO_DEFAULT, TC.toString),
        "outputCol": ("output column name", NO_DEFAULT, TC.toString),
        "handleInvalid": ("'skip', 'error' or 'keep'", "error", TC.toString),
    }

    def __init__(self, splits=None, inputCol=None, outputCol=None, handleInvalid=None):
        super().__init__()
        keyword_init(self, dict(splits=splits, inputCol=inputCol, outputCol=outputCol, handleInvalid=handleInvalid))

    def _transform(self, dataset):
        ic, oc = self.getInputCol(), self.getOutputCol()
        sp = torch.tensor(self.getSplits(), dtype=torch.float64)
        hi = self.getHandleInvalid()

        def fn(b, ctx):
            x = b.columns[ic].values.double()
            s = sp.to(b.device)
            idx = torch.searchsorted(s, x, right=True) - 1
            idx = torch.where(x == s[-1], torch.full_like(idx, len(s) - 2), idx)
            bad = torch.isnan(x) | (idx < 0) | (idx > len(s) - 2)
            out = idx.double()
            nb = b
            if bool(bad.any()):
                if hi == "error":
                    raise SparkException("Bucketizer found NaN or out-of-range values; set handleInvalid")
                if hi == "keep":
                    out = torch.where(bad, torch.full_like(out, float(len(s) - 1)), out)
                else:
                    nb = b.filter(~bad)
                    out = out[~bad]
            return nb.with_column(oc, ColumnData(out, T.DoubleType()))
        return dataset._new(MapPlan(dataset._plan, "Bucketizer", fn))


class QuantileDiscretizer(Estimator):
    _params = {
        "numBuckets": ("number of buckets", 2, TC.toInt),
        "inputCol": ("input column name", NO_DEFAULT, TC.toString),
        "outputCol": ("output column name", NO_DEFAULT, TC.toString),
        "relativeError": ("relative error", 0.001, TC.toFloat),
        "handleInvalid": ("'skip', 'error' or 'keep'", "error", TC.toString),
    }

    def __init__(self, numBuckets=None, inputCol=None, outputCol=None, relativeError=None, handleInvalid=None):
        super().__init__()
        keyword_init(self, dict(numBuckets=numBuckets, inputCol=inputCol, outputCol=outputCol,
                                relativeError=relativeError, handleInvalid=handleInvalid))

    def _fit(self, dataset):
        k = self.getNumBuckets()
        qs = dataset.approxQuantile(self.getInputCol(), [i / k for i in range(1, k)], self.getRelativeError())
        splits = [-float("inf")] + sorted(set(qs)) + [float("inf")]
        return Bucketizer(splits=splits, inputCol=self.getInputCol(), outputCol=self.getOutputCol(),
                          handleInvalid=self.getHandleInvalid())


class SQLTransformer(Transformer):
    _params = {"statement": ("SQL statement with __THIS__ placeholder", NO_DEFAULT, TC.toString)}

    def __init__(self, statement=None):
        super().__init__()
        keyword_init(self, dict(statement=statement))

    def _transform(self, dataset):
        name = f"__this_{self.uid[-8:]}"
        dataset.createOrReplaceTempView(name)
        return dataset._session.sql(self.getStatement().replace("__THIS__", name))


class Normalizer(Transformer):
    _params = {
        "p": ("the p norm value", 2.0, TC.toFloat),
        "inputCol": ("input column name", NO_DEFAULT, TC.toString),
        "outputCol": ("output column name", NO_DEFAULT, TC.toString),
    }

    def __init__(self, p=None, inputCol=None, outputCol=None):
        super().__init__()
        keyword_init(self, dict(p=p, inputCol=inputCol, outputCol=outputCol))

    def _transform(self, dataset):
        ic, oc, p = self.getInputCol(), self.getOutputCol(), self.getP()

        def fn(b, ctx):
            X = b.columns[ic].values.float()
            nrm = torch.linalg.vector_norm(X, ord=p, dim=1, keepdim=True)
            return b.with_column(oc, ColumnData(X / torch.where(nrm > 0, nrm, torch.ones_like(nrm)), T.VectorUDT()))
        return dataset._new(MapPlan(dataset._plan, "Normalizer", fn))


class PCA(Estimator):
    """Principal components from the MFMA Gram kernel (one data pass + host eigh)."""
    _params = {
        "k": ("number of principal components", NO_DEFAULT, TC.toInt),
        "inputCol": ("input column name", NO_DEFAULT, TC.toString),
        "outputCol": ("output column name", NO_DEFAULT, TC.toString),
    }

    def __init__(self, k=None, inputCol=None, outputCol=None):
        super().__init__()
        keyword_init(self, dict(k=k, inputCol=inputCol, outputCol=outputCol))

    def _fit(self, dataset):
        from .util import centered_gram, local_xyw
        X, _, _ = local_xyw(dataset, self.getInputCol(), keep_f64=True)
        n, _, C = centered_gram(X, dataset._session.comm)
        cov = C / max(n - 1, 1)
        w, v = torch.linalg.eigh(cov.cpu())
        order = torch.argsort(w, descending=True)[: self.getK()]
        pc = v[:, order].numpy()
        ev = (w[order] / w.clamp_min(0).sum()).numpy()
        return PCAModel(pc, ev)


class PCAModel(Model):
    _params = PCA._params

    def __init__(self, pc=None, explained=None):
        super().__init__()
        self._pc = np.asarray(pc if pc is not None else np.zeros((0, 0)))
        self._ev = np.asarray(explained if explained is not None else [])

    @property
    def pc(self):
        from .linalg import DenseMatrix
        return DenseMatrix(self._pc.shape[0], self._pc.shape[1], self._pc.T.reshape(-1))

    @property
    def explainedVariance(self):
        from .linalg import DenseVector
        return DenseVector(self._ev)

    def _transform(self, dataset):
        ic, oc = self.getInputCol(), self.getOutputCol()
        P = torch.tensor(self._pc, dtype=torch.float64)

        def fn(b, ctx):
            X = b.columns[ic].values
            X = X if X.dtype == torch.float64 else X.float()
            return b.with_column(oc, ColumnData(X @ P.to(b.device, X.dtype), T.VectorUDT()))
        return dataset._new(MapPlan(dataset._plan, "PCAModel", fn))

    def _save_state(self):
        return {}, {"pc": torch.tensor(self._pc), "ev": torch.tensor(self._ev)}

    def _load_state(self, extra, tensors, stages):
        self._pc, self._ev = tensors["pc"].numpy(), tensors["ev"].numpy()
