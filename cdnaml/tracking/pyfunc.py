"""Generic python_function flavor: ``load_model(uri).predict(X)`` and
``spark_udf(spark, uri)`` (ML 09 - AutoML.py:78-82; Labs/ML 12L:78-96).

For models of this framework ``spark_udf`` returns a device-native UDF: each
partition is wrapped as a DataFrame and run through the loaded
PipelineModel's native kernels (no pandas round trip).  Foreign models
(scikit-learn) take the Arrow-batch pandas path, loaded once per process.
"""
from __future__ import annotations

import os

import numpy as np
import pandas as pd

from ..sql import types as T
from .artifacts import resolve
from .models import Model as MLModel


class PyFuncModel:
    def __init__(self, impl, meta: MLModel, flavor: str):
        self._impl = impl
        self.metadata = meta
        self.flavor = flavor

    def predict(self, data):
        if hasattr(data, "toPandas"):
            data = data.toPandas()
        out = self._impl.predict(data)
        return out

    def unwrap_python_model(self):
        return self._impl

    def __repr__(self):
        return f"mlflow.pyfunc.loaded_model:\n  flavor: {self.flavor}"


def load_model(model_uri: str, suppress_warnings: bool = False, dst_path=None) -> PyFuncModel:
    p = resolve(model_uri)
    meta = MLModel.load(p)
    pf = meta.flavors.get("python_function", {})
    mod = pf.get("loader_module", "")
    if mod.endswith("sklearn"):
        from . import sklearn as sk
        return PyFuncModel(sk._load_pyfunc(os.path.join(p, pf.get("model_path", "model.pkl"))), meta, "sklearn")
    if mod.endswith("spark"):
        from . import spark as sp
        return PyFuncModel(sp._load_pyfunc(os.path.join(p, pf.get("data", "sparkml"))), meta, "spark")
    raise ValueError(f"unsupported pyfunc loader {mod!r}")


def spark_udf(spark, model_uri: str, result_type="double", env_manager=None):
    p = resolve(model_uri)
    meta = MLModel.load(p)
    names = meta.signature.inputs.input_names() if meta.signature is not None else None
    rt = T.to_type(result_type) if isinstance(result_type, str) else result_type
    pf = meta.flavors.get("python_function", {})
    if pf.get("loader_module", "").endswith("spark"):
        return _NativeUDF(os.path.join(p, pf.get("data", "sparkml")), names, rt)
    model = load_model(model_uri)

    from ..sql.udf import UserDefinedFunction

    def predict_batch(*cols):
        pdf = pd.concat(cols, axis=1)
        if names and len(names) == pdf.shape[1]:
            pdf.columns = names
        return pd.Series(np.asarray(model.predict(pdf)).reshape(-1))
    u = UserDefinedFunction(predict_batch, rt, "scalar")
    u.__name__ = "predict"
    return u


class _NativeUDF:
    """Callable producing a Column that runs a PipelineModel on each device partition.

    The pipeline's plan is built ONCE per (session, input names, schema) over a one-batch source whose batch is
    swapped per call, so every partition re-runs the same plan: the same stage objects, the same cached forest
    predictor (``models/inference.py``: uploaded once, its predict graph-captured per recurring staging buffer and
    replayed) -- no DataFrame plan, model upload or pandas conversion per batch (ML 12 - Inference with Pandas
    UDFs.py:73-143 loads the model once per executor for the same reason)."""

    def __init__(self, path, names, rt):
        import threading
        import weakref

        from ..models.pipeline import PipelineModel
        self.pm = PipelineModel.load(path)
        self.names = names
        self.rt = rt
        # the batch being evaluated is per THREAD: CrossValidator(parallelism=4) threads, threaded streaming sinks
        # and applyInPandas pools may evaluate the same UDF concurrently through the one cached plan
        self._tls = threading.local()
        self._lock = threading.Lock()
        # plans per session (weak: a new session can reuse a dead one's id()) and input schema
        self._plans: "weakref.WeakKeyDictionary" = weakref.WeakKeyDictionary()
        self.batches = 0
        self.plans_built = 0

    def _current(self):
        return [self._tls.cur]

    def _plan_for(self, sess, part):
        from ..sql.dataframe import DataFrame, SourcePlan
        schema = part.schema()
        key = tuple((f.name, f.dataType.simpleString()) for f in schema.fields)
        with self._lock:
            per = self._plans.setdefault(sess, {})
            plan = per.get(key)
            if plan is None:
                src = DataFrame(SourcePlan(sess, "udf-batch", self._current, schema), sess)
                plan = per[key] = self.pm.transform(src)._plan
                self.plans_built += 1
        return plan

    def __call__(self, *cols):
        from ..sql.column import Column, Func, _cast
        from ..sql.batch import Batch
        from ..sql.functions import col as _col
        exprs = [_col(c)._expr if isinstance(c, str) else c._expr for c in cols]
        names = self.names

        def ev(b, ctx, args):
            ns = names if names and len(names) == len(args) else [e.name() for e in exprs]
            cur = Batch({n: a for n, a in zip(ns, args)}, b.n, b.device)
            prev = getattr(self._tls, "cur", None)
            self._tls.cur = cur
            try:
                out = self._plan_for(ctx.session, cur).execute()
            finally:
                self._tls.cur = prev
            with self._lock:
                self.batches += 1
            c = out[0].columns["prediction"] if out else None
            if c is None or len(c) != b.n:
                raise RuntimeError("model dropped rows inside spark_udf (use handleInvalid='keep')")
            return _cast(c, self.rt) if not isinstance(self.rt, T.DoubleType) else c
        return Column(Func("predict", ev, exprs))
