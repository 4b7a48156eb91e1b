"""Drop-in import names for code written against the reference stack (SURVEY §0:
Spark/MLlib, MLflow, Hyperopt, sparkdl.xgboost, Delta, Koalas, Databricks
Feature Store / AutoML).

    import cdnaml.compat; cdnaml.compat.install()
    from pyspark.ml.regression import RandomForestRegressor   # -> cdnaml
    import mlflow                                              # -> cdnaml.tracking

``install()`` only claims names that are NOT importable as real packages
(pass ``force=True`` to shadow them).  Nothing is patched inside any real
library; the aliases are plain ``sys.modules`` entries pointing at this
framework's modules.
"""
from __future__ import annotations

import importlib
import importlib.util
import sys
import types
from typing import Dict, List

# alias -> module path inside cdnaml
_MAP: Dict[str, str] = {
    "pyspark": "cdnaml",
    "pyspark.sql": "cdnaml.sql",
    "pyspark.sql.functions": "cdnaml.sql.functions",
    "pyspark.sql.types": "cdnaml.sql.types",
    "pyspark.sql.column": "cdnaml.sql.column",
    "pyspark.sql.dataframe": "cdnaml.sql.dataframe",
    "pyspark.sql.session": "cdnaml.session",
    "pyspark.sql.streaming": "cdnaml.streaming",
    "pyspark.ml": "cdnaml.ml",
    "pyspark.ml.feature": "cdnaml.ml.feature",
    "pyspark.ml.regression": "cdnaml.ml.regression",
    "pyspark.ml.classification": "cdnaml.ml.classification",
    "pyspark.ml.clustering": "cdnaml.ml.clustering",
    "pyspark.ml.recommendation": "cdnaml.ml.recommendation",
    "pyspark.ml.evaluation": "cdnaml.ml.evaluation",
    "pyspark.ml.tuning": "cdnaml.ml.tuning",
    "pyspark.ml.linalg": "cdnaml.ml.linalg",
    "pyspark.ml.param": "cdnaml.ml.param",
    "pyspark.ml.stat": "cdnaml.ml.stat",
    "pyspark.ml.functions": "cdnaml.ml.functions",
    "pyspark.ml.pipeline": "cdnaml.models.pipeline",
    "pyspark.pandas": "cdnaml.pandas_api",
    "mlflow": "cdnaml.tracking",
    "mlflow.tracking": "cdnaml.tracking._tracking_ns",
    "mlflow.tracking.client": "cdnaml.tracking.client",
    "mlflow.models": "cdnaml.tracking.models",
    "mlflow.models.signature": "cdnaml.tracking.models",
    "mlflow.sklearn": "cdnaml.tracking.sklearn",
    "mlflow.spark": "cdnaml.tracking.spark",
    "mlflow.pyfunc": "cdnaml.tracking.pyfunc",
    "mlflow.entities": "cdnaml.tracking.entities",
    "mlflow.exceptions": "cdnaml.tracking.entities",
    "hyperopt": "cdnaml.hyperopt",
    "hyperopt.hp": "cdnaml.hyperopt.hp",
    "hyperopt.tpe": "cdnaml.hyperopt.tpe",
    "hyperopt.rand": "cdnaml.hyperopt.rand",
    "hyperopt.anneal": "cdnaml.hyperopt.anneal",
    "hyperopt.early_stop": "cdnaml.hyperopt.early_stop",
    "sparkdl": "cdnaml.ml",
    "sparkdl.xgboost": "cdnaml.ml.xgboost",
    "delta": "cdnaml.storage",
    "delta.tables": "cdnaml.storage.delta",
    "databricks.koalas": "cdnaml.pandas_api",
    "databricks.feature_store": "cdnaml.feature_store",
    "databricks.automl": "cdnaml.automl",
}

_installed: List[str] = []


def _real_exists(name: str) -> bool:
    top = name.split(".")[0]
    if top in sys.modules and not getattr(sys.modules[top], "__cdnaml_alias__", False):
        return True
    try:
        return importlib.util.find_spec(top) is not None
    except (ImportError, ValueError):
        return False


def install(force: bool = False) -> List[str]:
    """Register the aliases; returns the alias names that were installed."""
    tops: Dict[str, bool] = {}
    for alias, target in _MAP.items():
        top = alias.split(".")[0]
        if top not in tops:
            tops[top] = force or not _real_exists(alias)
        if not tops[top]:
            continue
        mod = importlib.import_module(target)
        sys.modules[alias] = mod
        _installed.append(alias)
    # "databricks" is a namespace package holding koalas / feature_store / automl
    if "databricks.koalas" in sys.modules and (force or "databricks" not in sys.modules):
        ns = types.ModuleType("databricks")
        ns.__cdnaml_alias__ = True
        ns.koalas = sys.modules["databricks.koalas"]
        ns.feature_store = sys.modules["databricks.feature_store"]
        ns.automl = sys.modules["databricks.automl"]
        ns.__path__ = []
        sys.modules["databricks"] = ns
        _installed.append("databricks")
    # attribute access along dotted paths (import pyspark; pyspark.sql.functions ...)
    for alias in list(_installed):
        parts = alias.split(".")
        for i in range(1, len(parts)):
            parent = sys.modules.get(".".join(parts[:i]))
            child = sys.modules.get(".".join(parts[: i + 1]))
            if parent is not None and child is not None and not hasattr(parent, parts[i]):
                try:
                    setattr(parent, parts[i], child)
                except (AttributeError, TypeError):
                    pass
    return list(_installed)


def uninstall():
    for alias in _installed:
        sys.modules.pop(alias, None)
    _installed.clear()
