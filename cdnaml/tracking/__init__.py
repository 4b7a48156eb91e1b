"""MLflow-compatible tracking, model registry and model flavors (SURVEY §2.7 O1–O6).

Use as ``from cdnaml import tracking as mlflow`` (or ``cdnaml.compat.install()``
to make ``import mlflow`` resolve here).  Storage is MLflow's file-store
layout under the tracking URI (default ``./mlruns``).
"""
from . import models  # noqa: F401
from .client import MlflowClient  # noqa: F401
from .entities import MlflowException, TrackingException  # noqa: F401
from .fluent import (active_run, create_experiment, delete_experiment, delete_run, delete_tag,  # noqa: F401
                     end_run, get_artifact_uri, get_experiment, get_experiment_by_name, get_registry_uri, get_run,
                     get_tracking_uri, list_experiments, log_artifact, log_artifacts, log_dict, log_figure,
                     log_image, log_metric, log_metrics, log_param, log_params, log_text, register_model,
                     search_experiments, search_runs, set_experiment, set_registry_uri, set_tag, set_tags,
                     set_tracking_uri, start_run)
from .models import ModelSignature, infer_signature  # noqa: F401


class _PySparkML:
    @staticmethod
    def autolog(log_models: bool = False, disable: bool = False, **kw):
        from . import autologging as _a
        _a.enable(log_models=log_models, disable=disable)


class _PySpark:
    ml = _PySparkML()


pyspark = _PySpark()


def autolog(log_models: bool = False, disable: bool = False, **kw):
    from . import autologging as _a
    _a.enable(log_models=log_models, disable=disable)


def __getattr__(name):
    import importlib
    if name in ("spark", "sklearn", "pyfunc", "client", "store", "artifacts"):
        return importlib.import_module(f"{__name__}.{name}")
    if name == "tracking":
        import types
        m = types.SimpleNamespace(MlflowClient=MlflowClient)
        return m
    raise AttributeError(name)
