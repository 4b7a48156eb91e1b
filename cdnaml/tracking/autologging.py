"""Autologging hook around every ``Estimator.fit``.

``tracking.pyspark.ml.autolog()`` / ``mlflow.pyspark.ml.autolog(log_models=False)``
(ML 08 - Hyperopt.py:144) makes each fit log its params (and optionally the
model) to the active run, creating a run if none is active.
"""
from __future__ import annotations

_state = {"enabled": False, "log_models": False, "disable": False, "depth": 0}


def enable(log_models: bool = False, disable: bool = False, **kw):
    _state["enabled"] = not disable
    _state["log_models"] = log_models


def wrap_fit(est, dataset):
    from ..models.base import Model
    _state["depth"] += 1
    try:
        model = est._fit(dataset)
    finally:
        _state["depth"] -= 1
    if isinstance(model, Model) and model.parent is None:
        model._post_fit(est)
    if _state["enabled"] and _state["depth"] == 0:
        try:
            from . import fluent
            fluent._autolog_fit(est, model, _state["log_models"])
        except Exception:  # autolog must never break a fit
            pass
    return model


def is_enabled() -> bool:
    return bool(_state["enabled"])
