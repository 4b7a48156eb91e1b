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


def _engine_counters(dataset):
    try:
        comm = dataset._session.comm
        return {"calls": comm.calls, "bytes": comm.bytes_reduced}
    except Exception:  # noqa: BLE001
        return {"calls": 0, "bytes": 0}


def wrap_fit(est, dataset):
    import time

    from ..models.base import Model
    top = _state["depth"] == 0 and _state["enabled"]
    c0 = _engine_counters(dataset) if top else None
    t0 = time.perf_counter()
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
            c1 = _engine_counters(dataset)
            # engine metrics of the fit: wall time, collectives, and the traced phase totals
            metrics = {"engine.fit_ms": (time.perf_counter() - t0) * 1e3,
                       "engine.collective_calls": float(c1["calls"] - (c0 or c1)["calls"]),
                       "engine.collective_MB": (c1["bytes"] - (c0 or c1)["bytes"]) / 1e6}
            from ..utils import tracing
            if tracing.is_enabled():
                for name, st in tracing.stats().items():
                    metrics[f"engine.{name}_ms"] = st["total_ms"]
            fluent._autolog_fit(est, model, _state["log_models"], metrics)
        except Exception:  # autolog must never break a fit
            pass
    return model


def is_enabled() -> bool:
    return bool(_state["enabled"])
