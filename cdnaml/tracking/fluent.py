"""Module-level tracking API with MLflow's names (SURVEY §2.7 O1–O5).

``with tracking.start_run(run_name=…) as run: tracking.log_param(…)`` etc.
(ML 04 - MLflow Tracking.py:77-228).  In SPMD jobs only rank 0 writes; the
run id is broadcast so every rank sees the same active run.
"""
from __future__ import annotations

import getpass
import json
import os
import re
import shutil
import tempfile
import threading
import time
from typing import Any, Dict, List, Optional

import numpy as np
import pandas as pd

from .entities import ActiveRun, Run, TrackingException
from .store import FileStore

_state = threading.local()
_global = {"uri": None, "experiment_id": None, "store": None, "store_uri": None, "stack": []}


def _rank() -> int:
    try:
        from ..session import SparkSession
        s = SparkSession.getActiveSession()
        return s.comm.rank if s is not None else 0
    except Exception:
        return 0


def _comm():
    try:
        from ..session import SparkSession
        s = SparkSession.getActiveSession()
        return s.comm if s is not None else None
    except Exception:
        return None


# ---------------------------------------------------------------- tracking uri
def set_tracking_uri(uri: str):
    if uri != _global["uri"]:
        _global["experiment_id"] = None  # experiment ids are per store
    _global["uri"] = uri


def get_tracking_uri() -> str:
    uri = _global["uri"] or os.environ.get("CDNAML_TRACKING_URI") or os.environ.get("MLFLOW_TRACKING_URI") or \
        "mlruns"
    if uri in ("databricks",) or uri.startswith("databricks"):
        uri = "mlruns"
    return uri


def set_registry_uri(uri: str):
    pass


def get_registry_uri() -> str:
    return get_tracking_uri()


def _store() -> FileStore:
    uri = get_tracking_uri()
    if _global["store"] is None or _global["store_uri"] != uri:
        _global["store"] = FileStore(uri)
        _global["store_uri"] = uri
    return _global["store"]


def is_tracking_uri_set() -> bool:
    return _global["uri"] is not None


# ---------------------------------------------------------------- experiments
def set_experiment(experiment_name: Optional[str] = None, experiment_id: Optional[str] = None):
    st = _store()
    if experiment_id is not None:
        exp = st.get_experiment(experiment_id)
    else:
        exp = st.get_experiment_by_name(experiment_name)
        if exp is None:
            eid = st.create_experiment(experiment_name) if _rank() == 0 else None
            c = _comm()
            if c is not None and c.distributed:
                eid = c.broadcast_object(eid)
            exp = st.get_experiment(eid)
    _global["experiment_id"] = exp.experiment_id
    return exp


def create_experiment(name, artifact_location=None, tags=None) -> str:
    return _store().create_experiment(name, artifact_location, tags)


def get_experiment(experiment_id):
    return _store().get_experiment(experiment_id)


def get_experiment_by_name(name):
    return _store().get_experiment_by_name(name)


def delete_experiment(experiment_id):
    _store().delete_experiment(experiment_id)


def search_experiments(view_type="ACTIVE_ONLY", max_results=None, filter_string=None, order_by=None):
    exps = _store().list_experiments(view_type if isinstance(view_type, str) else "ACTIVE_ONLY")
    if filter_string:
        m = re.match(r"\s*name\s*(=|LIKE)\s*'([^']*)'", filter_string, re.I)
        if m:
            pat = m.group(2)
            if m.group(1).upper() == "LIKE":
                rx = re.compile("^" + re.escape(pat).replace("%", ".*") + "$")
                exps = [e for e in exps if rx.match(e.name)]
            else:
                exps = [e for e in exps if e.name == pat]
    return exps[:max_results] if max_results else exps


list_experiments = search_experiments


def _default_experiment_id() -> str:
    if _global["experiment_id"] is not None:
        return _global["experiment_id"]
    env = os.environ.get("MLFLOW_EXPERIMENT_NAME")
    if env:
        return set_experiment(env).experiment_id
    return "0"


# ---------------------------------------------------------------- runs
def _stack() -> List[ActiveRun]:
    return _global["stack"]


def active_run() -> Optional[ActiveRun]:
    s = _stack()
    return s[-1] if s else None


def start_run(run_id: Optional[str] = None, experiment_id: Optional[str] = None, run_name: Optional[str] = None,
              nested: bool = False, tags: Optional[dict] = None, description: Optional[str] = None) -> ActiveRun:
    st = _store()
    if _stack() and not nested and run_id is None:
        raise TrackingException(f"Run with UUID {_stack()[-1].info.run_id} is already active. To start a nested "
                                f"run, call start_run with nested=True")
    if run_id is not None:
        run = st.get_run(run_id)
        if run.info.status != "RUNNING" and _rank() == 0:
            st.update_run(run_id, status="RUNNING", end_time=None)
        run = st.get_run(run_id)
    else:
        exp = experiment_id or _default_experiment_id()
        t = dict(tags or {})
        if nested and _stack():
            t["mlflow.parentRunId"] = _stack()[-1].info.run_id
        if description:
            t["mlflow.note.content"] = description
        t.setdefault("mlflow.source.type", "LOCAL")
        rid = None
        if _rank() == 0:
            rid = st.create_run(exp, _user(), None, t, run_name).info.run_id
        c = _comm()
        if c is not None and c.distributed:
            rid = c.broadcast_object(rid)
        run = st.get_run(rid)
    ar = ActiveRun(run)
    _stack().append(ar)
    return ar


def end_run(status: str = "FINISHED"):
    if not _stack():
        return
    ar = _stack().pop()
    if _rank() == 0:
        _store().update_run(ar.info.run_id, status=status, end_time=int(time.time() * 1000))


def _user():
    try:
        return getpass.getuser()
    except Exception:
        return "user"


def _rid(run_id=None) -> str:
    if run_id:
        return run_id
    ar = active_run()
    if ar is None:
        ar = start_run()
    return ar.info.run_id


def get_run(run_id) -> Run:
    return _store().get_run(run_id)


def last_active_run():
    return None


def delete_run(run_id):
    _store().delete_run(run_id)


# ---------------------------------------------------------------- logging
def log_param(key, value):
    if _rank() == 0:
        _store().log_param(_rid(), key, value)
    return value


def log_params(params: Dict[str, Any]):
    for k, v in params.items():
        log_param(k, v)


def log_metric(key, value, step=None, timestamp=None):
    if _rank() == 0:
        _store().log_metric(_rid(), key, value, timestamp, step or 0)


def log_metrics(metrics: Dict[str, float], step=None):
    for k, v in metrics.items():
        log_metric(k, v, step)


def set_tag(key, value):
    if _rank() == 0:
        _store().set_tag(_rid(), key, value)


def set_tags(tags: Dict[str, Any]):
    for k, v in tags.items():
        set_tag(k, v)


def delete_tag(key):
    _store().delete_tag(_rid(), key)


def get_artifact_uri(artifact_path: Optional[str] = None) -> str:
    base = _store().artifact_dir(_rid())
    return base if artifact_path is None else os.path.join(base, artifact_path)


def log_artifact(local_path: str, artifact_path: Optional[str] = None):
    if _rank() != 0:
        return
    dst = os.path.join(_store().artifact_dir(_rid()), artifact_path or "")
    os.makedirs(dst, exist_ok=True)
    shutil.copy2(local_path, os.path.join(dst, os.path.basename(local_path)))


def log_artifacts(local_dir: str, artifact_path: Optional[str] = None):
    if _rank() != 0:
        return
    dst = os.path.join(_store().artifact_dir(_rid()), artifact_path or "")
    shutil.copytree(local_dir, dst, dirs_exist_ok=True)


def log_text(text: str, artifact_file: str):
    if _rank() != 0:
        return
    p = os.path.join(_store().artifact_dir(_rid()), artifact_file)
    os.makedirs(os.path.dirname(p), exist_ok=True)
    with open(p, "w") as f:
        f.write(text)


def log_dict(d: dict, artifact_file: str):
    if artifact_file.endswith((".yaml", ".yml")):
        import yaml
        log_text(yaml.safe_dump(d), artifact_file)
    else:
        log_text(json.dumps(d, indent=2, default=str), artifact_file)


def log_figure(figure, artifact_file: str):
    if _rank() != 0:
        return
    p = os.path.join(_store().artifact_dir(_rid()), artifact_file)
    os.makedirs(os.path.dirname(p), exist_ok=True)
    figure.savefig(p)


def log_image(image, artifact_file: str):
    if _rank() != 0:
        return
    p = os.path.join(_store().artifact_dir(_rid()), artifact_file)
    os.makedirs(os.path.dirname(p), exist_ok=True)
    arr = np.asarray(image)
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    plt.imsave(p, arr)


# ---------------------------------------------------------------- search
_FILTER_CLAUSE = re.compile(
    r"\s*(?P<kind>params|metrics|metric|param|tags|tag|attributes|attribute|attr)\.(?P<key>`[^`]+`|\"[^\"]+\"|[\w.\-]+)"
    r"\s*(?P<op>=|!=|<=|>=|<|>|LIKE|ILIKE)\s*(?P<val>'[^']*'|\"[^\"]*\"|[-+\d.eE]+)\s*", re.I)


def _parse_filter(s: str):
    s = (s or "").strip()
    if not s:
        return []
    parts = re.split(r"\s+and\s+", s, flags=re.I)
    out = []
    for p in parts:
        m = _FILTER_CLAUSE.fullmatch(p)
        if not m:
            raise TrackingException(f"Invalid filter clause: {p!r}")
        kind = m.group("kind").lower()
        kind = {"param": "params", "metric": "metrics", "tag": "tags", "attribute": "attributes",
                "attr": "attributes"}.get(kind, kind)
        key = m.group("key").strip("`\"")
        val = m.group("val")
        if val[0] in "'\"":
            val = val[1:-1]
        else:
            val = float(val)
        out.append((kind, key, m.group("op").upper(), val))
    return out


def _match(run: Run, clauses) -> bool:
    for kind, key, op, val in clauses:
        if kind == "params":
            v = run.data.params.get(key)
        elif kind == "metrics":
            v = run.data.metrics.get(key)
        elif kind == "tags":
            v = run.data.tags.get(key)
        else:
            v = {"status": run.info.status, "run_id": run.info.run_id, "run_name": run.info.run_name,
                 "start_time": run.info.start_time, "end_time": run.info.end_time,
                 "artifact_uri": run.info.artifact_uri}.get(key)
        if v is None:
            return False
        if isinstance(val, float):
            try:
                v = float(v)
            except (TypeError, ValueError):
                return False
        if op == "=" and not v == val:
            return False
        if op == "!=" and not v != val:
            return False
        if op in ("<", ">", "<=", ">="):
            if not {"<": v < val, ">": v > val, "<=": v <= val, ">=": v >= val}[op]:
                return False
        if op in ("LIKE", "ILIKE"):
            rx = re.compile("^" + re.escape(str(val)).replace("%", ".*").replace("_", ".") + "$",
                            re.I if op == "ILIKE" else 0)
            if not rx.match(str(v)):
                return False
    return True


def _sort_runs(runs: List[Run], order_by):
    if not order_by:
        return sorted(runs, key=lambda r: -r.info.start_time)
    for ob in reversed(order_by):
        toks = ob.split()
        field = toks[0]
        desc = len(toks) > 1 and toks[1].lower() == "desc"
        kind, _, key = field.partition(".")
        kind = kind.lower()

        def keyf(r, kind=kind, key=key):
            if kind in ("metrics", "metric"):
                v = r.data.metrics.get(key)
            elif kind in ("params", "param"):
                v = r.data.params.get(key)
            elif kind in ("tags", "tag"):
                v = r.data.tags.get(key)
            else:
                v = getattr(r.info, key, None)
            return (v is None, v if v is not None else 0)
        runs = sorted(runs, key=keyf, reverse=desc)
        if desc:  # keep None last
            runs = [r for r in runs if keyf(r)[0] is False] + [r for r in runs if keyf(r)[0]]
    return runs


def _search(experiment_ids=None, filter_string="", order_by=None, max_results=None, run_view_type=None):
    st = _store()
    if experiment_ids is None:
        experiment_ids = [_default_experiment_id()]
    if isinstance(experiment_ids, (str, int)):
        experiment_ids = [experiment_ids]
    runs = st.search_runs([str(e) for e in experiment_ids])
    clauses = _parse_filter(filter_string)
    runs = [r for r in runs if _match(r, clauses)]
    runs = _sort_runs(runs, order_by)
    return runs[:max_results] if max_results else runs


def search_runs(experiment_ids=None, filter_string="", run_view_type=None, max_results=100000, order_by=None,
                output_format="pandas", experiment_names=None):
    if experiment_names:
        experiment_ids = [get_experiment_by_name(n).experiment_id for n in experiment_names]
    runs = _search(experiment_ids, filter_string, order_by, max_results)
    if output_format == "list":
        return runs
    rows = []
    for r in runs:
        d = {"run_id": r.info.run_id, "experiment_id": r.info.experiment_id, "status": r.info.status,
             "artifact_uri": r.info.artifact_uri,
             "start_time": pd.to_datetime(r.info.start_time, unit="ms", utc=True),
             "end_time": pd.to_datetime(r.info.end_time, unit="ms", utc=True) if r.info.end_time else pd.NaT}
        d.update({f"metrics.{k}": v for k, v in r.data.metrics.items()})
        d.update({f"params.{k}": v for k, v in r.data.params.items()})
        d.update({f"tags.{k}": v for k, v in r.data.tags.items()})
        rows.append(d)
    return pd.DataFrame(rows)


# ---------------------------------------------------------------- registry
def register_model(model_uri: str, name: str, await_registration_for: int = 300, tags=None):
    from .artifacts import parse_runs_uri
    st = _store()
    run_id, _ = parse_runs_uri(model_uri)
    source = model_uri
    try:
        st.get_registered_model(name)
    except TrackingException:
        st.create_registered_model(name)
    return st.create_model_version(name, source, run_id, tags)


# ---------------------------------------------------------------- autolog
def _autolog_fit(est, model, log_models: bool, metrics=None):
    created = False
    if active_run() is None:
        start_run()
        created = True
    try:
        params = {}
        from ..models.pipeline import Pipeline
        stages = est.getStages() if isinstance(est, Pipeline) else [est]
        for s in stages:
            for p, v in s.extractParamMap().items():
                if isinstance(v, (int, float, str, bool)) and v is not None:
                    key = p.name if len(stages) == 1 else f"{type(s).__name__}.{p.name}"
                    params[key] = v
        ar = active_run()
        existing = _store().get_run(ar.info.run_id).data.params
        for k, v in params.items():
            if k not in existing:
                log_param(k, v)
        set_tag("estimator_name", type(est).__name__)
        set_tag("estimator_class", f"{type(est).__module__}.{type(est).__name__}")
        for k, v in (metrics or {}).items():
            log_metric(k.replace("/", "_"), float(v))
        if log_models:
            from . import spark as _spark
            from ..models.pipeline import PipelineModel
            if isinstance(model, PipelineModel):
                _spark.log_model(model, "model")
    finally:
        if created:
            end_run()
