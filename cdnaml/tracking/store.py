"""MLflow-FileStore-compatible tracking + model-registry store (SURVEY §2.7 O1–O3, O6).

Layout (same as MLflow's file store, so existing tooling can read it)::

    <root>/<exp_id>/meta.yaml
    <root>/<exp_id>/<run_id>/{meta.yaml, params/<k>, metrics/<k>, tags/<k>, artifacts/}
    <root>/models/<name>/meta.yaml, <root>/models/<name>/version-<n>/meta.yaml

Process-safe: every metadata write is write-temp + atomic rename, metric
points are single O_APPEND writes — grouped ``applyInPandas`` workers log to
the same run concurrently (ML 13 - Training with Pandas Function API.py:93-101).
"""
from __future__ import annotations

import os
import re
import shutil
import time
import uuid
from typing import Dict, List, Optional

import yaml

from .entities import (Experiment, Metric, ModelVersion, RegisteredModel, Run, RunData, RunInfo,
                       TrackingException)

_NAME_BAD = re.compile(r"[/.:%\"']")


def _now():
    return int(time.time() * 1000)


def _atomic_write(path: str, text: str):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    tmp = f"{path}.tmp{uuid.uuid4().hex[:8]}"
    with open(tmp, "w") as f:
        f.write(text)
    os.replace(tmp, path)


def _read_yaml(path: str) -> dict:
    with open(path) as f:
        return yaml.safe_load(f) or {}


def _write_yaml(path: str, d: dict):
    _atomic_write(path, yaml.safe_dump(d, default_flow_style=False, sort_keys=True))


def _check_key(k: str):
    if not k or ".." in k or k.startswith("/") or "\\" in k:
        raise TrackingException(f"Invalid key '{k}'")


class FileStore:
    def __init__(self, root: str):
        if root.startswith("file:"):
            root = root[5:]
            while root.startswith("//"):
                root = root[1:]
        self.root = os.path.abspath(root)
        os.makedirs(self.root, exist_ok=True)
        if not os.path.exists(os.path.join(self.root, "0", "meta.yaml")):
            try:
                self._create_experiment_with_id("Default", "0")
            except FileExistsError:
                pass

    # ------------------------------------------------------------ experiments
    def _exp_dir(self, exp_id):
        return os.path.join(self.root, str(exp_id))

    def _create_experiment_with_id(self, name, exp_id, artifact_location=None, tags=None):
        d = self._exp_dir(exp_id)
        os.makedirs(d, exist_ok=True)
        now = _now()
        meta = {"artifact_location": artifact_location or f"file://{d}", "experiment_id": str(exp_id),
                "lifecycle_stage": "active", "name": name, "creation_time": now, "last_update_time": now}
        _write_yaml(os.path.join(d, "meta.yaml"), meta)
        for k, v in (tags or {}).items():
            _atomic_write(os.path.join(d, "tags", k), str(v))
        return str(exp_id)

    def list_experiments(self, view_type="ACTIVE_ONLY") -> List[Experiment]:
        out = []
        for e in sorted(os.listdir(self.root)):
            p = os.path.join(self.root, e, "meta.yaml")
            if e == "models" or not os.path.exists(p):
                continue
            m = _read_yaml(p)
            if view_type == "ACTIVE_ONLY" and m.get("lifecycle_stage") != "active":
                continue
            if view_type == "DELETED_ONLY" and m.get("lifecycle_stage") != "deleted":
                continue
            out.append(self._exp_from_meta(m))
        return out

    def _exp_from_meta(self, m) -> Experiment:
        tags = {}
        td = os.path.join(self._exp_dir(m["experiment_id"]), "tags")
        if os.path.isdir(td):
            for k in os.listdir(td):
                with open(os.path.join(td, k)) as f:
                    tags[k] = f.read()
        return Experiment(m["experiment_id"], m["name"], m["artifact_location"], m.get("lifecycle_stage", "active"),
                          tags, m.get("creation_time"), m.get("last_update_time"))

    def create_experiment(self, name: str, artifact_location=None, tags=None) -> str:
        if not name:
            raise TrackingException("Invalid experiment name: ''")
        if self.get_experiment_by_name(name) is not None:
            raise TrackingException(f"Experiment '{name}' already exists.")
        ids = [int(e) for e in os.listdir(self.root) if e.isdigit()]
        while True:
            new = str(max(ids + [0]) + 1 + int(uuid.uuid4().int % 1000)) if ids else "1"
            try:
                os.makedirs(self._exp_dir(new))
                break
            except FileExistsError:
                ids.append(int(new))
        return self._create_experiment_with_id(name, new, artifact_location, tags)

    def get_experiment(self, exp_id) -> Experiment:
        p = os.path.join(self._exp_dir(exp_id), "meta.yaml")
        if not os.path.exists(p):
            raise TrackingException(f"Could not find experiment with ID {exp_id}")
        return self._exp_from_meta(_read_yaml(p))

    def get_experiment_by_name(self, name: str) -> Optional[Experiment]:
        for e in self.list_experiments("ALL"):
            if e.name == name:
                return e
        return None

    def delete_experiment(self, exp_id):
        p = os.path.join(self._exp_dir(exp_id), "meta.yaml")
        m = _read_yaml(p)
        m["lifecycle_stage"] = "deleted"
        _write_yaml(p, m)

    def set_experiment_tag(self, exp_id, key, value):
        _atomic_write(os.path.join(self._exp_dir(exp_id), "tags", key), str(value))

    # ------------------------------------------------------------ runs
    def _run_dir(self, run_id) -> str:
        for e in os.listdir(self.root):
            d = os.path.join(self.root, e, run_id)
            if os.path.isdir(d) and os.path.exists(os.path.join(d, "meta.yaml")):
                return d
        raise TrackingException(f"Run '{run_id}' not found")

    def create_run(self, exp_id, user_id="", start_time=None, tags=None, run_name=None) -> Run:
        exp = self.get_experiment(exp_id)
        rid = uuid.uuid4().hex
        d = os.path.join(self._exp_dir(exp_id), rid)
        os.makedirs(os.path.join(d, "artifacts"), exist_ok=True)
        for sub in ("params", "metrics", "tags"):
            os.makedirs(os.path.join(d, sub), exist_ok=True)
        art = exp.artifact_location.rstrip("/") + f"/{rid}/artifacts"
        run_name = run_name or f"run-{rid[:8]}"
        meta = {"artifact_uri": art, "end_time": None, "entry_point_name": "", "experiment_id": str(exp_id),
                "lifecycle_stage": "active", "run_id": rid, "run_name": run_name, "run_uuid": rid, "source_name": "",
                "source_type": 4, "source_version": "", "start_time": start_time or _now(), "status": 1,
                "tags": [], "user_id": user_id}
        _write_yaml(os.path.join(d, "meta.yaml"), meta)
        tags = dict(tags or {})
        tags.setdefault("mlflow.runName", run_name)
        tags.setdefault("mlflow.user", user_id)
        for k, v in tags.items():
            self.set_tag(rid, k, v)
        return self.get_run(rid)

    _STATUS = {1: "RUNNING", 2: "SCHEDULED", 3: "FINISHED", 4: "FAILED", 5: "KILLED"}
    _STATUS_R = {v: k for k, v in _STATUS.items()}

    def get_run(self, run_id) -> Run:
        d = self._run_dir(run_id)
        m = _read_yaml(os.path.join(d, "meta.yaml"))
        params, tags, metrics = {}, {}, {}
        for k, sub in (("params", params), ("tags", tags)):
            base = os.path.join(d, k)
            for root, _, files in os.walk(base):
                for fn in files:
                    if ".tmp" in fn:
                        continue
                    with open(os.path.join(root, fn)) as f:
                        sub[os.path.relpath(os.path.join(root, fn), base)] = f.read()
        mbase = os.path.join(d, "metrics")
        for root, _, files in os.walk(mbase):
            for fn in files:
                pts = self._metric_points(os.path.join(root, fn))
                if pts:
                    last = max(pts, key=lambda p: (p.step, p.timestamp))
                    metrics[os.path.relpath(os.path.join(root, fn), mbase)] = last.value
        info = RunInfo(m["run_id"], m["experiment_id"], m.get("user_id", ""), self._STATUS.get(m["status"], "RUNNING"),
                       m["start_time"], m.get("end_time"), m["artifact_uri"], m.get("lifecycle_stage", "active"),
                       m.get("run_name") or tags.get("mlflow.runName"))
        return Run(info, RunData(metrics, params, tags))

    @staticmethod
    def _metric_points(path) -> List[Metric]:
        out = []
        key = os.path.basename(path)
        with open(path) as f:
            for line in f:
                parts = line.split()
                if len(parts) >= 2:
                    out.append(Metric(key, float(parts[1]), int(parts[0]), int(parts[2]) if len(parts) > 2 else 0))
        return out

    def get_metric_history(self, run_id, key) -> List[Metric]:
        return self._metric_points(os.path.join(self._run_dir(run_id), "metrics", key))

    def update_run(self, run_id, status=None, end_time=None, run_name=None):
        d = self._run_dir(run_id)
        p = os.path.join(d, "meta.yaml")
        m = _read_yaml(p)
        if status is not None:
            m["status"] = self._STATUS_R[status]
        if end_time is not None:
            m["end_time"] = end_time
        if run_name is not None:
            m["run_name"] = run_name
            self.set_tag(run_id, "mlflow.runName", run_name)
        _write_yaml(p, m)

    def delete_run(self, run_id):
        p = os.path.join(self._run_dir(run_id), "meta.yaml")
        m = _read_yaml(p)
        m["lifecycle_stage"] = "deleted"
        _write_yaml(p, m)

    def log_param(self, run_id, key, value):
        _check_key(key)
        p = os.path.join(self._run_dir(run_id), "params", key)
        v = str(value)
        if os.path.exists(p):
            with open(p) as f:
                old = f.read()
            if old != v:
                raise TrackingException(f"Changing param values is not allowed. Param with key='{key}' was already "
                                        f"logged with value='{old}' for run ID='{run_id}'. Attempted logging new "
                                        f"value '{v}'.")
            return
        _atomic_write(p, v)

    def log_metric(self, run_id, key, value, timestamp=None, step=0):
        _check_key(key)
        p = os.path.join(self._run_dir(run_id), "metrics", key)
        os.makedirs(os.path.dirname(p), exist_ok=True)
        line = f"{timestamp or _now()} {float(value)} {int(step or 0)}\n"
        fd = os.open(p, os.O_WRONLY | os.O_APPEND | os.O_CREAT, 0o644)
        try:
            os.write(fd, line.encode())
        finally:
            os.close(fd)

    def set_tag(self, run_id, key, value):
        _check_key(key)
        _atomic_write(os.path.join(self._run_dir(run_id), "tags", key), str(value))

    def delete_tag(self, run_id, key):
        p = os.path.join(self._run_dir(run_id), "tags", key)
        if os.path.exists(p):
            os.remove(p)

    def artifact_dir(self, run_id) -> str:
        return os.path.join(self._run_dir(run_id), "artifacts")

    def search_runs(self, exp_ids: List[str], include_deleted=False) -> List[Run]:
        out = []
        for e in exp_ids:
            d = self._exp_dir(e)
            if not os.path.isdir(d):
                continue
            for rid in os.listdir(d):
                if os.path.exists(os.path.join(d, rid, "meta.yaml")):
                    r = self.get_run(rid)
                    if include_deleted or r.info.lifecycle_stage == "active":
                        out.append(r)
        return out

    # ------------------------------------------------------------ registry
    def _models_dir(self):
        return os.path.join(self.root, "models")

    @staticmethod
    def _validate_model_name(name):
        if not name or not isinstance(name, str):
            raise TrackingException("Registered model name cannot be empty.")
        if any(ch in name for ch in "/.:"):
            raise TrackingException(f"Invalid model name '{name}': a registered model name must be a non-empty "
                                    f"UTF-8 string and cannot contain forward slashes(/), periods(.), or colons(:).")

    def create_registered_model(self, name, tags=None, description=None) -> RegisteredModel:
        self._validate_model_name(name)
        d = os.path.join(self._models_dir(), name)
        if os.path.exists(os.path.join(d, "meta.yaml")):
            raise TrackingException(f"Registered Model (name={name}) already exists.")
        now = _now()
        _write_yaml(os.path.join(d, "meta.yaml"), {"name": name, "creation_timestamp": now,
                                                   "last_updated_timestamp": now, "description": description or ""})
        for k, v in (tags or {}).items():
            _atomic_write(os.path.join(d, "tags", k), str(v))
        return self.get_registered_model(name)

    def get_registered_model(self, name) -> RegisteredModel:
        d = os.path.join(self._models_dir(), name)
        p = os.path.join(d, "meta.yaml")
        if not os.path.exists(p):
            raise TrackingException(f"Registered Model with name={name} not found")
        m = _read_yaml(p)
        versions = self.search_model_versions_for(name)
        latest = {}
        for v in versions:
            if v.current_stage not in latest or int(v.version) > int(latest[v.current_stage].version):
                latest[v.current_stage] = v
        return RegisteredModel(name, m["creation_timestamp"], m["last_updated_timestamp"], m.get("description", ""),
                               list(latest.values()))

    def update_registered_model(self, name, description):
        p = os.path.join(self._models_dir(), name, "meta.yaml")
        m = _read_yaml(p)
        m["description"] = description
        m["last_updated_timestamp"] = _now()
        _write_yaml(p, m)
        return self.get_registered_model(name)

    def rename_registered_model(self, name, new_name):
        os.replace(os.path.join(self._models_dir(), name), os.path.join(self._models_dir(), new_name))
        p = os.path.join(self._models_dir(), new_name, "meta.yaml")
        m = _read_yaml(p)
        m["name"] = new_name
        _write_yaml(p, m)

    def delete_registered_model(self, name):
        d = os.path.join(self._models_dir(), name)
        if not os.path.isdir(d):
            raise TrackingException(f"Registered Model with name={name} not found")
        shutil.rmtree(d)

    def list_registered_models(self) -> List[RegisteredModel]:
        md = self._models_dir()
        if not os.path.isdir(md):
            return []
        return [self.get_registered_model(n) for n in sorted(os.listdir(md))
                if os.path.exists(os.path.join(md, n, "meta.yaml"))]

    def create_model_version(self, name, source, run_id=None, tags=None, description=None) -> ModelVersion:
        d = os.path.join(self._models_dir(), name)
        if not os.path.exists(os.path.join(d, "meta.yaml")):
            self.create_registered_model(name)
        for _ in range(100):
            vs = [int(x.split("-", 1)[1]) for x in os.listdir(d) if x.startswith("version-")]
            v = max(vs + [0]) + 1
            vd = os.path.join(d, f"version-{v}")
            try:
                os.makedirs(vd)
                break
            except FileExistsError:
                continue
        now = _now()
        _write_yaml(os.path.join(vd, "meta.yaml"), {
            "name": name, "version": str(v), "source": source, "run_id": run_id or "", "current_stage": "None",
            "status": "READY", "status_message": "", "description": description or "",
            "creation_timestamp": now, "last_updated_timestamp": now, "user_id": ""})
        for k, val in (tags or {}).items():
            _atomic_write(os.path.join(vd, "tags", k), str(val))
        p = os.path.join(d, "meta.yaml")
        m = _read_yaml(p)
        m["last_updated_timestamp"] = now
        _write_yaml(p, m)
        return self.get_model_version(name, v)

    def _mv_path(self, name, version):
        return os.path.join(self._models_dir(), name, f"version-{int(version)}", "meta.yaml")

    def get_model_version(self, name, version) -> ModelVersion:
        p = self._mv_path(name, version)
        if not os.path.exists(p):
            raise TrackingException(f"Model Version (name={name}, version={version}) not found")
        m = _read_yaml(p)
        return ModelVersion(m["name"], str(m["version"]), m["creation_timestamp"], m["last_updated_timestamp"],
                            m.get("description", ""), m.get("user_id", ""), m["current_stage"], m["source"],
                            m.get("run_id", ""), m.get("status", "READY"), m.get("status_message", ""))

    def update_model_version(self, name, version, description=None, stage=None):
        p = self._mv_path(name, version)
        m = _read_yaml(p)
        if description is not None:
            m["description"] = description
        if stage is not None:
            m["current_stage"] = stage
        m["last_updated_timestamp"] = _now()
        _write_yaml(p, m)
        return self.get_model_version(name, version)

    def delete_model_version(self, name, version):
        d = os.path.dirname(self._mv_path(name, version))
        if not os.path.isdir(d):
            raise TrackingException(f"Model Version (name={name}, version={version}) not found")
        shutil.rmtree(d)

    def search_model_versions_for(self, name) -> List[ModelVersion]:
        d = os.path.join(self._models_dir(), name)
        if not os.path.isdir(d):
            return []
        out = []
        for x in os.listdir(d):
            if x.startswith("version-") and os.path.exists(os.path.join(d, x, "meta.yaml")):
                out.append(self.get_model_version(name, int(x.split("-", 1)[1])))
        return sorted(out, key=lambda v: int(v.version))
