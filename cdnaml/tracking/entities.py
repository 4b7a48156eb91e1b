"""Tracking entities with MLflow's attribute names (run.info.run_id, run.data.metrics …)."""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional


class TrackingException(Exception):
    """Equivalent of ``mlflow.exceptions.MlflowException``."""


MlflowException = TrackingException


@dataclass
class Metric:
    key: str
    value: float
    timestamp: int
    step: int = 0


@dataclass
class Param:
    key: str
    value: str


@dataclass
class RunInfo:
    run_id: str
    experiment_id: str
    user_id: str
    status: str
    start_time: int
    end_time: Optional[int]
    artifact_uri: str
    lifecycle_stage: str = "active"
    run_name: Optional[str] = None

    @property
    def run_uuid(self):
        return self.run_id


@dataclass
class RunData:
    metrics: Dict[str, float] = field(default_factory=dict)
    params: Dict[str, str] = field(default_factory=dict)
    tags: Dict[str, str] = field(default_factory=dict)


@dataclass
class Run:
    info: RunInfo
    data: RunData


@dataclass
class Experiment:
    experiment_id: str
    name: str
    artifact_location: str
    lifecycle_stage: str = "active"
    tags: Dict[str, str] = field(default_factory=dict)
    creation_time: Optional[int] = None
    last_update_time: Optional[int] = None


@dataclass
class ModelVersion:
    name: str
    version: str
    creation_timestamp: int
    last_updated_timestamp: int
    description: str
    user_id: str
    current_stage: str
    source: str
    run_id: str
    status: str = "READY"
    status_message: str = ""


@dataclass
class RegisteredModel:
    name: str
    creation_timestamp: int
    last_updated_timestamp: int
    description: str
    latest_versions: List[ModelVersion] = field(default_factory=list)


class ActiveRun:
    """Context manager returned by start_run (``with start_run() as run``)."""

    def __init__(self, run: Run):
        self._run = run

    @property
    def info(self):
        return self._run.info

    @property
    def data(self):
        from . import fluent
        return fluent._store().get_run(self._run.info.run_id).data

    def __enter__(self):
        return self

    def __exit__(self, exc_type, exc, tb):
        from . import fluent
        fluent.end_run("FINISHED" if exc_type is None else "FAILED")
        return False
