"""MLmodel format, signatures and the shared log/save helpers for flavors.

An artifact directory holds ``MLmodel`` (YAML: flavors, signature,
run_id, utc_time_created, saved_input_example_info), the flavor's payload,
``input_example.json``, ``conda.yaml`` and ``requirements.txt`` — the same
shape as MLflow (ML 04 - MLflow Tracking.py:243).
"""
from __future__ import annotations

import datetime as _dt
import json
import os
import shutil
import tempfile
from typing import Any, Dict, List, Optional

import numpy as np
import pandas as pd
import yaml


class ColSpec:
    def __init__(self, type, name=None):  # noqa: A002
        self.type = type
        self.name = name

    def to_dict(self):
        d = {"type": self.type}
        if self.name is not None:
            d["name"] = self.name
        return d

    def __repr__(self):
        return f"{self.name!r}: {self.type!r}" if self.name else repr(self.type)


class Schema:
    def __init__(self, inputs: List[ColSpec]):
        self.inputs = list(inputs)

    def input_names(self):
        return [c.name for c in self.inputs]

    def to_json(self):
        return json.dumps([c.to_dict() for c in self.inputs])

    @classmethod
    def from_json(cls, s):
        return cls([ColSpec(d["type"], d.get("name")) for d in json.loads(s)])

    def __repr__(self):
        return "[" + ", ".join(map(repr, self.inputs)) + "]"


class ModelSignature:
    def __init__(self, inputs: Schema, outputs: Optional[Schema] = None):
        self.inputs = inputs
        self.outputs = outputs

    def to_dict(self):
        return {"inputs": self.inputs.to_json(), "outputs": self.outputs.to_json() if self.outputs else None}

    @classmethod
    def from_dict(cls, d):
        return cls(Schema.from_json(d["inputs"]), Schema.from_json(d["outputs"]) if d.get("outputs") else None)

    def __repr__(self):
        return f"inputs:\n  {self.inputs!r}\noutputs:\n  {self.outputs!r}"


def _type_of(dtype) -> str:
    k = np.dtype(dtype).kind if not isinstance(dtype, str) else "O"
    return {"f": "double", "i": "long", "u": "long", "b": "boolean", "M": "datetime"}.get(k, "string")


def _schema_of(x) -> Schema:
    if hasattr(x, "toPandas"):
        x = x.limit(5).toPandas()
    if isinstance(x, pd.DataFrame):
        return Schema([ColSpec(_type_of(x[c].dtype), str(c)) for c in x.columns])
    if isinstance(x, pd.Series):
        return Schema([ColSpec(_type_of(x.dtype), x.name)])
    a = np.asarray(x)
    if a.ndim == 1:
        return Schema([ColSpec(_type_of(a.dtype))])
    return Schema([ColSpec(_type_of(a.dtype)) for _ in range(a.shape[1])])


def infer_signature(model_input, model_output=None) -> ModelSignature:
    return ModelSignature(_schema_of(model_input), _schema_of(model_output) if model_output is not None else None)


class Model:
    """In-memory MLmodel."""

    def __init__(self, artifact_path=None, run_id=None, flavors=None, signature=None, saved_input_example_info=None,
                 utc_time_created=None):
        self.artifact_path = artifact_path
        self.run_id = run_id
        self.flavors = flavors or {}
        self.signature = signature
        self.saved_input_example_info = saved_input_example_info
        self.utc_time_created = utc_time_created or _dt.datetime.utcnow().isoformat()

    def add_flavor(self, name, **params):
        self.flavors[name] = params
        return self

    def to_dict(self):
        d = {"artifact_path": self.artifact_path, "flavors": self.flavors, "utc_time_created": self.utc_time_created}
        if self.run_id:
            d["run_id"] = self.run_id
        if self.signature is not None:
            d["signature"] = self.signature.to_dict()
        if self.saved_input_example_info:
            d["saved_input_example_info"] = self.saved_input_example_info
        return d

    def save(self, path):
        with open(os.path.join(path, "MLmodel"), "w") as f:
            yaml.safe_dump(self.to_dict(), f, default_flow_style=False)

    @classmethod
    def load(cls, path):
        p = path if path.endswith("MLmodel") else os.path.join(path, "MLmodel")
        with open(p) as f:
            d = yaml.safe_load(f)
        m = cls(d.get("artifact_path"), d.get("run_id"), d.get("flavors"),
                ModelSignature.from_dict(d["signature"]) if d.get("signature") else None,
                d.get("saved_input_example_info"), d.get("utc_time_created"))
        return m


def write_common(path: str, mlmodel: Model, input_example=None, pip_requirements=None):
    if input_example is not None:
        ex = input_example
        if hasattr(ex, "toPandas"):
            ex = ex.limit(5).toPandas()
        if isinstance(ex, pd.DataFrame):
            ex = ex.head(5)
            with open(os.path.join(path, "input_example.json"), "w") as f:
                f.write(ex.to_json(orient="split", default_handler=str))
            mlmodel.saved_input_example_info = {"artifact_path": "input_example.json", "type": "dataframe",
                                                "pandas_orient": "split"}
            if mlmodel.signature is None:
                mlmodel.signature = ModelSignature(_schema_of(ex))
        else:
            with open(os.path.join(path, "input_example.json"), "w") as f:
                json.dump(np.asarray(ex).tolist(), f)
            mlmodel.saved_input_example_info = {"artifact_path": "input_example.json", "type": "ndarray"}
    reqs = pip_requirements or ["cdnaml", "torch", "numpy", "pandas"]
    with open(os.path.join(path, "requirements.txt"), "w") as f:
        f.write("\n".join(reqs) + "\n")
    with open(os.path.join(path, "conda.yaml"), "w") as f:
        yaml.safe_dump({"name": "cdnaml_env", "channels": ["conda-forge"],
                        "dependencies": ["python=3.10", "pip", {"pip": reqs}]}, f)
    with open(os.path.join(path, "python_env.yaml"), "w") as f:
        yaml.safe_dump({"python": "3.10", "dependencies": reqs}, f)
    mlmodel.save(path)


def log_to_run(save_fn, artifact_path: str, registered_model_name: Optional[str] = None, **kw):
    """Save via ``save_fn(local_dir)`` into the active run's artifacts (rank 0), optionally register."""
    from . import fluent
    rid = fluent._rid()
    info = None
    if fluent._rank() == 0:
        dst = os.path.join(fluent._store().artifact_dir(rid), artifact_path)
        if os.path.exists(dst):
            shutil.rmtree(dst)
        os.makedirs(dst, exist_ok=True)
        save_fn(dst, rid)
    c = fluent._comm()
    if c is not None and c.distributed:
        c.barrier()
    uri = f"runs:/{rid}/{artifact_path}"
    info = ModelInfo(uri, rid, artifact_path)
    if registered_model_name:
        mv = fluent.register_model(uri, registered_model_name)
        info.registered_model_version = mv.version
    return info


class ModelInfo:
    def __init__(self, model_uri, run_id, artifact_path):
        self.model_uri = model_uri
        self.run_id = run_id
        self.artifact_path = artifact_path
        self.registered_model_version = None
