"""Model persistence.

Spark-like, self-describing directory layout::

    path/metadata/part-00000   one JSON line: class, uid, paramMap, defaultParamMap, extra
    path/data/tensors.safetensors  device state (coefficients, tree arrays …), if any
    path/data/extra.json           small host state (labels, attributes …)
    path/stages/<i>_<uid>/         nested stages (Pipeline / PipelineModel / CrossValidatorModel)

``model.write().overwrite().save(path)`` / ``PipelineModel.load(path)`` and
the generic ``load`` (ML 03 - Linear Regression II.py:109-129;
Labs/ML 07L:209; MLE 00:36-39).  Loading never unpickles: tensors come from
safetensors, everything else from JSON.
"""
from __future__ import annotations

import importlib
import json
import os
import shutil
import time
from typing import Dict, Optional

import numpy as np
import torch


def _jsonable(v):
    if isinstance(v, (np.integer,)):
        return int(v)
    if isinstance(v, (np.floating,)):
        return float(v)
    if isinstance(v, np.ndarray):
        return v.tolist()
    if isinstance(v, (list, tuple)):
        return [_jsonable(x) for x in v]
    if isinstance(v, dict):
        return {str(k): _jsonable(x) for k, x in v.items()}
    if hasattr(v, "toArray"):
        return v.toArray().tolist()
    return v


class MLWriter:
    def __init__(self, instance):
        self.instance = instance
        self._overwrite = False

    def overwrite(self):
        self._overwrite = True
        return self

    def session(self, s):
        return self

    def option(self, k, v):
        return self

    def save(self, path: str):
        from ..sql.readwriter import _strip_dbfs
        path = _strip_dbfs(path)
        from ..session import SparkSession
        s = SparkSession.getActiveSession()
        rank = s.comm.rank if s is not None else 0
        if os.path.exists(path):
            if not self._overwrite:
                raise FileExistsError(f"Path {path} already exists. To overwrite it, please use "
                                      f"write.overwrite().save(path).")
            if rank == 0:
                shutil.rmtree(path)
        if s is not None:
            s.comm.barrier()
        if rank == 0:
            save_instance(self.instance, path)
        if s is not None:
            s.comm.barrier()


def save_instance(inst, path: str):
    os.makedirs(os.path.join(path, "metadata"), exist_ok=True)
    extra, tensors = inst._save_state() if hasattr(inst, "_save_state") else ({}, {})
    meta = {
        "class": f"{type(inst).__module__}.{type(inst).__name__}",
        "timestamp": int(time.time() * 1000),
        "sparkVersion": "3.3.0-cdnaml",
        "uid": inst.uid,
        "paramMap": _jsonable({k: v for k, v in inst._paramMap.items() if _is_simple(v)}),
        "defaultParamMap": _jsonable({k: v for k, v in inst._defaultParamMap.items() if _is_simple(v)}),
    }
    with open(os.path.join(path, "metadata", "part-00000"), "w") as f:
        f.write(json.dumps(meta) + "\n")
    os.makedirs(os.path.join(path, "data"), exist_ok=True)
    with open(os.path.join(path, "data", "extra.json"), "w") as f:
        json.dump(_jsonable(extra), f)
    if tensors:
        from safetensors.torch import save_file
        save_file({k: v.detach().cpu().contiguous() for k, v in tensors.items()},
                  os.path.join(path, "data", "tensors.safetensors"))
    for i, stage in enumerate(inst._sub_stages() if hasattr(inst, "_sub_stages") else []):
        save_instance(stage, os.path.join(path, "stages", f"{i}_{stage.uid}"))


def _is_simple(v):
    try:
        json.dumps(_jsonable(v))
        return True
    except (TypeError, ValueError):
        return False


def load_instance(path: str):
    from ..sql.readwriter import _strip_dbfs
    path = _strip_dbfs(path)
    with open(os.path.join(path, "metadata", "part-00000")) as f:
        meta = json.loads(f.readline())
    modname, clsname = meta["class"].rsplit(".", 1)
    cls = getattr(importlib.import_module(modname), clsname)
    inst = cls.__new__(cls)
    cls._init_for_load(inst)
    inst.uid = meta["uid"]
    # re-parent params
    from .param import Param
    for name, spec in cls._all_specs().items():
        object.__setattr__(inst, name, Param(inst, name, spec[0], spec[2]))
    inst._defaultParamMap.update(meta.get("defaultParamMap", {}))
    inst._paramMap.update(meta.get("paramMap", {}))
    extra = {}
    ep = os.path.join(path, "data", "extra.json")
    if os.path.exists(ep):
        with open(ep) as f:
            extra = json.load(f)
    tensors = {}
    tp = os.path.join(path, "data", "tensors.safetensors")
    if os.path.exists(tp):
        from safetensors.torch import load_file
        tensors = load_file(tp)
    stages = []
    sd = os.path.join(path, "stages")
    if os.path.isdir(sd):
        for name in sorted(os.listdir(sd), key=lambda x: int(x.split("_", 1)[0])):
            stages.append(load_instance(os.path.join(sd, name)))
    if hasattr(inst, "_load_state"):
        inst._load_state(extra, tensors, stages)
    return inst


class MLWritable:
    def write(self) -> MLWriter:
        return MLWriter(self)

    def save(self, path: str):
        self.write().save(path)


class MLReadable:
    @classmethod
    def _init_for_load(cls, inst):
        from .param import Params
        Params.__init__(inst)

    @classmethod
    def read(cls):
        class _R:
            def load(_, path):
                return cls.load(path)
        return _R()

    @classmethod
    def load(cls, path: str):
        inst = load_instance(path)
        return inst


class DefaultParamsReadable(MLReadable):
    pass


class DefaultParamsWritable(MLWritable):
    pass


def device():
    from ..session import SparkSession
    s = SparkSession.getActiveSession()
    return s.device if s is not None else torch.device("cpu")
