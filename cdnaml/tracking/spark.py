"""Flavor for this framework's Pipeline models (``mlflow.spark`` equivalent).

``log_model(pipeline_model, "model", input_example=…)`` — only PipelineModels
can be logged (ML 04 - MLflow Tracking.py:66).  The payload is the standard
model directory (metadata JSON + safetensors), so loading executes nothing
from the artifact; the pyfunc wrapper predicts on device.
"""
from __future__ import annotations

import os

from ..models.pipeline import PipelineModel
from .artifacts import resolve
from .entities import TrackingException
from .models import Model, log_to_run, write_common

FLAVOR_NAME = "spark"


def save_model(spark_model, path, input_example=None, signature=None, run_id=None, artifact_path=None, **kw):
    if not isinstance(spark_model, PipelineModel):
        raise TrackingException(f"Argument 'spark_model' should be a PipelineModel, got '{type(spark_model)}'")
    os.makedirs(path, exist_ok=True)
    spark_model.write().overwrite().save(os.path.join(path, "sparkml"))
    m = Model(artifact_path, run_id, signature=signature)
    m.add_flavor(FLAVOR_NAME, pyspark_version="3.3.0-cdnaml", model_data="sparkml", model_class=type(spark_model)
                 .__module__ + "." + type(spark_model).__name__)
    m.add_flavor("python_function", loader_module="cdnaml.tracking.spark", data="sparkml", env="conda.yaml")
    write_common(path, m, input_example)


def log_model(spark_model, artifact_path, registered_model_name=None, input_example=None, signature=None, **kw):
    if not isinstance(spark_model, PipelineModel):
        raise TrackingException(f"Argument 'spark_model' should be a PipelineModel, got '{type(spark_model)}'")
    return log_to_run(lambda d, rid: save_model(spark_model, d, input_example, signature, rid, artifact_path),
                      artifact_path, registered_model_name)


def load_model(model_uri, dfs_tmpdir=None, dst_path=None):
    p = resolve(model_uri)
    return PipelineModel.load(os.path.join(p, "sparkml"))


class _PyFuncSparkModel:
    """pyfunc wrapper: pandas in -> predictions out, executed on the GPU."""

    def __init__(self, pm: PipelineModel):
        self.pm = pm

    def predict(self, pdf):
        from ..session import SparkSession
        s = SparkSession.builder.getOrCreate()
        out = self.pm.transform(s.createDataFrame(pdf)).select("prediction").toPandas()
        return out["prediction"].to_numpy()


def _load_pyfunc(path):
    return _PyFuncSparkModel(PipelineModel.load(path))
