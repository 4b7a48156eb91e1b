"""``pyspark.ml``-compatible namespace over :mod:`cdnaml.models`."""
from ..models.base import Estimator, Evaluator, Model, Transformer  # noqa: F401
from ..models.pipeline import Pipeline, PipelineModel  # noqa: F401
