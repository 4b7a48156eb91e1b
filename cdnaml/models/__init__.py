"""ML library: Params, Pipelines, feature transformers, algorithms, evaluators, tuning."""
from .base import Estimator, Evaluator, Model, Transformer  # noqa: F401
from .pipeline import Pipeline, PipelineModel  # noqa: F401
