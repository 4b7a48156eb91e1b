from ..models.evaluation import (BinaryClassificationEvaluator, ClusteringEvaluator,  # noqa: F401
                                 MulticlassClassificationEvaluator, RegressionEvaluator)
from ..models.base import Evaluator  # noqa: F401
