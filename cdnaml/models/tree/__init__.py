"""Histogram tree learning engine shared by DT / RF / GBT / XGBoost-style models."""
from .binning import BinnedData, make_binned  # noqa: F401
from .engine import ForestTrainer, TreeParams  # noqa: F401
from .forest import Forest  # noqa: F401
