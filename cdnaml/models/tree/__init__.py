"""Histogram tree learning engine shared by DT / RF / GBT / XGBoost-style models."""
from .engine import BinnedData, Forest, ForestTrainer, TreeParams, make_binned  # noqa: F401
