"""``pyspark.sql``-compatible namespace: session, DataFrame, Column, Row, functions, types."""
from . import functions, types  # noqa: F401
from .column import AnalysisException, Column  # noqa: F401
from .dataframe import DataFrame  # noqa: F401
from .group import GroupedData  # noqa: F401
from .types import Row  # noqa: F401


def __getattr__(name):
    if name == "SparkSession":
        from ..session import SparkSession
        return SparkSession
    raise AttributeError(name)
