"""cdnaml — an MI355X-native distributed tabular-ML engine.

Spark-compatible DataFrame/SQL + MLlib-style Pipelines whose hot paths are
hand-written gfx950 HIP kernels (MFMA Gram, LDS histograms, tree predict)
and whose distributed collectives run over RCCL/xGMI, one process per GPU.
See SURVEY.md for the component map and README.md for usage.
"""
__version__ = "0.1.0"

from .session import SparkSession  # noqa: F401,E402
from .sql import functions, types  # noqa: F401,E402
from .sql.column import Column  # noqa: F401,E402
from .sql.dataframe import DataFrame  # noqa: F401,E402
from .sql.types import Row  # noqa: F401,E402
