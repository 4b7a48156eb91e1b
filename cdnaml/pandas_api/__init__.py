"""pandas API on the engine (Koalas; ML 14 - Koalas.py:41-194).

``import cdnaml.pandas_api as ks`` (or ``databricks.koalas`` / ``pyspark.pandas``
through :mod:`cdnaml.compat`):  ``ks.read_parquet``, ``ks.DataFrame(sdf)``,
``sdf.to_koalas()`` / ``kdf.to_spark()``, ``kdf[col].value_counts()``,
``kdf.filter(items=…)``, ``kdf.plot.hist(…)``, ``ks.sql("… {kdf}")`` and the
options system (``compute.default_index_type``, ``plotting.backend`` …).

Like Koalas' immutable InternalFrame, a pandas-API frame is an engine
DataFrame plus index metadata (an explicit index column); every operation
builds a new engine plan and nothing is collected until ``to_pandas`` /
``head`` / plotting.
"""
from .config import get_option, option_context, options, reset_option, set_option  # noqa: F401
from .frame import DataFrame, Series, from_pandas, from_spark  # noqa: F401
from .namespace import (concat, read_csv, read_delta, read_json, read_parquet, read_table, sql,  # noqa: F401
                        to_datetime)
