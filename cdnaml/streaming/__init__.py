"""Structured streaming (micro-batch file sources and sinks)."""
from .stream import (DataStreamReader, DataStreamWriter, StreamingQuery, StreamingQueryException,  # noqa: F401
                     StreamingQueryManager)
