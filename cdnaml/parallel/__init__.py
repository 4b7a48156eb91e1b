"""Distributed execution: RCCL/gloo collectives and shuffles."""
from .comm import Comm, init_from_env  # noqa: F401
