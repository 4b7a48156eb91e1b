"""Storage layer: versioned Delta-style tables and file-system utilities."""
from .delta import DeltaError, DeltaTable  # noqa: F401
