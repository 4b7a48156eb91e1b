"""Native compute ops (hand-written gfx950 HIP kernels with CPU references)."""
from . import _lib, kernels, philox  # noqa: F401
from .kernels import *  # noqa: F401,F403


def build(force: bool = False, verbose: bool = False) -> str:
    return _lib.build(force=force, verbose=verbose)


def native_available() -> bool:
    return _lib.available()
