"""Random search (``rand.suggest``): independent draws from the prior."""
from __future__ import annotations

from . import hp as _hp


def propose(space, history, rng, **kw):
    return _hp.sample(space, rng)


def suggest(*args, **kwargs):
    """Marker passed as ``algo=rand.suggest``."""
    raise RuntimeError("rand.suggest is an algorithm marker for fmin()")


suggest._propose = propose
