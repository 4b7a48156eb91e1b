"""Hyperopt-compatible tuning (ML 08 - Hyperopt.py:106-153,
Labs/ML 08L:56-112).

``fmin(fn, space, algo=tpe.suggest, max_evals, trials, rstate)`` with the
``hp`` space language, ``Trials`` (sequential driver loop around distributed
fits — ML 08:17-23) and ``SparkTrials`` / ``GPUTrials`` (concurrent trials —
Labs/ML 08L:89-112).  The hyperopt package is not installed; this is an
independent implementation of the subset the course uses, with the same
return conventions (``hp.choice`` best values are INDICES, L08:118).

GPUTrials on MI355X: trials run concurrently in worker threads, each bound to
its own HIP stream (and, with several visible GPUs, its own device), so
independent single-node fits overlap on the chip.  In an SPMD job every rank
runs the same driver loop (the proposer is deterministic given ``rstate``),
which keeps distributed fits inside ``fn`` collective-consistent.
"""
from .base import (STATUS_FAIL, STATUS_NEW, STATUS_OK, STATUS_RUNNING, JOB_STATE_DONE, Trials,  # noqa: F401
                   space_eval)
from .fmin import fmin  # noqa: F401
from .parallel import GPUTrials, SparkTrials  # noqa: F401
from . import hp, rand, tpe, anneal  # noqa: F401
from .early_stop import no_progress_loss  # noqa: F401
