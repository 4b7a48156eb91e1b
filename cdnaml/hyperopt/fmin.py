"""``fmin``: the driver loop (ML 08 - Hyperopt.py:140-153; Labs/ML 08L:98-112)."""
from __future__ import annotations

import functools
import math
import time
import traceback
from typing import Any, Callable, Dict, Optional

import numpy as np

from . import hp as _hp
from .base import JOB_STATE_DONE, JOB_STATE_ERROR, JOB_STATE_RUNNING, STATUS_FAIL, STATUS_OK, Trials, _now


def _resolve_algo(algo):
    """algo = tpe.suggest / rand.suggest / anneal.suggest, possibly functools.partial'd."""
    kw: Dict[str, Any] = {}
    if isinstance(algo, functools.partial):
        kw = dict(algo.keywords or {})
        algo = algo.func
    if algo is None:
        from . import tpe
        algo = tpe.suggest
    prop = getattr(algo, "_propose", None)
    if prop is None:
        raise ValueError(f"unsupported algo {algo!r}: use tpe.suggest, rand.suggest or anneal.suggest")
    return prop, kw


def _as_generator(rstate) -> np.random.Generator:
    if rstate is None:
        return np.random.default_rng()
    if isinstance(rstate, np.random.Generator):
        return rstate
    if isinstance(rstate, np.random.RandomState):
        return np.random.default_rng(int(rstate.randint(0, 2 ** 31 - 1)))
    return np.random.default_rng(int(rstate))


def _normalise_result(r) -> dict:
    if isinstance(r, dict):
        out = dict(r)
        out.setdefault("status", STATUS_OK if "loss" in out else STATUS_FAIL)
        if out.get("loss") is not None:
            out["loss"] = float(out["loss"])
        return out
    v = float(r)
    if math.isnan(v):
        return {"status": STATUS_FAIL, "loss": None, "failure": "loss is NaN"}
    return {"status": STATUS_OK, "loss": v}


def evaluate_trial(fn: Callable, space, trial: dict, catch: bool) -> dict:
    vals = {k: v[0] for k, v in trial["misc"]["vals"].items() if v}
    args = _hp.build(space, vals)
    trial["state"] = JOB_STATE_RUNNING
    trial["book_time"] = _now()
    try:
        res = _normalise_result(fn(args))
        trial["state"] = JOB_STATE_DONE
    except Exception as e:  # noqa: BLE001
        if not catch:
            trial["state"] = JOB_STATE_ERROR
            trial["result"] = {"status": STATUS_FAIL, "failure": repr(e)}
            raise
        res = {"status": STATUS_FAIL, "failure": repr(e), "traceback": traceback.format_exc()}
        trial["state"] = JOB_STATE_ERROR
    trial["result"] = res
    trial["refresh_time"] = _now()
    return res


def fmin(fn: Callable, space, algo=None, max_evals: Optional[int] = None, timeout: Optional[float] = None,
         loss_threshold: Optional[float] = None, trials: Optional[Trials] = None, rstate=None,
         allow_trials_fmin: bool = True, pass_expr_memo_ctrl=None, catch_eval_exceptions: bool = False,
         verbose: bool = False, return_argmin: bool = True, points_to_evaluate=None, max_queue_len: int = 1,
         show_progressbar: bool = False, early_stop_fn=None, trials_save_file: str = ""):
    """Minimise ``fn`` over ``space``; returns the best assignment (choice -> index)."""
    if max_evals is None and timeout is None:
        raise ValueError("fmin needs max_evals or timeout")
    max_evals = max_evals if max_evals is not None else 2 ** 31 - 1
    trials = trials if trials is not None else Trials()
    propose, akw = _resolve_algo(algo)
    rng = _as_generator(rstate)
    _hp.nodes(space)  # validates labels
    t0 = time.time()
    queue = list(points_to_evaluate or [])
    stop_state = None

    def next_assignment():
        if queue:
            p = queue.pop(0)
            full = _hp.sample(space, rng)
            full.update(p)
            return full
        return propose(space, trials.history(), rng, **akw)

    def should_stop():
        nonlocal stop_state
        if len(trials) >= max_evals:
            return True
        if timeout is not None and time.time() - t0 >= timeout:
            return True
        if loss_threshold is not None:
            ok = [l for l in trials.losses() if l is not None]
            if ok and min(ok) <= loss_threshold:
                return True
        if early_stop_fn is not None and len(trials):
            args = [] if stop_state is None else stop_state
            stop, stop_state = early_stop_fn(trials, *args)
            if stop:
                return True
        return False

    from ..models.tree import bincache
    runner = getattr(trials, "_run_parallel", None)
    # the trials of this search share binned training data (the same features re-binned per trial otherwise);
    # the cache lives only until fmin returns
    with bincache.scope():
        if runner is not None and getattr(trials, "parallelism", 1) > 1:
            runner(fn, space, next_assignment, should_stop, max_evals, catch_eval_exceptions)
        else:
            log = _TrialLogger(trials)
            while not should_stop():
                a = next_assignment()
                tr = trials.new_trial(a, space)
                evaluate_trial(fn, space, tr, catch_eval_exceptions)
                log.log(tr, a)
            log.close()
    if not return_argmin:
        return trials
    return trials.argmin


class _TrialLogger:
    """Logs trials as nested tracking runs when autologging is on or the trials
    object asks for it (SparkTrials on Databricks are auto-logged, L08:89)."""

    def __init__(self, trials):
        from ..tracking import autologging, fluent
        self.enabled = bool(getattr(trials, "_autolog", False)) or autologging.is_enabled()
        self.parent = None
        self.fluent = fluent
        if self.enabled:
            ar = fluent.active_run()
            self.parent = ar.info.run_id if ar is not None else None

    def log(self, trial, assignment):
        if not self.enabled or self.parent is None:
            return
        from ..tracking import MlflowClient
        c = MlflowClient()
        exp = self.fluent.get_run(self.parent).info.experiment_id
        r = c.create_run(exp, tags={"mlflow.parentRunId": self.parent, "trial_id": str(trial["tid"])},
                         run_name=f"trial-{trial['tid']}")
        for k, v in assignment.items():
            c.log_param(r.info.run_id, k, v)
        loss = trial["result"].get("loss")
        if loss is not None:
            c.log_metric(r.info.run_id, "loss", float(loss))
        c.set_terminated(r.info.run_id, "FINISHED" if trial["result"].get("status") == STATUS_OK else "FAILED")

    def close(self):
        pass
