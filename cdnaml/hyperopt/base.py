"""Trials bookkeeping with hyperopt's field names (ML 08:147; Labs/ML 08L:105)."""
from __future__ import annotations

import datetime
import threading
from typing import Any, Dict, List, Optional

from . import hp as _hp

STATUS_NEW = "new"
STATUS_RUNNING = "running"
STATUS_OK = "ok"
STATUS_FAIL = "fail"
STATUS_STRINGS = (STATUS_NEW, STATUS_RUNNING, STATUS_OK, STATUS_FAIL)
JOB_STATE_NEW, JOB_STATE_RUNNING, JOB_STATE_DONE, JOB_STATE_ERROR = 0, 1, 2, 3


class Trials:
    """Sequential trial store: ``fmin`` evaluates one configuration at a time (each
    evaluation may itself be a distributed multi-GPU fit)."""

    parallelism = 1
    asynchronous = False

    def __init__(self, exp_key=None):
        self._trials: List[dict] = []
        self._lock = threading.Lock()
        self.attachments: Dict[str, Any] = {}

    # ------------------------------------------------------------ storage
    def new_trial(self, vals: Dict[str, Any], space) -> dict:
        with self._lock:
            tid = len(self._trials)
            active = set(_hp.active_labels(space, vals)) if space is not None else set(vals)
            labels = list(_hp.nodes(space).keys()) if space is not None else list(vals)
            t = {"tid": tid, "state": JOB_STATE_NEW, "spec": None, "exp_key": None, "owner": None,
                 "version": 0, "book_time": None, "refresh_time": None,
                 "result": {"status": STATUS_NEW},
                 "misc": {"tid": tid, "cmd": ("domain_attachment", "FMinIter_Domain"), "workdir": None,
                          "idxs": {k: ([tid] if k in active else []) for k in labels},
                          "vals": {k: ([vals[k]] if k in active else []) for k in labels}}}
            self._trials.append(t)
            return t

    def refresh(self):
        pass

    # ------------------------------------------------------------ views
    @property
    def trials(self) -> List[dict]:
        return list(self._trials)

    def __len__(self):
        return len(self._trials)

    def __iter__(self):
        return iter(self._trials)

    def __getitem__(self, i):
        return self._trials[i]

    @property
    def tids(self):
        return [t["tid"] for t in self._trials]

    @property
    def results(self) -> List[dict]:
        return [t["result"] for t in self._trials]

    @property
    def miscs(self):
        return [t["misc"] for t in self._trials]

    @property
    def vals(self):
        out: Dict[str, list] = {}
        for t in self._trials:
            for k, v in t["misc"]["vals"].items():
                out.setdefault(k, []).extend(v)
        return out

    @property
    def idxs(self):
        out: Dict[str, list] = {}
        for t in self._trials:
            for k, v in t["misc"]["idxs"].items():
                out.setdefault(k, []).extend(v)
        return out

    def losses(self) -> List[Optional[float]]:
        return [t["result"].get("loss") for t in self._trials]

    def statuses(self) -> List[str]:
        return [t["result"].get("status") for t in self._trials]

    def _ok(self) -> List[dict]:
        return [t for t in self._trials if t["result"].get("status") == STATUS_OK and
                t["result"].get("loss") is not None]

    @property
    def best_trial(self) -> dict:
        ok = self._ok()
        if not ok:
            raise ValueError("no trial completed successfully (all trials failed)")
        return min(ok, key=lambda t: float(t["result"]["loss"]))

    @property
    def argmin(self) -> Dict[str, Any]:
        best = self.best_trial
        return {k: v[0] for k, v in best["misc"]["vals"].items() if v}

    def average_best_error(self):
        return float(self.best_trial["result"]["loss"])

    def history(self):
        """(assignment, loss) of completed OK trials, in tid order."""
        out = []
        for t in self._ok():
            a = {k: v[0] for k, v in t["misc"]["vals"].items() if v}
            out.append((a, float(t["result"]["loss"])))
        return out

    def count_by_state_unsynced(self, state):
        return sum(1 for t in self._trials if t["state"] == state)


def space_eval(space, hp_assignment: Dict[str, Any]):
    """Map ``fmin``'s argmin (choice indices) back to actual values."""
    return _hp.build(space, hp_assignment)


def _now():
    return datetime.datetime.now(datetime.timezone.utc)
