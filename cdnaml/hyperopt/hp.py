"""Search-space language: ``hp.choice``, ``hp.uniform``, ``hp.quniform``, ``hp.loguniform`` …

Each call returns an :class:`Apply` node; spaces are arbitrary nests of
dicts / lists / tuples containing nodes.  ``sample`` draws a flat assignment
``{label: value}`` (choice -> index) and ``build`` turns an assignment back
into the user's nested structure.
"""
from __future__ import annotations

import math
from typing import Any, Dict, List

import numpy as np


class Apply:
    kind = "apply"

    def __init__(self, label: str, kind: str, **args):
        self.label = label
        self.kind = kind
        self.args = args

    def __repr__(self):
        return f"hp.{self.kind}({self.label!r}, {self.args})"

    # ---- prior sampling
    def sample_prior(self, rng: np.random.Generator):
        a = self.args
        k = self.kind
        if k == "choice":
            return int(rng.integers(0, len(a["options"])))
        if k == "pchoice":
            p = np.asarray([w for w, _ in a["options"]], dtype=float)
            return int(rng.choice(len(p), p=p / p.sum()))
        if k == "randint":
            return int(rng.integers(a["low"], a["high"]))
        if k == "uniformint":
            return int(round(rng.uniform(a["low"], a["high"])))
        x = self._raw_prior(rng)
        return self._post(x)

    def _raw_prior(self, rng):
        a = self.args
        k = self.kind
        if k in ("uniform", "quniform"):
            return rng.uniform(a["low"], a["high"])
        if k in ("loguniform", "qloguniform"):
            return math.exp(rng.uniform(a["low"], a["high"]))
        if k in ("normal", "qnormal"):
            return rng.normal(a["mu"], a["sigma"])
        if k in ("lognormal", "qlognormal"):
            return math.exp(rng.normal(a["mu"], a["sigma"]))
        raise ValueError(k)

    def _post(self, x):
        q = self.args.get("q")
        if q is not None and self.kind.startswith("q"):
            return float(np.round(x / q) * q)
        return float(x)

    # ---- transform to the sampling ("latent") space used by TPE
    @property
    def is_log(self) -> bool:
        return self.kind in ("loguniform", "qloguniform", "lognormal", "qlognormal")

    @property
    def bounds(self):
        a = self.args
        if "low" in a and self.kind not in ("randint",):
            return a["low"], a["high"]
        if self.kind == "randint":
            return a["low"], a["high"] - 1
        return None

    @property
    def is_categorical(self) -> bool:
        return self.kind in ("choice", "pchoice", "randint")

    @property
    def n_options(self) -> int:
        if self.kind == "choice":
            return len(self.args["options"])
        if self.kind == "pchoice":
            return len(self.args["options"])
        if self.kind == "randint":
            return int(self.args["high"] - self.args["low"])
        return 0


def choice(label: str, options: List[Any]) -> Apply:
    return Apply(label, "choice", options=list(options))


def pchoice(label: str, p_options) -> Apply:
    return Apply(label, "pchoice", options=list(p_options))


def uniform(label: str, low: float, high: float) -> Apply:
    return Apply(label, "uniform", low=float(low), high=float(high))


def quniform(label: str, low: float, high: float, q: float) -> Apply:
    return Apply(label, "quniform", low=float(low), high=float(high), q=float(q))


def loguniform(label: str, low: float, high: float) -> Apply:
    return Apply(label, "loguniform", low=float(low), high=float(high))


def qloguniform(label: str, low: float, high: float, q: float) -> Apply:
    return Apply(label, "qloguniform", low=float(low), high=float(high), q=float(q))


def normal(label: str, mu: float, sigma: float) -> Apply:
    return Apply(label, "normal", mu=float(mu), sigma=float(sigma))


def qnormal(label: str, mu: float, sigma: float, q: float) -> Apply:
    return Apply(label, "qnormal", mu=float(mu), sigma=float(sigma), q=float(q))


def lognormal(label: str, mu: float, sigma: float) -> Apply:
    return Apply(label, "lognormal", mu=float(mu), sigma=float(sigma))


def qlognormal(label: str, mu: float, sigma: float, q: float) -> Apply:
    return Apply(label, "qlognormal", mu=float(mu), sigma=float(sigma), q=float(q))


def randint(label: str, low: int, high: int = None) -> Apply:
    if high is None:
        low, high = 0, low
    return Apply(label, "randint", low=int(low), high=int(high))


def uniformint(label: str, low: int, high: int) -> Apply:
    return Apply(label, "uniformint", low=int(low), high=int(high))


# ------------------------------------------------------------ space walking
def nodes(space) -> Dict[str, Apply]:
    """All hp nodes by label, including those nested inside choice options."""
    out: Dict[str, Apply] = {}

    def rec(s):
        if isinstance(s, Apply):
            if s.label in out and out[s.label] is not s:
                raise ValueError(f"duplicate hyperparameter label {s.label!r}")
            out[s.label] = s
            if s.kind == "choice":
                for o in s.args["options"]:
                    rec(o)
            elif s.kind == "pchoice":
                for _, o in s.args["options"]:
                    rec(o)
        elif isinstance(s, dict):
            for v in s.values():
                rec(v)
        elif isinstance(s, (list, tuple)):
            for v in s:
                rec(v)
    rec(space)
    return out


def active_labels(space, assignment: Dict[str, Any]) -> List[str]:
    """Labels actually used by ``assignment`` (conditional spaces)."""
    used: List[str] = []

    def rec(s):
        if isinstance(s, Apply):
            used.append(s.label)
            if s.kind in ("choice", "pchoice"):
                opts = s.args["options"]
                o = opts[int(assignment[s.label])]
                rec(o[1] if s.kind == "pchoice" else o)
        elif isinstance(s, dict):
            for v in s.values():
                rec(v)
        elif isinstance(s, (list, tuple)):
            for v in s:
                rec(v)
    rec(space)
    return used


def build(space, assignment: Dict[str, Any]):
    """Assignment (choice = index) -> the user's nested structure of values."""
    if isinstance(space, Apply):
        v = assignment[space.label]
        if space.kind == "choice":
            return build(space.args["options"][int(v)], assignment)
        if space.kind == "pchoice":
            return build(space.args["options"][int(v)][1], assignment)
        if space.kind == "randint":
            return int(v)
        return v
    if isinstance(space, dict):
        return {k: build(v, assignment) for k, v in space.items()}
    if isinstance(space, list):
        return [build(v, assignment) for v in space]
    if isinstance(space, tuple):
        return tuple(build(v, assignment) for v in space)
    return space


def sample(space, rng: np.random.Generator) -> Dict[str, Any]:
    out: Dict[str, Any] = {}

    def rec(s):
        if isinstance(s, Apply):
            v = s.sample_prior(rng)
            out[s.label] = v
            if s.kind == "choice":
                rec(s.args["options"][v])
            elif s.kind == "pchoice":
                rec(s.args["options"][v][1])
        elif isinstance(s, dict):
            for k in s:
                rec(s[k])
        elif isinstance(s, (list, tuple)):
            for v in s:
                rec(v)
    rec(space)
    return out
