"""Simulated-annealing style proposals (``anneal.suggest``): perturb the best
assignment so far with a neighbourhood that shrinks as trials accumulate."""
from __future__ import annotations

import math

import numpy as np

from . import hp as _hp


def propose(space, history, rng, avg_best_idx: float = 2.0, shrink_coef: float = 0.1, **kw):
    if not history:
        return _hp.sample(space, rng)
    losses = np.array([l for _, l in history])
    # pick one of the best trials (geometric preference for the very best)
    order = np.argsort(losses, kind="stable")
    k = min(len(order) - 1, int(rng.geometric(1.0 / avg_best_idx)) - 1)
    base = history[int(order[k])][0]
    scale = 1.0 / (1.0 + shrink_coef * len(history))
    out = {}

    def rec(s):
        if isinstance(s, _hp.Apply):
            lab = s.label
            if lab not in base:
                v = s.sample_prior(rng)
            elif s.is_categorical:
                v = base[lab] if rng.uniform() > scale else s.sample_prior(rng)
            else:
                b = s.bounds
                x = math.log(max(base[lab], 1e-300)) if s.is_log else float(base[lab])
                if b is not None:
                    lo, hi = b
                    width = (hi - lo) * scale
                    x = float(np.clip(rng.normal(x, width), lo, hi))
                else:
                    x = float(rng.normal(x, s.args["sigma"] * scale))
                v = s._post(math.exp(x) if s.is_log else x)
                if s.kind == "uniformint":
                    v = int(round(v))
            out[lab] = v
            if s.kind == "choice":
                rec(s.args["options"][v])
            elif s.kind == "pchoice":
                rec(s.args["options"][v][1])
        elif isinstance(s, dict):
            for key in s:
                rec(s[key])
        elif isinstance(s, (list, tuple)):
            for x in s:
                rec(x)
    rec(space)
    return out


def suggest(*args, **kwargs):
    """Marker passed as ``algo=anneal.suggest``."""
    raise RuntimeError("anneal.suggest is an algorithm marker for fmin()")


suggest._propose = propose
