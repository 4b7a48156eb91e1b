"""Tree-structured Parzen Estimator proposals (``tpe.suggest``).

Per hyperparameter (conditional labels only see trials where they were
active): split completed trials at the γ-quantile of the loss into "good" and
"bad", fit adaptive-bandwidth Parzen mixtures l(x) (good) and g(x) (bad) —
Gaussian kernels in the latent (linear or log) space, truncated to the
bounds, with the prior as one extra component — and among ``n_EI_candidates``
draws from l keep the one maximising l(x)/g(x).  Categorical labels use
smoothed counts.  The first ``n_startup_jobs`` proposals sample the prior.
"""
from __future__ import annotations

import math
from typing import Any, Dict, List, Tuple

import numpy as np

from . import hp as _hp

_DEFAULT = dict(n_startup_jobs=20, gamma=0.25, n_EI_candidates=24, prior_weight=1.0)


def _latent(node: _hp.Apply, v: float) -> float:
    return math.log(max(v, 1e-300)) if node.is_log else float(v)


def _prior(node: _hp.Apply) -> Tuple[float, float, float, float]:
    """(mu, sigma, low, high) in latent space."""
    a = node.args
    if "low" in a:
        lo, hi = a["low"], a["high"]
        if node.kind == "uniformint":
            lo, hi = lo - 0.5, hi + 0.5
        return (lo + hi) / 2.0, (hi - lo), lo, hi
    return a["mu"], a["sigma"], -math.inf, math.inf


def _parzen(obs: np.ndarray, prior_mu: float, prior_sigma: float, prior_w: float):
    """Adaptive Parzen estimator: one kernel per observation plus the prior; each
    bandwidth is the larger gap to its sorted neighbours, clipped to
    [prior_sigma / min(100, 1 + n), prior_sigma]."""
    mus = np.append(np.asarray(obs, dtype=float), prior_mu)
    order = np.argsort(mus, kind="stable")
    sm = mus[order]
    n = len(sm)
    prior_pos = int(np.where(order == n - 1)[0][0])
    if n == 1:
        sig = np.array([prior_sigma], dtype=float)
    else:
        gaps = np.diff(sm)
        sig = np.empty(n)
        sig[0], sig[-1] = gaps[0], gaps[-1]
        if n > 2:
            sig[1:-1] = np.maximum(gaps[:-1], gaps[1:])
    sig = np.clip(sig, prior_sigma / min(100.0, 1.0 + n), prior_sigma)
    sig[prior_pos] = prior_sigma
    w = np.ones(n)
    w[prior_pos] = prior_w
    return w / w.sum(), sm, sig


def _norm_cdf(x):
    return 0.5 * (1.0 + np.vectorize(math.erf)(x / math.sqrt(2.0)))


def _gmm_logpdf(x: np.ndarray, w, mu, sig, lo, hi, q=None, log_space=False):
    x = np.asarray(x, dtype=float)[:, None]
    if q is None:
        z = (x - mu[None]) / sig[None]
        logk = -0.5 * z * z - np.log(sig[None] * math.sqrt(2 * math.pi))
        mass = _norm_cdf((hi - mu) / sig) - _norm_cdf((lo - mu) / sig) if np.isfinite([lo, hi]).any() else \
            np.ones_like(mu)
        logk = logk - np.log(np.maximum(mass, 1e-300))[None]
        return _logsumexp(logk + np.log(np.maximum(w, 1e-300))[None], 1)
    # quantised: probability mass of the rounding interval (in the value space)
    xv = np.exp(x) if log_space else x
    ub = xv + q / 2.0
    lb = xv - q / 2.0
    if log_space:
        ub, lb = np.log(np.maximum(ub, 1e-300)), np.log(np.maximum(lb, 1e-300))
    p = (_norm_cdf((ub - mu[None]) / sig[None]) - _norm_cdf((lb - mu[None]) / sig[None]))
    mass = _norm_cdf((hi - mu) / sig) - _norm_cdf((lo - mu) / sig) if np.isfinite([lo, hi]).any() else \
        np.ones_like(mu)
    p = p / np.maximum(mass, 1e-300)[None]
    return np.log(np.maximum((p * w[None]).sum(1), 1e-300))


def _logsumexp(a, axis):
    m = a.max(axis=axis, keepdims=True)
    return (m + np.log(np.exp(a - m).sum(axis=axis, keepdims=True))).squeeze(axis)


def _sample_gmm(rng, n, w, mu, sig, lo, hi):
    out = np.empty(n)
    for i in range(n):
        for _ in range(100):
            k = rng.choice(len(w), p=w)
            v = rng.normal(mu[k], sig[k])
            if lo <= v <= hi:
                break
        else:
            v = min(max(v, lo), hi)
        out[i] = v
    return out


def _propose_numeric(node, good, bad, rng, cfg):
    mu0, s0, lo, hi = _prior(node)
    lg = np.array([_latent(node, v) for v in good], dtype=float)
    lb = np.array([_latent(node, v) for v in bad], dtype=float)
    wg, mg, sg = _parzen(lg, mu0, s0, cfg["prior_weight"])
    wb, mb, sb = _parzen(lb, mu0, s0, cfg["prior_weight"])
    cand = _sample_gmm(rng, cfg["n_EI_candidates"], wg, mg, sg, lo, hi)
    q = node.args.get("q") if node.kind.startswith("q") else None
    if q is not None:
        vals = np.round((np.exp(cand) if node.is_log else cand) / q) * q
        latent = np.log(np.maximum(vals, 1e-300)) if node.is_log else vals
    else:
        latent = cand
    score = _gmm_logpdf(latent, wg, mg, sg, lo, hi, q, node.is_log) - \
        _gmm_logpdf(latent, wb, mb, sb, lo, hi, q, node.is_log)
    best = latent[int(np.argmax(score))]
    v = math.exp(best) if node.is_log else float(best)
    if q is not None:
        v = float(np.round(v / q) * q)
    if node.kind == "uniformint":
        v = int(round(v))
    return v


def _propose_categorical(node, good, bad, rng, cfg):
    k = node.n_options
    if node.kind == "pchoice":
        prior = np.array([w for w, _ in node.args["options"]], dtype=float)
        prior /= prior.sum()
    else:
        prior = np.full(k, 1.0 / k)
    off = node.args["low"] if node.kind == "randint" else 0
    cg = np.bincount(np.asarray(good, dtype=int) - off, minlength=k)[:k].astype(float)
    cb = np.bincount(np.asarray(bad, dtype=int) - off, minlength=k)[:k].astype(float)
    pw = cfg["prior_weight"]
    pg = (cg + pw * prior * k) / (cg.sum() + pw * k)
    pb = (cb + pw * prior * k) / (cb.sum() + pw * k)
    cand = rng.choice(k, size=cfg["n_EI_candidates"], p=pg / pg.sum())
    score = np.log(pg[cand]) - np.log(pb[cand])
    return int(cand[int(np.argmax(score))]) + off


def propose(space, history: List[Tuple[Dict[str, Any], float]], rng: np.random.Generator, **kw) -> Dict[str, Any]:
    cfg = dict(_DEFAULT, **{k: v for k, v in kw.items() if k in _DEFAULT})
    if len(history) < cfg["n_startup_jobs"]:
        return _hp.sample(space, rng)
    losses = np.array([l for _, l in history])
    order = np.argsort(losses, kind="stable")
    n_below = int(math.ceil(cfg["gamma"] * math.sqrt(len(history))))
    good_idx = set(order[:n_below].tolist())
    out: Dict[str, Any] = {}

    def rec(s):
        if isinstance(s, _hp.Apply):
            good = [a[s.label] for i, (a, _) in enumerate(history) if i in good_idx and s.label in a]
            bad = [a[s.label] for i, (a, _) in enumerate(history) if i not in good_idx and s.label in a]
            if s.is_categorical:
                v = _propose_categorical(s, good, bad, rng, cfg)
            else:
                v = _propose_numeric(s, good, bad, rng, cfg)
            out[s.label] = v
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
    """Marker passed as ``algo=tpe.suggest``; ``fmin`` calls :func:`propose`."""
    raise RuntimeError("tpe.suggest is an algorithm marker for fmin(); call fmin(..., algo=tpe.suggest)")


suggest._propose = propose
