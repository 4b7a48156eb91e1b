"""Estimator / Transformer / Model / Evaluator contracts.

A Transformer appends columns to a DataFrame; an Estimator's ``fit``
returns a Model (itself a Transformer) — ML 01 - Data Cleansing.py:242-256.
Every ``fit`` passes through the tracking autolog hook (ML 08:144).
"""
from __future__ import annotations

from typing import Optional

from .param import Params
from .persistence import MLReadable, MLWritable


class Transformer(Params, MLWritable, MLReadable):
    def transform(self, dataset, params: Optional[dict] = None):
        if params:
            return self.copy(params)._transform(dataset)
        return self._transform(dataset)

    def _transform(self, dataset):  # pragma: no cover - abstract
        raise NotImplementedError


class Estimator(Params, MLWritable, MLReadable):
    def fit(self, dataset, params=None):
        if isinstance(params, (list, tuple)):
            return [self.fit(dataset, p) for p in params]
        est = self.copy(params) if params else self
        from ..tracking import autologging as _al
        return _al.wrap_fit(est, dataset)

    def fitMultiple(self, dataset, paramMaps):
        for i, pm in enumerate(paramMaps):
            yield i, self.fit(dataset, pm)

    def _fit(self, dataset):  # pragma: no cover - abstract
        raise NotImplementedError


class Model(Transformer):
    parent = None

    def _post_fit(self, estimator):
        self.parent = estimator
        estimator._copyValues(self)
        return self


class Evaluator(Params, MLWritable, MLReadable):
    def evaluate(self, dataset, params=None):
        if params:
            return self.copy(params)._evaluate(dataset)
        return self._evaluate(dataset)

    def _evaluate(self, dataset):  # pragma: no cover
        raise NotImplementedError

    def isLargerBetter(self) -> bool:
        return True


class UnaryTransformer(Transformer):
    pass
