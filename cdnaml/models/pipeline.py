"""Pipeline / PipelineModel.

``Pipeline(stages=[…]).fit(df)`` fits estimators in order, transforming the
data between them; ``PipelineModel.stages[-1]`` is the last fitted stage; a
CrossValidator may itself be a stage (ML 07:143-149; Labs/ML 07L:151-166).
"""
from __future__ import annotations

from .base import Estimator, Model, Transformer
from .param import keyword_init


class Pipeline(Estimator):
    _params = {"stages": ("a list of pipeline stages", [], None)}

    def __init__(self, stages=None):
        super().__init__()
        if stages is not None:
            self.set("stages", list(stages))

    def setStages(self, stages):
        return self.set("stages", list(stages))

    def getStages(self):
        return list(self.getOrDefault("stages"))

    def copy(self, extra=None):
        that = super().copy(extra)
        that._paramMap["stages"] = [s.copy(extra) for s in self.getStages()]
        return that

    def _fit(self, dataset):
        stages = self.getStages()
        last_est = max((i for i, s in enumerate(stages) if isinstance(s, Estimator)), default=-1)
        fitted = []
        df = dataset
        for i, s in enumerate(stages):
            if isinstance(s, Estimator):
                m = s.fit(df)
                fitted.append(m)
                if i < last_est:
                    df = m.transform(df)
            else:
                fitted.append(s)
                if i < last_est:
                    df = s.transform(df)
        pm = PipelineModel(fitted)
        pm.uid = self.uid
        return pm

    def _sub_stages(self):
        return self.getStages()

    def _save_state(self):
        return {"numStages": len(self.getStages())}, {}

    def _load_state(self, extra, tensors, stages):
        self._paramMap["stages"] = stages


class PipelineModel(Model):
    def __init__(self, stages=None):
        super().__init__()
        self.stages = list(stages or [])

    def _transform(self, dataset):
        df = dataset
        for s in self.stages:
            df = s.transform(df)
        return df

    def copy(self, extra=None):
        that = super().copy(extra)
        that.stages = [s.copy(extra) for s in self.stages]
        return that

    def _sub_stages(self):
        return self.stages

    def _save_state(self):
        return {"numStages": len(self.stages)}, {}

    def _load_state(self, extra, tensors, stages):
        self.stages = stages
