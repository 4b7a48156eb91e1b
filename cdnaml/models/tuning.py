"""Model selection (§2.9 P5).

``CrossValidator`` assigns folds from a Philox uniform keyed by (seed, GLOBAL
row id) — the same folds on 1 or 8 GPUs — materialises the fold-tagged data
once in HBM (``cache``), and evaluates folds × param maps.

For the engine's DecisionTree / RandomForest estimators -- bare or as the last
stage of a Pipeline -- the folds × maps run through ``tree/fused.py``: per fold
the prefix stages are fitted and the training rows binned once, and every map
of a (numTrees, maxDepth) grid is a prefix of one forest ("4 maps × 3 folds + 1
refit" = 3 forest fits + 1 refit), bit-identical to fitting each map.
Other estimators take the generic path: ``parallelism`` > 1 runs param maps
concurrently on separate HIP streams of the same GPU (single-process jobs); in
multi-GPU SPMD jobs each fit is itself data-parallel over all ranks and maps
run in lock-step order.  Reference: ML 07 - Random Forests and Hyperparameter
Tuning.py:72-158.
"""
from __future__ import annotations

import itertools
from concurrent.futures import ThreadPoolExecutor
from typing import Dict, List

import numpy as np
import torch

from ..sql import functions as F
from .base import Estimator, Model
from .param import NO_DEFAULT, Param, TypeConverters as TC, keyword_init
from .tree.fused import FusedTreeTuner


class ParamGridBuilder:
    def __init__(self):
        self._grid: Dict[Param, list] = {}

    def addGrid(self, param: Param, values):
        self._grid[param] = list(values)
        return self

    def baseOn(self, *args):
        if len(args) == 1 and isinstance(args[0], dict):
            for k, v in args[0].items():
                self.addGrid(k, [v])
        else:
            for k, v in args:
                self.addGrid(k, [v])
        return self

    def build(self) -> List[dict]:
        keys = list(self._grid)
        return [dict(zip(keys, vals)) for vals in itertools.product(*[self._grid[k] for k in keys])]


_TUNE = {
    "estimator": ("estimator to be cross-validated", None, None),
    "estimatorParamMaps": ("estimator param maps", None, None),
    "evaluator": ("evaluator used to select hyper-parameters that maximize the validator metric", None, None),
    "seed": ("random seed", None, TC.toInt),
    "parallelism": ("the number of threads to use when running parallel algorithms (>= 1)", 1, TC.toInt),
    "collectSubModels": ("whether to collect a list of sub-models trained during tuning", False, TC.toBoolean),
}


def _run_maps(est, maps, train, valid, evaluator, parallelism, session):
    """Fit + evaluate every param map on one (train, valid) split."""
    def one(pm):
        if session.device.type == "cuda" and parallelism > 1:
            with torch.cuda.stream(torch.cuda.Stream(session.device)):
                m = est.fit(train, pm)
                metric = evaluator.evaluate(m.transform(valid))
                torch.cuda.current_stream().synchronize()
                return m, metric
        m = est.fit(train, pm)
        return m, evaluator.evaluate(m.transform(valid))
    if parallelism > 1 and not session.comm.distributed:
        with ThreadPoolExecutor(max_workers=parallelism) as ex:
            return list(ex.map(one, maps))
    return [one(pm) for pm in maps]


class CrossValidator(Estimator):
    _params = dict(_TUNE, **{
        "numFolds": ("number of folds for cross validation", 3, TC.toInt),
        "foldCol": ("Param for the column name of user specified fold number", "", TC.toString),
    })

    def __init__(self, estimator=None, estimatorParamMaps=None, evaluator=None, numFolds=None, seed=None,
                 parallelism=None, collectSubModels=None, foldCol=None):
        super().__init__()
        keyword_init(self, dict(estimator=estimator, estimatorParamMaps=estimatorParamMaps, evaluator=evaluator,
                                numFolds=numFolds, seed=seed, parallelism=parallelism,
                                collectSubModels=collectSubModels, foldCol=foldCol))

    def copy(self, extra=None):
        that = super().copy(extra)
        est = self.getEstimator()
        if est is not None and extra:
            that._paramMap["estimator"] = est.copy(extra)
        return that

    def _fit(self, dataset):
        est = self.getEstimator()
        maps = self.getEstimatorParamMaps() or [{}]
        ev = self.getEvaluator()
        k = self.getNumFolds()
        seed = self.getSeed() if self.getSeed() is not None else 0x5EED
        session = dataset._session
        fold_col = self.getFoldCol()
        if fold_col:
            tagged = dataset.withColumn("__fold", F.col(fold_col).cast("int")).cache()
        else:
            tagged = dataset._with_global_uniform(seed, "__u").withColumn(
                "__fold", F.floor(F.col("__u") * k).cast("int")).drop("__u").cache()
        metrics = np.zeros((len(maps), k))
        subs = [[None] * len(maps) for _ in range(k)]
        fused = FusedTreeTuner(est, maps, dataset) if FusedTreeTuner.supported(est, maps) else None
        for f in range(k):
            valid = tagged.filter(F.col("__fold") == f).drop("__fold")
            train = tagged.filter(F.col("__fold") != f).drop("__fold")
            if fused is not None:
                # one prefix fit + one binned training set + one forest per map group for the fold, every map
                # a prefix of that forest: the generic path's models, bit for bit (tree/fused.py)
                train, valid = train.cache(), valid.cache()
                models, prefix = fused.fit_split(train)
                res = list(zip(models, fused.evaluate(models, prefix, valid, ev)))
                train.unpersist()
                valid.unpersist()
            else:
                res = _run_maps(est, maps, train, valid, ev, self.getParallelism(), session)
            for j, (m, met) in enumerate(res):
                metrics[j, f] = met
                if self.getCollectSubModels():
                    subs[f][j] = m
        avg = metrics.mean(1)
        std = metrics.std(1)
        best = int(np.argmax(avg) if ev.isLargerBetter() else np.argmin(avg))
        best_model = est.fit(dataset, maps[best])
        tagged.unpersist()
        cvm = CrossValidatorModel(best_model, avg.tolist(), subs if self.getCollectSubModels() else None,
                                  std.tolist())
        cvm._post_fit(self)
        return cvm

    def _sub_stages(self):
        return [self.getEstimator(), self.getEvaluator()]

    def _save_state(self):
        return {"paramMaps": _maps_json(self.getEstimatorParamMaps())}, {}

    def _load_state(self, extra, tensors, stages):
        self._paramMap["estimator"], self._paramMap["evaluator"] = stages[0], stages[1]
        self._paramMap["estimatorParamMaps"] = _maps_from_json(extra.get("paramMaps", []), stages[0])


def _maps_json(maps):
    out = []
    for m in maps or []:
        out.append([{"parent": p.parent, "name": p.name, "value": v} for p, v in m.items()])
    return out


def _maps_from_json(js, est):
    """Re-bind saved param maps to the (re-loaded) estimator tree by uid/name."""
    from .pipeline import Pipeline
    owners = {}

    def walk(o):
        if o is None:
            return
        owners[o.uid] = o
        if isinstance(o, Pipeline):
            for s in o.getStages():
                walk(s)
        if hasattr(o, "getEstimator") and callable(getattr(o, "getEstimator", None)):
            try:
                walk(o.getEstimator())
            except Exception:
                pass
    walk(est)
    maps = []
    for m in js:
        d = {}
        for e in m:
            o = owners.get(e["parent"])
            if o is not None and o.hasParam(e["name"]):
                d[o.getParam(e["name"])] = e["value"]
        maps.append(d)
    return maps


class CrossValidatorModel(Model):
    _params = dict(CrossValidator._params)

    def __init__(self, bestModel=None, avgMetrics=None, subModels=None, stdMetrics=None):
        super().__init__()
        self.bestModel = bestModel
        self.avgMetrics = list(avgMetrics or [])
        self.stdMetrics = list(stdMetrics or [])
        self.subModels = subModels

    def _transform(self, dataset):
        return self.bestModel.transform(dataset)

    def copy(self, extra=None):
        that = super().copy(extra)
        that.bestModel = self.bestModel.copy(extra) if self.bestModel is not None else None
        return that

    def _sub_stages(self):
        out = [self.bestModel]
        est, ev = self._get("estimator"), self._get("evaluator")
        if est is not None and ev is not None:
            out += [est, ev]
        return out

    def _save_state(self):
        return {"avgMetrics": self.avgMetrics, "stdMetrics": self.stdMetrics,
                "paramMaps": _maps_json(self._get("estimatorParamMaps"))}, {}

    def _load_state(self, extra, tensors, stages):
        self.bestModel = stages[0]
        self.avgMetrics = extra["avgMetrics"]
        self.stdMetrics = extra.get("stdMetrics", [])
        self.subModels = None
        if len(stages) >= 3:
            self._paramMap["estimator"], self._paramMap["evaluator"] = stages[1], stages[2]
            self._paramMap["estimatorParamMaps"] = _maps_from_json(extra.get("paramMaps", []), stages[1])


class TrainValidationSplit(Estimator):
    _params = dict(_TUNE, **{"trainRatio": ("ratio between training set and validation set (>= 0 && <= 1)", 0.75,
                                            TC.toFloat)})

    def __init__(self, estimator=None, estimatorParamMaps=None, evaluator=None, trainRatio=None, seed=None,
                 parallelism=None, collectSubModels=None):
        super().__init__()
        keyword_init(self, dict(estimator=estimator, estimatorParamMaps=estimatorParamMaps, evaluator=evaluator,
                                trainRatio=trainRatio, seed=seed, parallelism=parallelism,
                                collectSubModels=collectSubModels))

    def _fit(self, dataset):
        est, maps, ev = self.getEstimator(), self.getEstimatorParamMaps() or [{}], self.getEvaluator()
        seed = self.getSeed() if self.getSeed() is not None else 0x5EED
        tr = self.getTrainRatio()
        train, valid = dataset.randomSplit([tr, 1 - tr], seed)
        train, valid = train.cache(), valid.cache()
        if FusedTreeTuner.supported(est, maps):
            fused = FusedTreeTuner(est, maps, dataset)
            models, prefix = fused.fit_split(train)
            res = list(zip(models, fused.evaluate(models, prefix, valid, ev)))
        else:
            res = _run_maps(est, maps, train, valid, ev, self.getParallelism(), dataset._session)
        metrics = [m for _, m in res]
        best = int(np.argmax(metrics) if ev.isLargerBetter() else np.argmin(metrics))
        bm = est.fit(dataset, maps[best])
        tvm = TrainValidationSplitModel(bm, metrics, [m for m, _ in res] if self.getCollectSubModels() else None)
        tvm._post_fit(self)
        return tvm


class TrainValidationSplitModel(Model):
    _params = dict(TrainValidationSplit._params)

    def __init__(self, bestModel=None, validationMetrics=None, subModels=None):
        super().__init__()
        self.bestModel = bestModel
        self.validationMetrics = list(validationMetrics or [])
        self.subModels = subModels

    def _transform(self, dataset):
        return self.bestModel.transform(dataset)

    def _sub_stages(self):
        return [self.bestModel]

    def _save_state(self):
        return {"validationMetrics": self.validationMetrics}, {}

    def _load_state(self, extra, tensors, stages):
        self.bestModel = stages[0]
        self.validationMetrics = extra["validationMetrics"]
