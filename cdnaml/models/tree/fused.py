"""Fused tree-ensemble tuning: CrossValidator / TrainValidationSplit over a tree estimator, or over a
``Pipeline`` ending in one, fit once per data split instead of once per param map
(ML 07 - Random Forests and Hyperparameter Tuning.py:72-158 -- the CV of
``Pipeline([StringIndexer, VectorAssembler, rf])`` at ML 07:107 --, Labs/ML 07L - Hyperparameter Tuning
Lab.py:105-141).

The generic tuner fits every (fold, param map) pair from scratch: the course's 2 x 2 grid with 3 folds is
12 fits + 1 refit, each re-fitting the pipeline's prefix stages, re-sampling quantiles, re-binning and
re-drawing bootstraps.  Two facts make most of that work shared WITHOUT changing any result:

* Everything up to the tree estimator's histograms depends on the split's training rows, the prefix
  stages and (maxBins, seed) only -- not on ``numTrees`` / ``maxDepth``.  Per split, the prefix stages are
  fitted once, the training rows transformed once, and the binned matrix built once, exactly as one
  generic fit on that split builds them (the same filtered DataFrame, the same global row ids, the same
  quantile sample and Poisson streams).
* Tree t of a forest sees bootstrap stream (seed, t) and feature subsets hashed from (seed, t, node), and
  its level-d histograms are exact integers.  So among maps that differ only in ``numTrees`` and
  ``maxDepth``, every model is a prefix of the largest one: the first ``numTrees`` trees, cut at
  ``maxDepth`` (a node at depth D keeps its stored leaf value).  One forest per split, with the largest
  numTrees and maxDepth of the group, gives the whole grid.

Hence the fused CV's ``avgMetrics``, ``bestModel`` and sub-models are bit-identical to the generic path's
(``tests/test_tuning_fused.py`` pins it for bare estimators and pipelines): the 2 x 2 x 3 grid becomes 3
forest fits + 1 refit.  Maps are grouped by everything else (including the resolved feature-subset size,
and numTrees == 1, which switches off bagging); regression groups also split at maxDepth 8 (a different
histogram path).  A Pipeline qualifies when its last stage is one of the engine's DecisionTree /
RandomForest estimators and every param map touches that stage only.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from ...ops import kernels as K
from .engine import ForestTrainer, TreeParams
from .forest import Forest, freeze_cut

FUSED_TUNING = os.environ.get("CDNAML_FUSED_TUNING", "1") != "0"

_VARYING = ("numTrees", "maxDepth")
_IGNORED = ("predictionCol", "rawPredictionCol", "probabilityCol", "varianceCol", "leafCol", "thresholds",
            "checkpointInterval", "cacheNodeIds", "maxMemoryInMB")


def estimator_kind(est) -> Optional[Tuple[str, bool]]:
    """('rf' | 'dt', classification) for the engine's tree estimators, else None."""
    from ..classification import DecisionTreeClassifier, RandomForestClassifier
    from ..regression import DecisionTreeRegressor, RandomForestRegressor
    if type(est) is RandomForestRegressor:
        return "rf", False
    if type(est) is RandomForestClassifier:
        return "rf", True
    if type(est) is DecisionTreeRegressor:
        return "dt", False
    if type(est) is DecisionTreeClassifier:
        return "dt", True
    return None


def forest_arrays(forest: Forest) -> dict:
    """A finished forest's node fields as arrays (views of its NodeFields), for several truncate_forest calls on
    the same forest."""
    return {n: f.array() for n, f in forest.lists().items()}


def truncate_forest(forest: Forest, num_trees: int, max_depth: int, arrays: Optional[dict] = None) -> Forest:
    """The first ``num_trees`` trees cut at depth ``max_depth`` (depth-D nodes become leaves with the value
    they already store), renumbered compactly (per tree, by original id).

    One level-synchronous numpy sweep over the kept nodes instead of a Python walk per node: the fused tuner cuts
    every fold's 100-tree depth-10 forest for each of the grid's maps (L07's 3 x 3 grid: 27 cuts of up to 2e5
    nodes, ~3.5 s of per-node attribute traffic before)."""
    A = arrays if arrays is not None else forest_arrays(forest)
    feat, left, right = A["feat"], A["left"], A["right"]
    roots = np.asarray(forest.roots[:num_trees], dtype=np.int64)
    nodes, trees, inner = [], [], []
    fr, tr, level = roots, np.arange(len(roots), dtype=np.int64), 0
    while len(fr):
        inn = (feat[fr] >= 0) & (level < max_depth)
        nodes.append(fr)
        trees.append(tr)
        inner.append(inn)
        ii, ti = fr[inn], tr[inn]
        fr, tr = np.concatenate([left[ii], right[ii]]), np.concatenate([ti, ti])
        level += 1
    out = Forest(forest.K)
    if not nodes:
        return out
    g, tt, inn = np.concatenate(nodes), np.concatenate(trees), np.concatenate(inner)
    order = np.lexsort((g, tt))
    g, inn = g[order], inn[order]
    newid = np.full(len(feat), -1, dtype=np.int64)
    newid[g] = np.arange(len(g), dtype=np.int64)
    O = out.lists()
    lnew = np.where(inn, newid[np.where(inn, left[g], 0)], -1)
    rnew = np.where(inn, newid[np.where(inn, right[g], 0)], -1)
    O["feat"].extend(np.where(inn, feat[g], -1))
    O["thr"].extend(np.where(inn, A["thr"][g], 0.0))
    O["bin"].extend(np.where(inn, A["bin"][g], 0))
    O["left"].extend(lnew)
    O["right"].extend(rnew)
    O["catmask"].extend(np.where(inn[:, None], A["catmask"][g], 0))
    O["is_cat"].extend(A["is_cat"][g] & inn)
    O["value"].extend(A["value"][g])
    O["weight"].extend(A["weight"][g])
    O["gain"].extend(np.where(inn, A["gain"][g], 0.0))
    O["impurity"].extend(A["impurity"][g])
    O["depth"].extend(A["depth"][g])
    out.roots.extend(newid[roots].tolist())
    freeze_cut(out)
    return out


class FusedTreeTuner:
    """Fits all param maps of a tree estimator (or of a Pipeline ending in one) per data split (module doc)."""

    def __init__(self, est, maps: List[dict], dataset=None):
        from ..pipeline import Pipeline
        self.pipeline = est if isinstance(est, Pipeline) else None
        self.prefix = est.getStages()[:-1] if self.pipeline is not None else []
        self.tree = est.getStages()[-1] if self.pipeline is not None else est
        self.kind, self.cls = estimator_kind(self.tree)
        self.maps = list(maps) or [{}]
        self.ests = [self.tree.copy(pm) if pm else self.tree for pm in self.maps]
        self.dataset = dataset

    @staticmethod
    def supported(est, maps) -> bool:
        from ..pipeline import Pipeline
        if not FUSED_TUNING:
            return False
        if isinstance(est, Pipeline):
            stages = est.getStages()
            if not stages or estimator_kind(stages[-1]) is None:
                return False
            uid = stages[-1].uid
            # every map must touch the tree stage only: the prefix is then the same for all maps
            return all(getattr(p, "parent", None) == uid for pm in (maps or []) for p in pm)
        return estimator_kind(est) is not None

    # ------------------------------------------------------------------ planning
    def _key(self, e, d: int) -> tuple:
        from ..regression import resolve_subset
        vals = []
        for p, v in sorted(e.extractParamMap().items(), key=lambda kv: kv[0].name):
            if p.name in _VARYING or p.name in _IGNORED:
                continue
            vals.append((p.name, repr(v)))
        T = e.getNumTrees() if self.kind == "rf" else 1
        D = e.getMaxDepth()
        strategy = e.getFeatureSubsetStrategy() if self.kind == "rf" else "all"
        sub = resolve_subset(strategy, d, T, self.cls)
        # regression deeper than 8 takes the record path down to level 8 (engine.DEEP_REG): the depth-8 prefix of a
        # deep forest is then the depth-8 forest, as for classification
        from .engine import DEEP_REG
        return tuple(vals) + (("subset", sub), ("bagged", T > 1), ("deep", (not self.cls) and D > 8 and (T == 1 or not DEEP_REG)))

    def groups(self, d: int) -> List[List[int]]:
        groups: Dict[tuple, List[int]] = {}
        for j, e in enumerate(self.ests):
            groups.setdefault(self._key(e, d), []).append(j)
        return list(groups.values())

    # ------------------------------------------------------------------ training
    def prefix_fit(self, train):
        """The pipeline's prefix stages fitted on ``train`` (once per split) -> (PipelineModel | None, train
        transformed)."""
        if self.pipeline is None:
            return None, train
        from ..pipeline import Pipeline
        pm = Pipeline(stages=self.prefix).fit(train)
        return pm, pm.transform(train)

    def fit_forest(self, prep, e, T: int, D: int, mask: Optional[torch.Tensor] = None) -> Tuple[Forest, int]:
        """One forest of ``e``'s params with T trees of depth D on prepared (binned) training data -- what
        ``e.fit`` does after its own ``tree_fit_prepare``."""
        from ..classification import _num_classes
        from ..regression import _bag_weights, _combine_weights, resolve_subset
        session, data, y, w, seed, meta, train = prep
        if self.kind == "rf":
            strategy, bootstrap, rate = e.getFeatureSubsetStrategy(), e.getBootstrap(), e.getSubsamplingRate()
        else:
            strategy, bootstrap, rate = "all", False, 1.0
        subset = resolve_subset(strategy, data.d, T, self.cls)
        C = 0
        if self.cls:
            C = max(2, _num_classes(session, y, (train.schema[e.getLabelCol()].metadata or {}).get("ml_attr")))
        p = TreeParams(max_depth=D, max_bins=e.getMaxBins(), min_instances=float(e.getMinInstancesPerNode()),
                       min_info_gain=e.getMinInfoGain(), impurity=e.getImpurity(), num_classes=C,
                       feature_subset=subset, bootstrap=bootstrap, subsampling_rate=rate, seed=seed)
        weights = _bag_weights(data, T, bootstrap, rate, seed)
        if w is not None:
            weights = _combine_weights(weights, w, T)
        if mask is not None:
            m = mask.to(torch.uint8)[None, :]
            weights = m.expand(T, -1).contiguous() if weights is None else (weights * m).contiguous()
        stats = {"label": y.int()} if self.cls else {"v0": None, "v1": y.float()}
        return ForestTrainer(session, data, p).train(T, stats, weights), data.d

    def prep(self, e):
        """Binned data of the tuner's whole dataset (cached per (maxBins, seed, columns)): the shared input of the
        batched per-group fits (models/grouped.py)."""
        cache = self.__dict__.setdefault("_preps", {})
        key = self._prep_key(e)
        if key not in cache:
            cache[key] = self.prepare(e, self.dataset)
        return cache[key]

    def fit_forest_mask(self, e, T: int, D: int, mask: Optional[torch.Tensor]) -> Tuple[Forest, int]:
        """A forest on the whole dataset's bins with the rows outside ``mask`` weighted 0."""
        return self.fit_forest(self.prep(e), e, T, D, mask)

    def prepare(self, e, train):
        """Binned training data for (maxBins, seed, columns) -- ``tree_fit_prepare`` of the generic fit."""
        from ..regression import tree_fit_prepare
        return tree_fit_prepare(e, train, classification=self.cls) + (train,)

    @staticmethod
    def _prep_key(e) -> tuple:
        return (e.getMaxBins(), e.getOrDefault("seed"), e.getFeaturesCol(), e.getLabelCol(),
                e.getWeightCol() if e.hasParam("weightCol") else None)

    def model(self, e, forest: Forest, d: int):
        """The estimator's own model class around a (truncated) forest."""
        from ..classification import DecisionTreeClassificationModel, RandomForestClassificationModel
        from ..regression import DecisionTreeRegressionModel, RandomForestRegressionModel
        T = len(forest.roots)
        if self.kind == "rf":
            cls_ = RandomForestClassificationModel if self.cls else RandomForestRegressionModel
            m = cls_(forest, d, np.ones(T) if self.cls else np.full(T, 1.0 / T))
        else:
            cls_ = DecisionTreeClassificationModel if self.cls else DecisionTreeRegressionModel
            m = cls_(forest, d, [1.0])
        m._post_fit(e)
        return m

    def fit_split(self, train) -> Tuple[list, object]:
        """Every map fitted on the DataFrame ``train`` -> (models, prefix model or None).  Models are the tree
        models (wrapped in the map's PipelineModel for a Pipeline), each equal to ``est.fit(train, map)``."""
        from ..pipeline import PipelineModel
        pm, tt = self.prefix_fit(train)
        models: list = [None] * len(self.ests)
        preps: Dict[tuple, tuple] = {}   # binned data per (maxBins, seed, columns): shared by the groups
        d = 0
        for e in self.ests:
            key = self._prep_key(e)
            if key not in preps:
                preps[key] = self.prepare(e, tt)
            d = preps[key][1].d
        for grp in self.groups(d):
            es = [self.ests[j] for j in grp]
            e0 = es[0]
            key = self._prep_key(e0)
            Tm = max((e.getNumTrees() if self.kind == "rf" else 1) for e in es)
            Dm = max(e.getMaxDepth() for e in es)
            forest, dd = self.fit_forest(preps[key], e0, Tm, Dm)
            arrays = None
            for j, e in zip(grp, es):
                T = e.getNumTrees() if self.kind == "rf" else 1
                D = e.getMaxDepth()
                if T == Tm and D == Dm:
                    sub = forest
                else:
                    arrays = arrays if arrays is not None else forest_arrays(forest)
                    sub = truncate_forest(forest, T, D, arrays)
                tm = self.model(e, sub, dd)
                if pm is not None:
                    full = PipelineModel(list(pm.stages) + [tm])
                    full.uid = self.pipeline.uid
                    tm = full
                models[j] = tm
        return models, pm

    def evaluate(self, models, prefix_model, valid, evaluator) -> List[float]:
        """Metric of every model on ``valid`` (a Pipeline's prefix transforms ``valid`` once for all maps)."""
        if prefix_model is None:
            return [evaluator.evaluate(m.transform(valid)) for m in models]
        vt = prefix_model.transform(valid).cache()
        try:
            return [evaluator.evaluate(m.stages[-1].transform(vt)) for m in models]
        finally:
            vt.unpersist()
