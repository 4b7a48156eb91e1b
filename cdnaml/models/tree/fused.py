"""Fused tree-ensemble tuning: CrossValidator / TrainValidationSplit over ONE binned dataset
(ML 07 - Random Forests and Hyperparameter Tuning.py:72-158,
Labs/ML 07L - Hyperparameter Tuning Lab.py:105-141).

The generic tuner fits every (fold, param map) pair from scratch: the course's 2 x 2 grid with 3 folds is
12 fits + 1 refit, each re-sampling quantiles, re-binning 1e8 x 100 features and re-drawing bootstraps.
For the engine's tree ensembles three facts make most of that work shared:

* The binned matrix depends on the features, ``maxBins`` and ``seed`` only.  It is built once per
  (maxBins, seed), from the global quantile sample of the whole dataset, and kept in HBM for every fold,
  map and the refit.  The generic path bins each training fold's own sample instead; this is a deliberate
  divergence from Spark: the split candidates see the validation rows' features, never their labels.
* A fold is a weight mask.  Rows whose Philox fold id (the same draw as the generic path's ``__fold``
  column) equals f get weight 0, multiplied into the Poisson bootstrap weights.  No fold is copied out.
* Tree t of a forest sees bootstrap stream (seed, t) and feature subsets hashed from (seed, t, node), and
  its level-d histograms are exact integers.  So among maps that differ only in ``numTrees`` and
  ``maxDepth``, every model is a prefix of the largest one: the first ``numTrees`` trees, cut at
  ``maxDepth`` (a node at depth D keeps its stored leaf value).  One forest per fold, with the largest
  numTrees and maxDepth of the group, gives the whole grid, bit-identically to fitting each map
  (``tests/test_tuning_fused.py``).  The 2 x 2 x 3 grid becomes 3 fits of 10 trees at depth 5.

Maps are grouped by everything else (including the resolved feature-subset size, and numTrees == 1, which
switches off bagging).  Regression groups also split at maxDepth 8, because deeper trees take a different
histogram path.  Estimators other than the engine's DecisionTree / RandomForest use the generic path.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from ...ops import kernels as K
from .engine import Forest, ForestTrainer, TreeParams

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


def truncate_forest(forest: Forest, num_trees: int, max_depth: int) -> Forest:
    """The first ``num_trees`` trees cut at depth ``max_depth`` (depth-D nodes become leaves with the value
    they already store), renumbered compactly."""
    out = Forest(forest.K)
    for t in range(num_trees):
        r = forest.roots[t]
        base = forest.depth[r]
        keep = [i for i in forest.tree_nodes(t) if forest.depth[i] - base <= max_depth]
        pos = {g: j + len(out.feat) for j, g in enumerate(keep)}
        for g in keep:
            j = out.add(forest.value[g], forest.weight[g], forest.depth[g], forest.impurity[g])
            inner = forest.feat[g] >= 0 and forest.depth[g] - base < max_depth
            if inner:
                out.feat[j], out.thr[j], out.bin[j] = forest.feat[g], forest.thr[g], forest.bin[g]
                out.is_cat[j], out.catmask[j], out.gain[j] = forest.is_cat[g], forest.catmask[g], forest.gain[g]
        for g in keep:
            j = pos[g]
            if out.feat[j] >= 0:
                out.left[j], out.right[j] = pos[forest.left[g]], pos[forest.right[g]]
        out.roots.append(pos[r])
    return out


class FusedTreeTuner:
    """Fits all param maps of a tree estimator fold by fold on shared binned data (see module doc)."""

    def __init__(self, est, maps: List[dict], dataset):
        self.est = est
        self.kind, self.cls = estimator_kind(est)
        self.dataset = dataset
        self.ests = [est.copy(pm) if pm else est for pm in maps]
        self._preps: Dict[tuple, tuple] = {}
        self.groups = self._group()

    # ------------------------------------------------------------------ planning
    def _key(self, e) -> tuple:
        from ..regression import resolve_subset
        vals = []
        for p, v in sorted(e.extractParamMap().items(), key=lambda kv: kv[0].name):
            if p.name in _VARYING or p.name in _IGNORED:
                continue
            vals.append((p.name, repr(v)))
        T = e.getNumTrees() if self.kind == "rf" else 1
        D = e.getMaxDepth()
        strategy = e.getFeatureSubsetStrategy() if self.kind == "rf" else "all"
        d = self.prep(e)[1].d
        sub = resolve_subset(strategy, d, T, self.cls)
        return tuple(vals) + (("subset", sub), ("bagged", T > 1), ("deep", (not self.cls) and D > 8))

    def _group(self) -> List[List[int]]:
        groups: Dict[tuple, List[int]] = {}
        for j, e in enumerate(self.ests):
            groups.setdefault(self._key(e), []).append(j)
        return list(groups.values())

    @staticmethod
    def supported(est, maps) -> bool:
        return FUSED_TUNING and estimator_kind(est) is not None

    # ------------------------------------------------------------------ training
    def prep(self, e):
        """Binned data of the whole dataset for (maxBins, seed, columns): built once, shared by folds + refit."""
        from ..regression import _default_seed, tree_fit_prepare
        seed = e.getOrDefault("seed")
        seed = _default_seed(type(e)) if seed is None else seed
        key = (e.getMaxBins(), seed, e.getFeaturesCol(), e.getLabelCol(), e.getWeightCol())
        if key not in self._preps:
            self._preps[key] = tree_fit_prepare(e, self.dataset, classification=self.cls)
        return self._preps[key]

    def row_uniform(self, seed: int) -> torch.Tensor:
        """Per local row: the Philox uniform(seed, global row, stream 11) of ``DataFrame._with_global_uniform``
        (the generic tuner's fold draw and ``randomSplit``'s draw)."""
        data = self.prep(self.ests[0])[1]
        return K.uniform(data.n_local, seed, data.row_offset, 11, device=data.bins.device)

    def fold_ids(self, seed: int, k: int) -> torch.Tensor:
        return torch.floor(self.row_uniform(seed) * k).to(torch.int32)

    def fit_forest(self, e, T: int, D: int, mask: Optional[torch.Tensor]) -> Tuple[Forest, int]:
        from ..classification import _num_classes
        from ..regression import _bag_weights, _combine_weights, resolve_subset
        session, data, y, w, seed, meta = self.prep(e)
        if self.kind == "rf":
            strategy, bootstrap, rate = e.getFeatureSubsetStrategy(), e.getBootstrap(), e.getSubsamplingRate()
        else:
            strategy, bootstrap, rate = "all", False, 1.0
        subset = resolve_subset(strategy, data.d, T, self.cls)
        C = 0
        if self.cls:
            C = max(2, _num_classes(session, y, (self.dataset.schema[e.getLabelCol()].metadata or {}).get("ml_attr")))
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

    def fit_split(self, mask: Optional[torch.Tensor]) -> List:
        """Models of every map trained on the rows where ``mask`` is 1 (all rows when None)."""
        models = [None] * len(self.ests)
        for grp in self.groups:
            es = [self.ests[j] for j in grp]
            Tm = max((e.getNumTrees() if self.kind == "rf" else 1) for e in es)
            Dm = max(e.getMaxDepth() for e in es)
            forest, d = self.fit_forest(es[0], Tm, Dm, mask)
            for j, e in zip(grp, es):
                T = e.getNumTrees() if self.kind == "rf" else 1
                D = e.getMaxDepth()
                sub = forest if (T == Tm and D == Dm) else truncate_forest(forest, T, D)
                models[j] = self.model(e, sub, d)
        return models

    def refit(self, j: int):
        """Map j on the full dataset (the binned data is shared; identical to ``est.fit(dataset, map_j)``)."""
        e = self.ests[j]
        forest, d = self.fit_forest(e, e.getNumTrees() if self.kind == "rf" else 1, e.getMaxDepth(), None)
        return self.model(e, forest, d)
