"""Many models: one model per group, trained in batched passes (SURVEY §2.4 B6, §2.9 P7;
ML 13 - Training with Pandas Function API.py:73-130,161).

The course trains one scikit-learn forest per IoT device inside ``groupBy("device_id").applyInPandas``.
That stays supported: it is a generic pandas UDF, and groups now run concurrently (``sql/udf.py``).  When
the per-group model is one of this engine's tree estimators, ``GroupedEstimator`` trains every group in a
few forest passes over ONE binned copy of the data:

* group g's tree t is tree g*T + t of a batched forest;
* its weights are the bootstrap draws of tree t, times the indicator of group g;
* its feature subsets hash as logical tree t (``TreeParams.tree_ids``).

Group g's model is then bit-identical to fitting that estimator on group g's rows alone with the same
shared bins (``tests/test_grouped.py``).  Ten 10-tree groups are one 100-tree pass, not ten fits.
Groups are batched so that (trees per pass x rows) stays under ``cdnaml.grouped.maxTreeRows``, because the
mask formulation scans every row for every tree of a pass.

``GroupedModel.transform`` scores each row with its own group's model (rows of unseen groups get null).
"""
from __future__ import annotations

from typing import Dict, List

import numpy as np
import torch

from ..sql.batch import ColumnData
from .base import Estimator, Model
from .param import TypeConverters as TC, keyword_init


class GroupedEstimator(Estimator):
    _params = {
        "estimator": ("per-group estimator (one of this engine's DecisionTree / RandomForest estimators)", None,
                      None),
        "groupCol": ("column whose values define the groups", "group", TC.toString),
        "maxTreeRows": ("batched-pass budget: trees per pass x rows", 4_000_000_000, TC.toInt),
    }

    def __init__(self, estimator=None, groupCol=None, maxTreeRows=None):
        super().__init__()
        keyword_init(self, dict(estimator=estimator, groupCol=groupCol, maxTreeRows=maxTreeRows))

    def _fit(self, dataset):
        from .tree.fused import FusedTreeTuner, estimator_kind
        est = self.getEstimator()
        if estimator_kind(est) is None:
            raise TypeError("GroupedEstimator batches this engine's DecisionTree / RandomForest estimators; "
                            "use groupBy().applyInPandas for other per-group models")
        gcol = self.getGroupCol()
        keys = _key_values(dataset, gcol)
        uniq, inv = np.unique(keys, return_inverse=True)
        # agree on the global set of groups (every rank trains every group's trees)
        comm = dataset._session.comm
        if comm.distributed:
            allk = comm.all_gather_object(uniq.tolist())
            uniq = np.unique(np.concatenate([np.asarray(a, dtype=uniq.dtype) for a in allk]))
            inv = np.searchsorted(uniq, keys)
        tuner = FusedTreeTuner(est, [{}], dataset)
        e = tuner.ests[0]
        data = tuner.prep(e)[1]
        dev = data.bins.device
        gid = torch.from_numpy(inv.astype(np.int32)).to(dev)
        T_ = e.getNumTrees() if tuner.kind == "rf" else 1
        per_pass = max(1, int(self.getMaxTreeRows() // max(1, T_ * max(data.n_global, 1))))
        models = {}
        for g0 in range(0, len(uniq), per_pass):
            gs = list(range(g0, min(len(uniq), g0 + per_pass)))
            forest, d = _fit_groups(tuner, e, T_, gid, gs)
            for j, g in enumerate(gs):
                sub = _slice_forest(forest, j * T_, (j + 1) * T_)
                models[_py(uniq[g])] = tuner.model(e, sub, d)
        gm = GroupedModel(models, gcol)
        gm._post_fit(self)
        return gm


def _py(v):
    return v.item() if hasattr(v, "item") else v


def _key_values(df, col) -> np.ndarray:
    from .util import local_batch
    b = local_batch(df, [col])
    return b.columns[col].to_numpy()


def _fit_groups(tuner, e, T_: int, gid: torch.Tensor, groups: List[int]):
    """One forest pass: tree g*T + t = tree t of group g (weights: bootstrap t x [row in g])."""
    from .classification import _num_classes
    from .regression import _bag_weights, _combine_weights, resolve_subset
    from .tree.engine import ForestTrainer, TreeParams
    session, data, y, w, seed, meta = tuner.prep(e)[:6]
    if tuner.kind == "rf":
        strategy, bootstrap, rate = e.getFeatureSubsetStrategy(), e.getBootstrap(), e.getSubsamplingRate()
    else:
        strategy, bootstrap, rate = "all", False, 1.0
    subset = resolve_subset(strategy, data.d, T_, tuner.cls)
    C = 0
    if tuner.cls:
        C = max(2, _num_classes(session, y, (tuner.dataset.schema[e.getLabelCol()].metadata or {}).get("ml_attr")))
    G = len(groups)
    p = TreeParams(max_depth=e.getMaxDepth(), max_bins=e.getMaxBins(), min_instances=float(e.getMinInstancesPerNode()),
                   min_info_gain=e.getMinInfoGain(), impurity=e.getImpurity(), num_classes=C, feature_subset=subset,
                   bootstrap=bootstrap, subsampling_rate=rate, seed=seed,
                   tree_ids=np.tile(np.arange(T_), G))
    base = _bag_weights(data, T_, bootstrap, rate, seed)
    if w is not None:
        base = _combine_weights(base, w, T_)
    n = data.n_local
    dev = data.bins.device
    masks = torch.stack([(gid == g) for g in groups]).to(torch.uint8) if n else \
        torch.zeros((G, 0), dtype=torch.uint8, device=dev)
    if base is None:
        weights = masks.repeat_interleave(T_, 0).contiguous()
    else:
        weights = (masks[:, None, :] * base[None, :, :]).reshape(G * T_, n).contiguous()
    stats = {"label": y.int()} if tuner.cls else {"v0": None, "v1": y.float()}
    return ForestTrainer(session, data, p).train(G * T_, stats, weights), data.d


def _slice_forest(forest, t0: int, t1: int):
    from .tree.fused import truncate_forest
    from .tree.forest import Forest
    sub = Forest(forest.K)
    sub.roots = forest.roots[t0:t1]
    for name in ("feat", "thr", "bin", "left", "right", "catmask", "is_cat", "value", "weight", "gain",
                 "impurity", "depth"):
        setattr(sub, name, getattr(forest, name))
    return truncate_forest(sub, t1 - t0, 1 << 30)  # compact copy of just these trees


class GroupedModel(Model):
    _params = {"groupCol": ("column whose values define the groups", "group", TC.toString)}

    def __init__(self, models: Dict = None, groupCol: str = "group"):
        super().__init__()
        self.models = dict(models or {})
        self._set(groupCol=groupCol)

    def _transform(self, dataset):
        from ..sql.dataframe import MapPlan
        gcol = self.getGroupCol()
        models = self.models
        any_m = next(iter(models.values()))
        out_df = any_m.transform(dataset.limit(0))
        new_cols = [f for f in out_df.schema.fields if f.name not in dataset.columns]

        def fn(b, ctx):
            from ..sql.dataframe import DataFrame, SourcePlan
            keys = b.columns[gcol].to_numpy()
            outs = {f.name: None for f in new_cols}
            for k in np.unique(keys):
                m = models.get(_py(k))
                if m is None:
                    continue
                idx = torch.from_numpy(np.nonzero(keys == k)[0]).to(b.device)
                part = b.take(idx)
                sess = ctx.session
                res = m.transform(DataFrame(SourcePlan(sess, "group-part", lambda p=part: [p], part.schema()),
                                            sess))._plan.execute()[0]
                for f in new_cols:
                    c = res.columns[f.name]
                    if outs[f.name] is None:
                        vals = torch.zeros((b.n,) + tuple(c.values.shape[1:]), dtype=c.values.dtype, device=b.device)
                        outs[f.name] = [vals, torch.zeros(b.n, dtype=torch.bool, device=b.device), c.dtype]
                    outs[f.name][0][idx] = c.values
                    outs[f.name][1][idx] = True
            nb = b
            for f in new_cols:
                o = outs[f.name]
                if o is None:
                    o = [torch.zeros(b.n, dtype=torch.float64, device=b.device),
                         torch.zeros(b.n, dtype=torch.bool, device=b.device), f.dataType]
                nb = nb.with_column(f.name, ColumnData(o[0], o[2], o[1]))
            return nb
        return dataset._new(MapPlan(dataset._plan, f"GroupedModel({gcol})", fn))

    def _sub_stages(self):
        return list(self.models.values())

    def _save_state(self):
        return {"keys": [_py(k) for k in self.models]}, {}

    def _load_state(self, extra, tensors, stages):
        self.models = dict(zip(extra["keys"], stages))

