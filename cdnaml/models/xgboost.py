"""Distributed XGBoost-style gradient boosting (ML 11 - XGBoost.py:27-103).

API of ``sparkdl.xgboost``: ``XgboostRegressor(n_estimators=100, learning_rate=0.1,
max_depth=4, random_state=42, missing=0)`` in a Pipeline after StringIndexer +
VectorAssembler, ``num_workers`` data-parallel workers, ``use_gpu``.

MI355X design: the binned matrix is built once and stays in HBM for all
rounds.  Each round computes per-row gradient/hessian on device (K9), builds
(Σh, Σg) histograms with the EXACT fixed-point integer LDS kernel (hist v4,
two int64 planes), all-reduces the level histogram over RCCL (one fused
collective per level; the reduction replaces XGBoost's Rabit allreduce),
scans XGBoost gain ``½[G_L²/(H_L+λ) + G_R²/(H_R+λ) − G²/(H+λ)] − γ`` with
``min_child_weight``, and learns a default direction for missing values
(sparsity-aware split finding: bin 0 holds NaN / ``missing``, both routings
are scored).  The training margin is updated in place by the binned predict
kernel, so no raw-feature traversal happens during training.

``num_workers`` maps to the SPMD world (one process per GPU); the engine
already shards rows across ranks, so it is validated but not needed.
"""
from __future__ import annotations

import math
from typing import Dict, Optional

import numpy as np
import torch

from ..ops import kernels as K
from ..utils import tracing as _tr
from ..sql import types as T
from ..sql.batch import ColumnData
from ..sql.dataframe import MapPlan
from .base import Estimator, Model
from .linalg import SparseVector
from .param import TypeConverters as TC, keyword_init
from .regression import _default_seed
from .tree.binning import make_binned
from .tree.engine import ForestTrainer, TreeParams
from .tree.forest import Forest
from .util import IllegalArgumentException, categorical_info, global_count, global_offset, local_batch, \
    streamed_columns, \
    require_vector

_XGB = {
    "featuresCol": ("features column name", "features", TC.toString),
    "labelCol": ("label column name", "label", TC.toString),
    "predictionCol": ("prediction column name", "prediction", TC.toString),
    "weightCol": ("instance weight column name", None, TC.toString),
    "baseMarginCol": ("column holding per-row base margins", None, TC.toString),
    "validationIndicatorCol": ("boolean column marking validation rows (early stopping)", None, TC.toString),
    "n_estimators": ("number of boosting rounds", 100, TC.toInt),
    "learning_rate": ("boosting learning rate (eta)", 0.3, TC.toFloat),
    "max_depth": ("maximum tree depth", 6, TC.toInt),
    "min_child_weight": ("minimum sum of instance hessian in a child", 1.0, TC.toFloat),
    "gamma": ("minimum loss reduction to make a split", 0.0, TC.toFloat),
    "reg_lambda": ("L2 regularisation on leaf weights", 1.0, TC.toFloat),
    "reg_alpha": ("L1 regularisation on leaf weights", 0.0, TC.toFloat),
    "subsample": ("row subsample ratio per round", 1.0, TC.toFloat),
    "colsample_bytree": ("feature subsample ratio per tree", 1.0, TC.toFloat),
    "colsample_bynode": ("feature subsample ratio per node", 1.0, TC.toFloat),
    "max_bin": ("histogram bins per feature (<= 256; one is reserved for missing values)", 256, TC.toInt),
    "base_score": ("initial prediction (global bias)", None, TC.toFloat),
    "missing": ("value treated as missing (NaN is always missing)", float("nan"), TC.toFloat),
    "random_state": ("random seed", 0, TC.toInt),
    "objective": ("learning objective", None, TC.toString),
    "num_workers": ("number of data-parallel workers (= GPUs of the SPMD job)", 1, TC.toInt),
    "use_gpu": ("train on the GPU (always true when one is present)", False, TC.toBoolean),
    "checkpoint_interval": ("save the booster every N rounds under SparkContext.setCheckpointDir and resume "
                            "an interrupted fit from it (-1: off)", -1, TC.toInt),
    "early_stopping_rounds": ("stop when the validation metric has not improved for this many rounds", None,
                              TC.toInt),
    "eval_metric": ("validation metric (rmse / logloss / mlogloss / error)", None, TC.toString),
    "tree_method": ("hist (the only method: device histograms)", "hist", TC.toString),
    "n_jobs": ("ignored (threads of the CPU library)", 1, TC.toInt),
    "verbosity": ("ignored", 1, TC.toInt),
}


def _sigmoid(x):
    return torch.sigmoid(x)


class _Booster:
    """Minimal Booster view: feature scores and raw margins."""

    def __init__(self, model: "_XgbModelBase"):
        self._m = model

    def get_score(self, importance_type: str = "weight") -> Dict[str, float]:
        f = self._m._forest
        score: Dict[int, float] = {}
        count: Dict[int, int] = {}
        for t in range(len(f.roots)):
            for i in f.tree_nodes(t):
                if f.feat[i] >= 0:
                    j = f.feat[i]
                    count[j] = count.get(j, 0) + 1
                    g = f.gain[i] if importance_type in ("gain", "total_gain") else (
                        f.weight[i] if importance_type in ("cover", "total_cover") else 1.0)
                    score[j] = score.get(j, 0.0) + g
        if importance_type in ("gain", "cover"):
            score = {j: score[j] / count[j] for j in score}
        return {f"f{j}": float(v) for j, v in sorted(score.items())}

    def trees_to_dataframe(self):
        import pandas as pd
        f = self._m._forest
        rows = []
        for t in range(len(f.roots)):
            for i in f.tree_nodes(t):
                rows.append({"Tree": t, "Node": i, "Feature": f"f{f.feat[i]}" if f.feat[i] >= 0 else "Leaf",
                             "Split": f.thr[i] if f.feat[i] >= 0 else float("nan"),
                             "Yes": f.left[i], "No": f.right[i], "Gain": f.gain[i] if f.feat[i] >= 0 else
                             float(f.value[i][0]), "Cover": f.weight[i]})
        return pd.DataFrame(rows)


class _XgbEstimatorBase(Estimator):
    _params = _XGB
    _classification = False

    def __init__(self, **kwargs):
        super().__init__()
        keyword_init(self, kwargs)

    # --------------------------------------------------------- shared fit
    def _prepare(self, dataset):
        fc, lc = self.getFeaturesCol(), self.getLabelCol()
        require_vector(dataset, fc)
        session = dataset._session
        W = session.comm.world_size
        nw = self.getNum_workers()
        if nw > 1 and nw != W and W > 1:
            raise IllegalArgumentException(
                f"num_workers={nw} but the SPMD job has {W} ranks: launch one process per worker "
                f"(torchrun --nproc-per-node {nw})")
        cols = [fc, lc]
        for c in (self.getWeightCol(), self.getBaseMarginCol(), self.getValidationIndicatorCol()):
            if c:
                cols.append(c)
        src = streamed_columns(dataset, fc, cols[1:])
        if src is not None:  # out-of-core: features streamed into the bins, never resident
            X, b_cols, _ = src
        else:
            b = local_batch(dataset, cols)
            X = b.columns[fc].values.float().contiguous()
            b_cols = b.columns
        y = b_cols[lc].values.double()
        w = b_cols[self.getWeightCol()].values.double() if self.getWeightCol() else None
        bm = b_cols[self.getBaseMarginCol()].values.double() if self.getBaseMarginCol() else None
        val = b_cols[self.getValidationIndicatorCol()].values.bool() if self.getValidationIndicatorCol() \
            else None
        n = X.shape[0]
        mb = self.getMax_bin()
        if not 3 <= mb <= 256:
            raise IllegalArgumentException("max_bin must be in [3, 256]")
        seed = self.getRandom_state()
        if seed is None:
            seed = _default_seed(type(self))
        data = make_binned(session, X, {}, mb, seed, global_offset(session, n), global_count(session, n),
                           missing=float(self.getMissing()))
        return session, data, X, y, w, bm, val, seed

    def _params_tree(self, d: int, seed: int) -> TreeParams:
        cb_tree, cb_node = self.getColsample_bytree(), self.getColsample_bynode()
        frac = cb_tree * cb_node
        subset = None if frac >= 1.0 else max(1, int(math.floor(frac * d + 1e-9)))
        return TreeParams(max_depth=self.getMax_depth(), max_bins=self.getMax_bin(), min_instances=0.0,
                          min_info_gain=0.0, impurity="xgb", feature_subset=subset, seed=seed,
                          reg_lambda=self.getReg_lambda(), gamma=self.getGamma(),
                          min_child_weight=self.getMin_child_weight(),
                          subset_scope="node" if cb_node < 1.0 else "tree")

    def _boost(self, session, data, grad_hess, F, seed, n_out, val_mask, y, metric_fn, unit_hess=False):
        """Rounds of K trees (one per output); F [n, n_out] float32 margins (in place)."""
        dev = data.bins.device
        n = data.n_local
        p = self._params_tree(data.d, seed)
        trainer = ForestTrainer(session, data, p)
        forest = Forest(1)
        eta = self.getLearning_rate()
        esr = self.getEarly_stopping_rounds()
        best, best_round, history = float("inf"), -1, []
        train_w = None if val_mask is None else (~val_mask).to(torch.uint8)
        from .tree.checkpoint import RoundCheckpointer
        ck = RoundCheckpointer(session, self, data, self.getCheckpoint_interval(), labels=y)
        start = 0
        resumed = ck.load()
        if resumed is not None:
            start, forest, Fm, extra = resumed
            F.copy_(Fm.to(F.device).view_as(F))
            best, best_round, history = extra["best"], extra["best_round"], list(extra["history"])
        for m in range(start, self.getN_estimators()):
            with _tr.span("xgb.grad_hess", round=m):
                g, h = grad_hess(F)  # [n, n_out] each
            bag = None
            rate = self.getSubsample()
            if rate < 1.0:
                u = K.uniform(n, seed + 7919 * m, data.row_offset, 0x300, device=dev)
                bag = (u < rate).to(torch.uint8)
            if train_w is not None:
                bag = train_w if bag is None else bag * train_w
            for k in range(n_out):
                trainer.p.seed = (seed * 1000003 + m * 131 + k) & 0x7FFFFFFF
                # unit hessians (squared error, unweighted): H = row count, so the histogram
                # takes the single-statistic (packed count|sum) path
                v0 = None if unit_hess else h[:, k].float().contiguous()
                # the margins of the rows updated by the level partitions as each row reaches its leaf (no walk of
                # the finished tree) when the trainer's level loop allows it (every row in the tree, reg_alpha 0:
                # the leaf values are the trainer's own)
                fk = F[:, k]
                margin = (fk, eta) if (bag is None and fk.is_contiguous() and self.getReg_alpha() <= 0) else None
                v1 = g[:, k].float().contiguous()
                if n_out == 1 and getattr(g, "_cdna_absmax", None) is not None:
                    v1._cdna_absmax = g._cdna_absmax  # max |g| from the grad / hess pass (K.grad_hess)
                trainer.train(1, {"v0": v0, "v1": v1},
                              None if bag is None else bag[None, :].contiguous(), forest, margin=margin)
                t = len(forest.roots) - 1
                with _tr.span("xgb.update_margin", round=m):
                    self._apply_l1(forest, t)
                    if not (margin is not None and trainer.margin_applied):
                        nodes, vals, masks = forest.binned_arrays(dev, t)
                        col = fk if fk.is_contiguous() else fk.contiguous()
                        K.predict_binned_add(data.bins, nodes, 0, vals, masks, eta, col)
                        if col.data_ptr() != fk.data_ptr():
                            F[:, k] = col
            if val_mask is not None and metric_fn is not None:
                v = metric_fn(F, val_mask)
                history.append(v)
                if v < best - 1e-12:
                    best, best_round = v, m
                elif esr and m - best_round >= esr:
                    keep = (best_round + 1) * n_out
                    forest = _truncate(forest, keep)
                    break
            ck.maybe_save(m + 1, forest, F, {"best": best, "best_round": best_round, "history": history})
        ck.finish()
        data.release_fit_copies()
        return forest, history

    def _apply_l1(self, forest: Forest, t: int):
        """reg_alpha: soft-threshold leaf weights w = -sign(G) max(|G| - alpha, 0) / (H + lambda)."""
        a = self.getReg_alpha()
        if a <= 0:
            return
        lam = self.getReg_lambda()
        for i in forest.tree_nodes(t):
            if forest.feat[i] < 0:
                w = float(forest.value[i][0])
                H = forest.weight[i]
                G = -w * (H + lam)
                Gs = math.copysign(max(abs(G) - a, 0.0), G)
                forest.value[i] = np.array([-Gs / (H + lam)])
        forest._dev = {}


def _truncate(forest: Forest, keep: int) -> Forest:
    if keep >= len(forest.roots):
        return forest
    forest.roots = forest.roots[:keep]
    forest._dev = {}
    return forest


# ================================================================ regressor
class XgboostRegressor(_XgbEstimatorBase):
    """reg:squarederror (default) / reg:absoluteerror / reg:pseudohubererror / count:poisson."""

    def _fit(self, dataset):
        session, data, X, y, w, bm, val, seed = self._prepare(dataset)
        n = data.n_local
        dev = data.bins.device
        obj = self.getObjective() or "reg:squarederror"
        yf = y.float()
        wf = None if w is None else w.float()
        base = self.getBase_score()
        if base is None:
            base = 0.5  # XGBoost 1.x default
        base_margin = math.log(base) if obj == "count:poisson" and base > 0 else base
        F = torch.full((n, 1), float(base_margin), dtype=torch.float32, device=dev)
        if bm is not None:
            F[:, 0] += bm.float()

        def grad_hess(F):
            if F.is_cuda and obj in K.GRAD_HESS_OBJ:
                return K.grad_hess(F, yf, wf, K.GRAD_HESS_OBJ[obj])  # K9 HIP kernel
            f = F[:, 0]
            if obj in ("reg:squarederror", "reg:linear"):
                g, h = f - yf, torch.ones_like(f)
            elif obj == "reg:absoluteerror":
                g, h = torch.sign(f - yf), torch.ones_like(f)
            elif obj == "reg:pseudohubererror":
                r = f - yf
                s = torch.sqrt(1 + r * r)
                g, h = r / s, 1 / (s * s * s)
            elif obj == "count:poisson":
                e = torch.exp(f.double())
                g, h = (e - yf.double()).float(), (e * math.exp(0.7)).float()
            else:
                raise IllegalArgumentException(f"unsupported objective {obj}")
            if wf is not None:
                g, h = g * wf, h * wf
            return g[:, None], h[:, None]

        def metric(F, vm):
            e = (F[:, 0] - yf)[vm]
            s = torch.tensor([float((e * e).sum()), float(vm.sum())], dtype=torch.float64, device=dev)
            session.comm.all_reduce(s)
            return math.sqrt(float(s[0]) / max(float(s[1]), 1.0))

        unit = obj in ("reg:squarederror", "reg:linear", "reg:absoluteerror") and wf is None
        forest, hist = self._boost(session, data, grad_hess, F, seed, 1, val, y, metric, unit_hess=unit)
        model = XgboostRegressorModel(forest, data.d, base_margin, data.thresholds, data.nthr, obj)
        model._copyValues_from(self)
        model.evals_result_ = {"validation": hist}
        return model


class _XgbModelBase(Model):
    _params = _XGB

    def __init__(self, forest: Optional[Forest] = None, numFeatures: int = 0, base_margin: float = 0.0,
                 thresholds=None, nthr=None, objective: str = "", n_out: int = 1):
        super().__init__()
        self._forest = forest
        self._numFeatures = numFeatures
        self._base = float(base_margin)
        self._thr = np.asarray(thresholds if thresholds is not None else np.zeros((0, 1)))
        self._nthr = np.asarray(nthr if nthr is not None else [], dtype=np.int32)
        self._objective = objective
        self._n_out = n_out
        self._dev = {}

    def _copyValues_from(self, est):
        est._copyValues(self)
        self.parent = est

    def get_booster(self):
        return _Booster(self)

    @property
    def featureImportances(self):
        imp = self._forest.feature_importances(self._numFeatures)
        nz = np.nonzero(imp)[0]
        return SparseVector(self._numFeatures, nz.tolist(), imp[nz].tolist())

    def _margins(self, X: torch.Tensor) -> torch.Tensor:
        """Binned prediction: missing values follow each node's learned default direction."""
        n = X.shape[0]
        dev = X.device
        key = str(dev)
        if key not in self._dev:
            thr = torch.from_numpy(self._thr.astype(np.float32)).to(dev)
            self._dev[key] = (thr, torch.from_numpy(self._nthr).to(dev))
        thr, nthr = self._dev[key]
        Xf = X.float()
        bins = K.binize(Xf, thr, nthr, missing=float(self.getMissing()))  # missing -> bin 0 inside the kernel
        eta = self.getLearning_rate()
        F = torch.full((n, self._n_out), self._base, dtype=torch.float32, device=dev)
        if dev.type == "cpu":
            K.predict_binned_forest_host(bins, [self._forest.binned_arrays(dev, t)
                                                for t in range(len(self._forest.roots))], eta, F)
            return F
        for t in range(len(self._forest.roots)):
            nodes, vals, masks = self._forest.binned_arrays(dev, t)
            k = t % self._n_out
            col = F[:, k] if F[:, k].is_contiguous() else F[:, k].contiguous()
            K.predict_binned_add(bins, nodes, 0, vals, masks, eta, col)
            if col.data_ptr() != F[:, k].data_ptr():
                F[:, k] = col
        return F

    def _save_state(self):
        return {"numFeatures": self._numFeatures, "base": self._base, "objective": self._objective,
                "n_out": self._n_out}, dict(self._forest.state(), thr=torch.from_numpy(self._thr.copy()),
                                            nthr=torch.from_numpy(self._nthr.copy()))

    def _load_state(self, extra, tensors, stages):
        self._forest = Forest.from_state(tensors)
        self._numFeatures = int(extra["numFeatures"])
        self._base = float(extra["base"])
        self._objective = extra["objective"]
        self._n_out = int(extra.get("n_out", 1))
        self._thr = tensors["thr"].numpy()
        self._nthr = tensors["nthr"].numpy().astype(np.int32)
        self._dev = {}


class XgboostRegressorModel(_XgbModelBase):
    def _transform(self, dataset):
        fc, pc = self.getFeaturesCol(), self.getPredictionCol()
        require_vector(dataset, fc)

        def fn(b, ctx):
            X = b.columns[fc].values
            if X.shape[0] == 0:
                p = torch.zeros(0, dtype=torch.float64, device=X.device)
            else:
                p = self._margins(X)[:, 0].double()
                if self._objective == "count:poisson":
                    p = torch.exp(p)
            return b.with_column(pc, ColumnData(p, T.DoubleType()))
        return dataset._new(MapPlan(dataset._plan, f"XgboostRegressorModel -> {pc}", fn))


# =============================================================== classifier
class XgboostClassifier(_XgbEstimatorBase):
    """binary:logistic (2 classes) / multi:softprob (softmax over K one-tree-per-class rounds)."""
    _params = dict(_XGB, **{
        "rawPredictionCol": ("raw prediction (margin) column name", "rawPrediction", TC.toString),
        "probabilityCol": ("class probability column name", "probability", TC.toString),
    })

    def _fit(self, dataset):
        session, data, X, y, w, bm, val, seed = self._prepare(dataset)
        n = data.n_local
        dev = data.bins.device
        mx = torch.tensor([float(y.max()) if n else 0.0], dtype=torch.float64, device=session.comm.device)
        session.comm.all_reduce(mx, "max")
        C = max(2, int(mx) + 1)
        obj = self.getObjective() or ("binary:logistic" if C == 2 else "multi:softprob")
        yi = y.long()
        wf = None if w is None else w.float()
        if obj.startswith("binary"):
            base = self.getBase_score()
            base = 0.5 if base is None else base
            base_margin = math.log(base / (1 - base))
            n_out = 1
        else:
            base_margin = 0.0
            n_out = C
        F = torch.full((n, n_out), float(base_margin), dtype=torch.float32, device=dev)
        if bm is not None:
            F += bm.float()[:, None]

        def grad_hess(F):
            if F.is_cuda:
                return K.grad_hess(F, yi.float(), wf, 4 if n_out == 1 else 5)  # K9 HIP kernel
            # host path in fp64, rounded once to fp32: vectorised and scalar-tail transcendentals then agree,
            # so a row's gradient does not depend on where the shard boundary puts it (any world size)
            if n_out == 1:
                pr = _sigmoid(F[:, 0].double())
                g = (pr - yi.double()).float()
                h = (pr * (1 - pr)).clamp_min(1e-16).float()
                g, h = g[:, None], h[:, None]
            else:
                pr = torch.softmax(F.double(), dim=1)
                oh = torch.nn.functional.one_hot(yi.clamp(0, C - 1), C).double()
                g = (pr - oh).float()
                h = (2.0 * pr * (1 - pr)).clamp_min(1e-16).float()
            if wf is not None:
                g, h = g * wf[:, None], h * wf[:, None]
            return g, h

        def metric(F, vm):
            if n_out == 1:
                pr = _sigmoid(F[:, 0])[vm].double().clamp(1e-15, 1 - 1e-15)
                yy = yi[vm].double()
                ll = -(yy * torch.log(pr) + (1 - yy) * torch.log(1 - pr)).sum()
            else:
                lp = torch.log_softmax(F.double(), 1)[vm]
                ll = -lp.gather(1, yi[vm][:, None]).sum()
            s = torch.tensor([float(ll), float(vm.sum())], dtype=torch.float64, device=dev)
            session.comm.all_reduce(s)
            return float(s[0]) / max(float(s[1]), 1.0)

        forest, hist = self._boost(session, data, grad_hess, F, seed, n_out, val, y, metric)
        model = XgboostClassifierModel(forest, data.d, base_margin, data.thresholds, data.nthr, obj, n_out)
        model._copyValues_from(self)
        model._num_classes = C
        model.evals_result_ = {"validation": hist}
        return model


class XgboostClassifierModel(_XgbModelBase):
    _params = XgboostClassifier._params
    _num_classes = 2

    @property
    def numClasses(self):
        return self._num_classes

    def _transform(self, dataset):
        fc = self.getFeaturesCol()
        require_vector(dataset, fc)
        rc, prc, pc = self.getRawPredictionCol(), self.getProbabilityCol(), self.getPredictionCol()

        def fn(b, ctx):
            X = b.columns[fc].values
            if X.shape[0] == 0:
                F = torch.zeros((0, self._n_out), dtype=torch.float32, device=X.device)
            else:
                F = self._margins(X)
            if self._n_out == 1:
                p1 = _sigmoid(F[:, 0])
                prob = torch.stack([1 - p1, p1], 1)
                raw = torch.stack([-F[:, 0], F[:, 0]], 1)
            else:
                prob = torch.softmax(F, 1)
                raw = F
            pred = torch.argmax(prob, 1).double()
            nb = b
            if rc:
                nb = nb.with_column(rc, ColumnData(raw.float(), T.VectorUDT()))
            if prc:
                nb = nb.with_column(prc, ColumnData(prob.float(), T.VectorUDT()))
            return nb.with_column(pc, ColumnData(pred, T.DoubleType()))
        return dataset._new(MapPlan(dataset._plan, "XgboostClassifierModel", fn))

    def _save_state(self):
        extra, tensors = super()._save_state()
        extra["num_classes"] = self._num_classes
        return extra, tensors

    def _load_state(self, extra, tensors, stages):
        super()._load_state(extra, tensors, stages)
        self._num_classes = int(extra.get("num_classes", 2))
