"""Evaluators (SURVEY §2.5.4 V1–V3): fused device reductions + one all-reduce.

RegressionEvaluator uses the K13 ``reg_metrics`` kernel (8 sufficient sums
in f64); the binary evaluator builds the ROC/PR curves from a global sort
(one GPU) or a 2^20-bucket score histogram all-reduced over RCCL
(multi-GPU); the multiclass evaluator all-reduces a confusion matrix.
Reference usage: ML 02:146-151, ML 03:150-157 (``setMetricName`` chaining),
Labs/ML 07L:125,197, MLE 03:65-68,125-132.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ..ops import kernels as K
from .base import Evaluator
from .param import NO_DEFAULT, TypeConverters as TC, keyword_init
from .util import IllegalArgumentException, local_batch


class RegressionEvaluator(Evaluator):
    _params = {
        "predictionCol": ("prediction column name", "prediction", TC.toString),
        "labelCol": ("label column name", "label", TC.toString),
        "metricName": ("metric name in evaluation - one of: rmse (default), mse, r2, mae, var", "rmse", TC.toString),
        "weightCol": ("weight column name", None, TC.toString),
        "throughOrigin": ("whether the regression is through the origin", False, TC.toBoolean),
    }

    def __init__(self, predictionCol=None, labelCol=None, metricName=None, weightCol=None, throughOrigin=None):
        super().__init__()
        keyword_init(self, dict(predictionCol=predictionCol, labelCol=labelCol, metricName=metricName,
                                weightCol=weightCol, throughOrigin=throughOrigin))

    def _evaluate(self, dataset):
        pc, lc, wc = self.getPredictionCol(), self.getLabelCol(), self.getWeightCol()
        cols = [lc, pc] + ([wc] if wc else [])
        b = local_batch(dataset, cols)
        y = b.columns[lc].values.double()
        p = b.columns[pc].values.double()
        w = b.columns[wc].values.double() if wc else None
        ok = ~(torch.isnan(y) | torch.isnan(p))
        for c in (b.columns[lc], b.columns[pc]):
            if c.valid is not None:
                ok &= c.valid
        if not bool(ok.all()):
            y, p = y[ok], p[ok]
            w = None if w is None else w[ok]
        acc = K.reg_metrics(y, p, w)
        dataset._session.comm.all_reduce(acc)
        a = acc.cpu().numpy()
        return _regression_metric(self.getMetricName(), a, self.getThroughOrigin())

    def isLargerBetter(self):
        return self.getMetricName() in ("r2", "var")


def _regression_metric(name, a, through_origin=False):
    W, sse, sae, sy, syy, sp, spp, syp = a.tolist()
    if W <= 0:
        return float("nan")
    mse = sse / W
    if name == "rmse":
        return math.sqrt(mse)
    if name == "mse":
        return mse
    if name == "mae":
        return sae / W
    if name == "r2":
        sst = syy if through_origin else syy - sy * sy / W
        return 1.0 - sse / sst if sst != 0 else float("nan")
    if name == "var":
        ybar = sy / W
        return (spp - 2 * ybar * sp + ybar * ybar * W) / W
    raise IllegalArgumentException(f"unsupported metric {name}")


def _score_column(b, col):
    c = b.columns[col]
    v = c.values
    if v.dim() == 2:
        return v[:, 1].double() if v.shape[1] > 1 else v[:, 0].double()
    return v.double()


def _roc_pr_exact(score: np.ndarray, label: np.ndarray, weight: np.ndarray):
    order = np.argsort(-score, kind="stable")
    s, l, w = score[order], label[order], weight[order]
    distinct = np.r_[np.nonzero(np.diff(s))[0], len(s) - 1] if len(s) else np.array([], dtype=np.int64)
    tp = np.cumsum(w * l)[distinct]
    fp = np.cumsum(w * (1 - l))[distinct]
    return tp, fp


def _roc_pr_exact_device(score: torch.Tensor, label: torch.Tensor, weight: torch.Tensor):
    """``_roc_pr_exact`` on the GPU: one device sort of the scores (descending) and fp64 cumulative sums; only the
    counts at the distinct-score boundaries come to the host.  The host version's np.argsort of a 3.3e6-row
    validation fold took 250 ms of a 20 ms RandomForestClassifier fit (the CrossValidator's evaluate dominated
    the L07 grid: 4.6 s for 13 fits at 1e7 rows).  With 0/1 labels and unit weights the sums are exact integers,
    so the counts equal the host path's."""
    n = score.numel()
    if n == 0:
        return np.zeros(0), np.zeros(0)
    s, order = torch.sort(score, descending=True, stable=True)
    lw = (weight * label)[order]
    tp = torch.cumsum(lw, 0)
    fp = torch.cumsum((weight * (1 - label))[order], 0)
    last = torch.ones(n, dtype=torch.bool, device=score.device)
    last[:-1] = s[1:] != s[:-1]
    idx = K.compact_mask(last)
    out = torch.stack([tp[idx], fp[idx]]).cpu().numpy()
    return out[0], out[1]


def _downsample(tp, fp, num_bins: int):
    """Spark's curve down-sampling (BinaryClassificationMetrics(numBins)): with more than 2 * numBins distinct
    scores, consecutive score points are grouped ``countsSize / numBins`` at a time (one partition: the grouping
    runs over the whole descending order) and the curve keeps the cumulative counts at each group's end."""
    k = len(tp)
    if num_bins <= 0 or k == 0:
        return tp, fp
    grouping = k // num_bins
    if grouping < 2:
        return tp, fp
    ends = np.arange(grouping - 1, k, grouping)
    if ends[-1] != k - 1:
        ends = np.r_[ends, k - 1]
    return tp[ends], fp[ends]


def _auc_from_counts(tp, fp, metric):
    P = tp[-1] if len(tp) else 0.0
    N = fp[-1] if len(fp) else 0.0
    if metric == "areaUnderROC":
        if P == 0 or N == 0:
            return float("nan")
        tpr = np.r_[0.0, tp / P, 1.0]
        fpr = np.r_[0.0, fp / N, 1.0]
        return float(np.trapezoid(tpr, fpr))
    if metric == "areaUnderPR":
        if P == 0:
            return float("nan")
        rec = tp / P
        prec = tp / np.maximum(tp + fp, 1e-300)
        rec = np.r_[0.0, rec]
        prec = np.r_[prec[0] if len(prec) else 1.0, prec]
        return float(np.trapezoid(prec, rec))
    raise IllegalArgumentException(f"unsupported metric {metric}")


class BinaryClassificationEvaluator(Evaluator):
    _params = {
        "rawPredictionCol": ("raw prediction (a.k.a. confidence) column name", "rawPrediction", TC.toString),
        "labelCol": ("label column name", "label", TC.toString),
        "metricName": ("metric name in evaluation (areaUnderROC|areaUnderPR)", "areaUnderROC", TC.toString),
        "weightCol": ("weight column name", None, TC.toString),
        "numBins": ("number of bins to down-sample the curves to", 1000, TC.toInt),
    }

    def __init__(self, rawPredictionCol=None, labelCol=None, metricName=None, weightCol=None, numBins=None):
        super().__init__()
        keyword_init(self, dict(rawPredictionCol=rawPredictionCol, labelCol=labelCol, metricName=metricName,
                                weightCol=weightCol, numBins=numBins))

    def _evaluate(self, dataset):
        rc, lc, wc = self.getRawPredictionCol(), self.getLabelCol(), self.getWeightCol()
        b = local_batch(dataset, [rc, lc] + ([wc] if wc else []))
        score = _score_column(b, rc)
        label = b.columns[lc].values.double()
        w = b.columns[wc].values.double() if wc else torch.ones_like(label)
        comm = dataset._session.comm
        metric = self.getMetricName()
        if not comm.distributed:
            if score.is_cuda and not bool(torch.isnan(score).any()):
                tp, fp = _roc_pr_exact_device(score.double(), label, w)
            else:
                tp, fp = _roc_pr_exact(score.cpu().numpy(), label.cpu().numpy(), w.cpu().numpy())
            return _auc_from_counts(*_downsample(tp, fp, self.getNumBins()), metric)
        lo = torch.tensor([float(score.min()) if score.numel() else float("inf")], device=comm.device)
        hi = torch.tensor([float(score.max()) if score.numel() else float("-inf")], device=comm.device)
        comm.all_reduce(lo, "min")
        comm.all_reduce(hi, "max")
        nb = 1 << 20
        h = K.score_hist(score, label, float(lo), float(hi), nb)
        comm.all_reduce(h)
        h = h.cpu().numpy()[::-1]  # descending score
        nz = (h.sum(1) > 0)
        tp = np.cumsum(h[:, 1])[nz]
        fp = np.cumsum(h[:, 0])[nz]
        return _auc_from_counts(*_downsample(tp, fp, self.getNumBins()), metric)

    def isLargerBetter(self):
        return True


class MulticlassClassificationEvaluator(Evaluator):
    _params = {
        "predictionCol": ("prediction column name", "prediction", TC.toString),
        "labelCol": ("label column name", "label", TC.toString),
        "metricName": ("metric name in evaluation (f1|accuracy|weightedPrecision|weightedRecall|"
                       "weightedTruePositiveRate|weightedFalsePositiveRate|weightedFMeasure|"
                       "truePositiveRateByLabel|falsePositiveRateByLabel|precisionByLabel|recallByLabel|"
                       "fMeasureByLabel|logLoss|hammingLoss)", "f1", TC.toString),
        "metricLabel": ("the class whose metric will be computed in *ByLabel", 0.0, TC.toFloat),
        "beta": ("the beta value used in weightedFMeasure|fMeasureByLabel", 1.0, TC.toFloat),
        "probabilityCol": ("probability column name", "probability", TC.toString),
        "weightCol": ("weight column name", None, TC.toString),
        "eps": ("log-loss clipping epsilon", 1e-15, TC.toFloat),
    }

    def __init__(self, predictionCol=None, labelCol=None, metricName=None, metricLabel=None, beta=None,
                 probabilityCol=None, weightCol=None, eps=None):
        super().__init__()
        keyword_init(self, dict(predictionCol=predictionCol, labelCol=labelCol, metricName=metricName,
                                metricLabel=metricLabel, beta=beta, probabilityCol=probabilityCol,
                                weightCol=weightCol, eps=eps))

    def _evaluate(self, dataset):
        comm = dataset._session.comm
        metric = self.getMetricName()
        pc, lc, wc = self.getPredictionCol(), self.getLabelCol(), self.getWeightCol()
        if metric == "logLoss":
            prc = self.getProbabilityCol()
            b = local_batch(dataset, [prc, lc] + ([wc] if wc else []))
            P = b.columns[prc].values.double()
            y = b.columns[lc].values.long()
            w = b.columns[wc].values.double() if wc else torch.ones(b.n, dtype=torch.float64, device=P.device)
            pr = P[torch.arange(b.n, device=P.device), y].clamp(self.getEps(), 1 - self.getEps())
            acc = torch.stack([(-torch.log(pr) * w).sum(), w.sum()])
            comm.all_reduce(acc)
            return float(acc[0] / acc[1])
        b = local_batch(dataset, [pc, lc] + ([wc] if wc else []))
        p = b.columns[pc].values.double()
        y = b.columns[lc].values.double()
        w = b.columns[wc].values.double() if wc else torch.ones_like(y)
        mx = torch.tensor([max(float(p.max()) if p.numel() else 0, float(y.max()) if y.numel() else 0)],
                          device=comm.device)
        comm.all_reduce(mx, "max")
        C = int(mx) + 1
        cm = torch.zeros(C * C, dtype=torch.float64, device=p.device)
        cm.index_add_(0, (y.long() * C + p.long()), w)
        comm.all_reduce(cm)
        M = cm.view(C, C).cpu().numpy()  # rows = true, cols = predicted
        return _multiclass_metric(metric, M, self.getMetricLabel(), self.getBeta())

    def isLargerBetter(self):
        return self.getMetricName() not in ("weightedFalsePositiveRate", "falsePositiveRateByLabel", "logLoss",
                                            "hammingLoss")


def _multiclass_metric(metric, M, label, beta):
    tot = M.sum()
    tp = np.diag(M)
    actual = M.sum(1)
    pred = M.sum(0)
    with np.errstate(divide="ignore", invalid="ignore"):
        prec = np.where(pred > 0, tp / pred, 0.0)
        rec = np.where(actual > 0, tp / actual, 0.0)
        fp = pred - tp
        neg = tot - actual
        fpr = np.where(neg > 0, fp / neg, 0.0)
        b2 = beta * beta
        f = np.where((b2 * prec + rec) > 0, (1 + b2) * prec * rec / (b2 * prec + rec), 0.0)
    wts = actual / tot if tot else actual
    li = int(label)
    if metric == "accuracy":
        return float(tp.sum() / tot) if tot else float("nan")
    if metric == "hammingLoss":
        return float(1 - tp.sum() / tot)
    if metric in ("f1", "weightedFMeasure"):
        return float((wts * f).sum())
    if metric == "weightedPrecision":
        return float((wts * prec).sum())
    if metric in ("weightedRecall", "weightedTruePositiveRate"):
        return float((wts * rec).sum())
    if metric == "weightedFalsePositiveRate":
        return float((wts * fpr).sum())
    if metric in ("truePositiveRateByLabel", "recallByLabel"):
        return float(rec[li])
    if metric == "falsePositiveRateByLabel":
        return float(fpr[li])
    if metric == "precisionByLabel":
        return float(prec[li])
    if metric == "fMeasureByLabel":
        return float(f[li])
    raise IllegalArgumentException(f"unsupported metric {metric}")


class ClusteringEvaluator(Evaluator):
    """Silhouette with squared Euclidean distance (Spark's closed form via cluster sums)."""
    _params = {
        "predictionCol": ("prediction column name", "prediction", TC.toString),
        "featuresCol": ("features column name", "features", TC.toString),
        "metricName": ("metric name (silhouette)", "silhouette", TC.toString),
        "distanceMeasure": ("squaredEuclidean", "squaredEuclidean", TC.toString),
    }

    def __init__(self, predictionCol=None, featuresCol=None, metricName=None, distanceMeasure=None):
        super().__init__()
        keyword_init(self, dict(predictionCol=predictionCol, featuresCol=featuresCol, metricName=metricName,
                                distanceMeasure=distanceMeasure))

    def _evaluate(self, dataset):
        comm = dataset._session.comm
        b = local_batch(dataset, [self.getFeaturesCol(), self.getPredictionCol()])
        X = b.columns[self.getFeaturesCol()].values.double()
        c = b.columns[self.getPredictionCol()].values.long()
        kmax = torch.tensor([float(c.max()) if c.numel() else 0.0], device=comm.device)
        comm.all_reduce(kmax, "max")
        k = int(kmax) + 1
        d = X.shape[1]
        sq = (X * X).sum(1)
        S = torch.zeros((k, d), dtype=torch.float64, device=X.device)
        S.index_add_(0, c, X)
        Q = torch.zeros(k, dtype=torch.float64, device=X.device).index_add_(0, c, sq)
        N = torch.zeros(k, dtype=torch.float64, device=X.device).index_add_(0, c, torch.ones_like(sq))
        comm.all_reduce_many([S, Q, N])
        # mean squared distance of each point to each cluster: (N_j |x|^2 - 2 x.S_j + Q_j) / N_j
        D = (N[None, :] * sq[:, None] - 2 * X @ S.T + Q[None, :]) / N.clamp_min(1)[None, :]
        own = D[torch.arange(b.n, device=X.device), c]
        n_own = N[c]
        a = own * n_own / (n_own - 1).clamp_min(1)
        D2 = D.clone()
        D2[torch.arange(b.n, device=X.device), c] = float("inf")
        bmin = D2.min(1).values
        s = torch.where(n_own > 1, (bmin - a) / torch.maximum(a, bmin), torch.zeros_like(a))
        acc = torch.stack([s.sum(), torch.tensor(float(b.n), dtype=torch.float64, device=X.device)])
        comm.all_reduce(acc)
        return float(acc[0] / acc[1])
