"""Classification algorithms.

LogisticRegression (binomial): every L-BFGS / OWL-QN iteration is ONE pass of
the fused K11 HIP kernel (margin, log-loss and gradient together) plus one
RCCL all-reduce of d+2 doubles; its margins are fp64 (Spark's Double).  Multinomial uses fp64 GEMMs at course
sizes, fp32 device GEMMs above MULTINOMIAL_F64_MAX.  Tree
classifiers (DT / RF / GBT) share the histogram engine with class-count
statistics (gini / entropy).  Reference: MLE 03 - Logistic Regression
Lab.py:99-158; Labs/ML 07L:42-209 (RandomForestClassifier + AUC).
"""
from __future__ import annotations

import math
from typing import Optional

import numpy as np
import torch

from ..ops import kernels as K
from ..sql import types as T
from ..sql.batch import ColumnData
from ..sql.dataframe import MapPlan
from .base import Estimator, Model
from .linalg import DenseMatrix, DenseVector
from .optim import minimize
from .param import NO_DEFAULT, TypeConverters as TC, keyword_init
from .regression import (_GBT, _PRED, _RF, _TREE, _TreeModelBase, _bag_weights, _combine_weights, _num_classes,
                         _subforest, resolve_subset, tree_fit_prepare)
from .tree.engine import ForestTrainer, TreeParams
from .tree.forest import Forest
from .util import VECTOR_F64_MAX, IllegalArgumentException, centered_gram, local_batch, local_xyw, require_vector

# multinomial logistic regression: fp64 logits / gradients up to this many n*d*C multiply-adds per pass (course
# sizes; Spark's Double), the fp32 device GEMMs above
MULTINOMIAL_F64_MAX = 4e9

_CLS = dict(_PRED, **{
    "probabilityCol": ("Column name for predicted class conditional probabilities.", "probability", TC.toString),
    "rawPredictionCol": ("raw prediction (a.k.a. confidence) column name", "rawPrediction", TC.toString),
    "thresholds": ("Thresholds in multi-class classification to adjust the probability of predicting each class.",
                   None, TC.toListFloat),
})


def _append_cls_outputs(b, raw, prob, pred, names):
    rc, pc, pr = names
    nb = b
    # Spark's rawPrediction / probability are Double vectors: kept fp64 at course scale (util.VECTOR_F64_MAX)
    vdt = torch.float64 if raw.numel() <= VECTOR_F64_MAX else torch.float32
    if rc:
        nb = nb.with_column(rc, ColumnData(raw.to(vdt), T.VectorUDT()))
    if pr:
        nb = nb.with_column(pr, ColumnData(prob.to(vdt), T.VectorUDT()))
    return nb.with_column(pc, ColumnData(pred.double(), T.DoubleType()))


def _argmax_with_thresholds(prob, thresholds):
    if thresholds:
        t = torch.tensor(thresholds, dtype=prob.dtype, device=prob.device)
        return torch.argmax(prob / t.clamp_min(1e-300), dim=1)
    return torch.argmax(prob, dim=1)


# ========================================================= LogisticRegression
class LogisticRegression(Estimator):
    _params = dict(_CLS, **{
        "maxIter": ("max number of iterations (>= 0)", 100, TC.toInt),
        "regParam": ("regularization parameter (>= 0)", 0.0, TC.toFloat),
        "elasticNetParam": ("the ElasticNet mixing parameter, in range [0, 1]", 0.0, TC.toFloat),
        "tol": ("the convergence tolerance for iterative algorithms (>= 0)", 1e-6, TC.toFloat),
        "fitIntercept": ("whether to fit an intercept term", True, TC.toBoolean),
        "threshold": ("Threshold in binary classification prediction, in range [0, 1].", 0.5, TC.toFloat),
        "standardization": ("whether to standardize the training features before fitting the model", True,
                            TC.toBoolean),
        "weightCol": ("weight column name", None, TC.toString),
        "aggregationDepth": ("suggested depth for treeAggregate (>= 2)", 2, TC.toInt),
        "family": ("The name of family: auto, binomial, multinomial", "auto", TC.toString),
    })

    def __init__(self, **kwargs):
        super().__init__()
        keyword_init(self, kwargs)

    def _fit(self, dataset):
        fc, lc, wc = self.getFeaturesCol(), self.getLabelCol(), self.getWeightCol()
        X, y, w = local_xyw(dataset, fc, lc, wc, keep_f64=True)
        session = dataset._session
        comm = session.comm
        d = X.shape[1]
        C = _num_classes(session, y, (dataset.schema[lc].metadata or {}).get("ml_attr"))
        C = max(C, 2)
        family = self.getFamily()
        if family == "auto":
            family = "binomial" if C <= 2 else "multinomial"
        if family == "binomial" and C > 2:
            raise IllegalArgumentException(f"Binomial family only supports 1 or 2 outcome classes but found {C}.")
        # feature std from the centred Gram (a raw-moment std weighs narrow, far-from-zero features wrongly in the
        # standardised L2 penalty)
        n, _, Cg = centered_gram(X, comm)
        var = np.clip(torch.diagonal(Cg).cpu().numpy(), 0, None) / max(n - 1, 1)
        if w is not None:
            wsum = torch.tensor([float(w.sum())], dtype=torch.float64, device=X.device)
            comm.all_reduce(wsum)
            n_eff = float(wsum)
        else:
            n_eff = n
        sd = np.sqrt(var)
        sdz = np.where(sd > 0, sd, 1.0)
        lam, alpha = self.getRegParam(), self.getElasticNetParam()
        std = self.getStandardization()
        fit_int = self.getFitIntercept()
        # L2/L1 weights in the standardized space
        p2 = np.ones(d) if std else 1.0 / (sdz * sdz)
        p1 = np.ones(d) if std else 1.0 / sdz
        if family == "binomial":
            def fg(theta):
                bs = theta[:d]
                b0 = theta[d] if fit_int else 0.0
                wt = torch.tensor(bs / sdz, dtype=torch.float64, device=X.device)
                g, loss = K.logistic_grad(X, y, wt, b0, w)
                acc = torch.cat([g, loss.reshape(1)])
                comm.all_reduce(acc)
                a = acc.cpu().numpy() / max(n_eff, 1e-300)
                grad = np.zeros(d + 1)
                grad[:d] = a[:d] / sdz + lam * (1 - alpha) * p2 * bs
                grad[d] = a[d] if fit_int else 0.0
                f = a[d + 1] + 0.5 * lam * (1 - alpha) * float(np.sum(p2 * bs * bs))
                return f, grad
            theta0 = np.zeros(d + 1)
            if fit_int:
                # initialise intercept at log-odds of the label mean (Spark does the same)
                pos = torch.tensor([float((y * (w if w is not None else 1)).sum())], dtype=torch.float64,
                                   device=X.device)
                comm.all_reduce(pos)
                pm = min(max(float(pos) / max(n_eff, 1e-300), 1e-12), 1 - 1e-12)
                theta0[d] = math.log(pm / (1 - pm))
            l1 = np.r_[lam * alpha * p1, 0.0] if lam * alpha > 0 else None
            theta, hist, iters = minimize(fg, theta0, self.getMaxIter(), self.getTol(), l1=l1)
            coef = theta[:d] / sdz
            coef[sd == 0] = 0.0
            model = LogisticRegressionModel(coef[None, :], np.array([theta[d] if fit_int else 0.0]), 2, False)
        else:
            Yoh = torch.nn.functional.one_hot(y.long(), C).double() if y.numel() else \
                torch.zeros((0, C), dtype=torch.float64, device=X.device)
            sd_t = torch.tensor(sdz, dtype=torch.float32, device=X.device)
            wv = w if w is not None else None

            # course-sized problems take fp64 logits and gradients (Spark's Double); large ones the fp32 GEMMs
            f64 = X.dtype == torch.float64 or X.shape[0] * d * C <= MULTINOMIAL_F64_MAX
            if f64:
                sd_t = sd_t.double()

            def fg(theta):
                Wm = theta[: C * d].reshape(C, d)
                b = theta[C * d:] if fit_int else np.zeros(C)
                Wt = torch.tensor(Wm, dtype=sd_t.dtype, device=X.device) / sd_t[None, :]
                logits = (_margins64(X, Wt) if f64 else (X @ Wt.T).double()) + \
                    torch.tensor(b, dtype=torch.float64, device=X.device)
                lse = torch.logsumexp(logits, 1)
                ll = lse - (logits * Yoh).sum(1)
                P = torch.softmax(logits, 1)
                R = P - Yoh
                if wv is not None:
                    ll = ll * wv
                    R = R * wv[:, None]
                gW = ((R.T @ X.double()) if f64 else (R.float().T @ X).double()) / sd_t.double()[None, :]
                gb = R.sum(0)
                acc = torch.cat([gW.reshape(-1), gb, ll.sum().reshape(1)])
                comm.all_reduce(acc)
                a = acc.cpu().numpy() / max(n_eff, 1e-300)
                grad = np.zeros(C * d + C)
                grad[: C * d] = a[: C * d] + lam * (1 - alpha) * (np.tile(p2, C) * theta[: C * d])
                grad[C * d:] = a[C * d: C * d + C] if fit_int else 0.0
                f = a[-1] + 0.5 * lam * (1 - alpha) * float(np.sum(np.tile(p2, C) * theta[: C * d] ** 2))
                return f, grad
            theta0 = np.zeros(C * d + C)
            l1 = np.r_[np.tile(lam * alpha * p1, C), np.zeros(C)] if lam * alpha > 0 else None
            theta, hist, iters = minimize(fg, theta0, self.getMaxIter(), self.getTol(), l1=l1)
            Wm = theta[: C * d].reshape(C, d) / sdz[None, :]
            b = theta[C * d:] if fit_int else np.zeros(C)
            if fit_int:
                b = b - b.mean()  # Spark centres multinomial intercepts
            model = LogisticRegressionModel(Wm, b, C, True)
        model._post_fit(self)
        model.summary = _LogRegTrainingSummary(model, dataset, hist, iters)
        return model


def _margins64(X: torch.Tensor, W: torch.Tensor, chunk: int = 1 << 20) -> torch.Tensor:
    """X [n, d] (fp32 features) @ W[C, d].T with fp64 products and sums (Spark's Double margins), in row chunks
    so the fp64 copy of X stays small."""
    W = W.to(X.device, torch.float64)
    out = torch.empty((X.shape[0], W.shape[0]), dtype=torch.float64, device=X.device)
    for r0 in range(0, X.shape[0], chunk):
        out[r0:r0 + chunk] = X[r0:r0 + chunk].double() @ W.T
    return out


class LogisticRegressionModel(Model):
    _params = LogisticRegression._params

    def __init__(self, coefficientMatrix=None, interceptVector=None, numClasses=2, isMultinomial=False):
        super().__init__()
        self._W = np.asarray(coefficientMatrix if coefficientMatrix is not None else np.zeros((1, 0)),
                             dtype=np.float64)
        self._b = np.asarray(interceptVector if interceptVector is not None else [0.0], dtype=np.float64)
        self._C = int(numClasses)
        self._multi = bool(isMultinomial)
        self.summary = None

    @property
    def coefficients(self):
        if self._multi:
            raise RuntimeError("Multinomial models contain a matrix of coefficients, use coefficientMatrix")
        return DenseVector(self._W[0])

    @property
    def intercept(self):
        if self._multi:
            raise RuntimeError("Multinomial models contain a vector of intercepts, use interceptVector")
        return float(self._b[0])

    @property
    def coefficientMatrix(self):
        return DenseMatrix(self._W.shape[0], self._W.shape[1], self._W.T.reshape(-1))

    @property
    def interceptVector(self):
        return DenseVector(self._b)

    @property
    def numClasses(self):
        return self._C

    @property
    def numFeatures(self):
        return self._W.shape[1]

    @property
    def hasSummary(self):
        return self.summary is not None

    def _transform(self, dataset):
        fc = self.getFeaturesCol()
        require_vector(dataset, fc)
        names = (self.getRawPredictionCol(), self.getPredictionCol(), self.getProbabilityCol())
        W = torch.tensor(self._W, dtype=torch.float64)
        bvec = torch.tensor(self._b, dtype=torch.float64)
        multi, thr = self._multi, self.getThreshold()
        thresholds = self.getThresholds()

        def fn(b, ctx):
            X = b.columns[fc].values
            X = X if X.dtype == torch.float64 else X.float()
            Wd, bd = W.to(X.device), bvec.to(X.device)
            if X.shape[0] == 0:
                z = torch.zeros((0, max(self._C, 2)), dtype=torch.float64, device=X.device)
                return _append_cls_outputs(b, z, z, z[:, 0], (names[0], names[1], names[2]))
            if not multi:
                m = _margins64(X, Wd[:1])[:, 0] + bd[0]
                raw = torch.stack([-m, m], 1)
                p1 = torch.sigmoid(m)
                prob = torch.stack([1 - p1, p1], 1)
                pred = (p1 > thr).double() if not thresholds else _argmax_with_thresholds(prob, thresholds)
            else:
                raw = _margins64(X, Wd) + bd
                prob = torch.softmax(raw, 1)
                pred = _argmax_with_thresholds(prob, thresholds)
            return _append_cls_outputs(b, raw, prob, pred, (names[0], names[1], names[2]))
        return dataset._new(MapPlan(dataset._plan, "LogisticRegressionModel", fn))

    def predict(self, features):
        x = np.asarray(features.toArray() if hasattr(features, "toArray") else features)
        if not self._multi:
            return float(1.0 / (1 + math.exp(-(x @ self._W[0] + self._b[0]))) > self.getThreshold())
        return float(np.argmax(self._W @ x + self._b))

    def evaluate(self, dataset):
        return _LogRegSummary(self, dataset)

    def _save_state(self):
        return {"numClasses": self._C, "isMultinomial": self._multi}, {"W": torch.tensor(self._W),
                                                                     "b": torch.tensor(self._b)}

    def _load_state(self, extra, tensors, stages):
        self._W, self._b = tensors["W"].numpy(), tensors["b"].numpy()
        self._C, self._multi = int(extra["numClasses"]), bool(extra["isMultinomial"])
        self.summary = None


class _LogRegSummary:
    def __init__(self, model, dataset):
        self._model = model
        self.predictions = model.transform(dataset)
        self.labelCol = model.getLabelCol()
        self.predictionCol = model.getPredictionCol()
        self.probabilityCol = model.getProbabilityCol()

    def _mc(self, metric, **kw):
        from .evaluation import MulticlassClassificationEvaluator
        return MulticlassClassificationEvaluator(labelCol=self.labelCol, predictionCol=self.predictionCol,
                                                 metricName=metric, **kw).evaluate(self.predictions)

    @property
    def accuracy(self):
        return self._mc("accuracy")

    @property
    def weightedPrecision(self):
        return self._mc("weightedPrecision")

    @property
    def weightedRecall(self):
        return self._mc("weightedRecall")

    @property
    def weightedFMeasure(self):
        return self._mc("weightedFMeasure")

    @property
    def areaUnderROC(self):
        from .evaluation import BinaryClassificationEvaluator
        return BinaryClassificationEvaluator(labelCol=self.labelCol,
                                             rawPredictionCol=self._model.getRawPredictionCol()).evaluate(
            self.predictions)

    def _curve(self, kind):
        from ..sql.batch import batch_from_pandas
        import pandas as pd
        pdf = self.predictions.select(self.probabilityCol, self.labelCol).toPandas()
        s = np.array([v[1] for v in pdf[self.probabilityCol]])
        l = pdf[self.labelCol].to_numpy(np.float64)
        from .evaluation import _roc_pr_exact
        tp, fp = _roc_pr_exact(s, l, np.ones_like(l))
        P, N = max(tp[-1], 1e-300), max(fp[-1], 1e-300)
        sess = self.predictions._session
        if kind == "roc":
            return sess.createDataFrame(pd.DataFrame({"FPR": np.r_[0.0, fp / N, 1.0], "TPR": np.r_[0.0, tp / P, 1.0]}))
        prec = tp / np.maximum(tp + fp, 1e-300)
        return sess.createDataFrame(pd.DataFrame({"recall": np.r_[0.0, tp / P], "precision": np.r_[prec[0], prec]}))

    @property
    def roc(self):
        return self._curve("roc")

    @property
    def pr(self):
        return self._curve("pr")


class _LogRegTrainingSummary(_LogRegSummary):
    def __init__(self, model, dataset, hist, iters):
        super().__init__(model, dataset)
        self.objectiveHistory = hist
        self.totalIterations = iters


# ========================================================= tree classifiers
class _TreeClassifierModel(_TreeModelBase):
    _counts_raw = False  # DecisionTree: raw = leaf class counts; forests: raw = sum of probabilities

    @property
    def numClasses(self):
        return self._forest.K

    def _transform(self, dataset):
        fc = self.getFeaturesCol()
        require_vector(dataset, fc)
        names = (self.getRawPredictionCol(), self.getPredictionCol(), self.getProbabilityCol())
        forest, tw = self._forest, self._tree_w
        kind = "counts" if self._counts_raw else "value"
        thresholds = self.getThresholds()
        from .inference import predictor_for
        predictor = predictor_for(self, kind)

        def fn(b, ctx):
            X = b.columns[fc].values
            if X.shape[0] == 0:
                z = torch.zeros((0, forest.K), dtype=torch.float64, device=X.device)
                return _append_cls_outputs(b, z, z, z[:, 0], names)
            raw = predictor(X).double()
            s = raw.sum(1, keepdim=True)
            prob = raw / torch.where(s > 0, s, torch.ones_like(s))
            pred = _argmax_with_thresholds(prob, thresholds)
            out = _append_cls_outputs(b, raw, prob, pred, names)
            extra = {}
            self._leaf_col(b, extra)
            for k, v in extra.items():
                out = out.with_column(k, v)
            return out
        return dataset._new(MapPlan(dataset._plan, f"{type(self).__name__}", fn))

    def predict(self, features):
        x = torch.tensor(np.asarray(features.toArray() if hasattr(features, "toArray") else features),
                         dtype=torch.float32)[None, :]
        raw = self._forest.predict(x, self._tree_w, None, "counts" if self._counts_raw else "value")
        return float(torch.argmax(raw[0]))

    def evaluate(self, dataset):
        return _LogRegSummary(self, dataset)


def _train_forest_cls(est, dataset, T_, subset_strategy, bootstrap, rate, impurity):
    session, data, y, w, seed, meta = tree_fit_prepare(est, dataset, classification=True)
    C = _num_classes(session, y, (dataset.schema[est.getLabelCol()].metadata or {}).get("ml_attr"))
    C = max(C, 2)
    subset = resolve_subset(subset_strategy, data.d, T_, True)
    p = TreeParams(max_depth=est.getMaxDepth(), max_bins=est.getMaxBins(),
                   min_instances=float(est.getMinInstancesPerNode()), min_info_gain=est.getMinInfoGain(),
                   impurity=impurity, num_classes=C, feature_subset=subset, bootstrap=bootstrap,
                   subsampling_rate=rate, seed=seed)
    weights = _bag_weights(data, T_, bootstrap, rate, seed)
    if w is not None:
        weights = _combine_weights(weights, w, T_)
    forest = ForestTrainer(session, data, p).train(T_, {"label": y.int()}, weights)
    return forest, data.d


class DecisionTreeClassifier(Estimator):
    _params = dict(_CLS, **_TREE, **{
        "impurity": ("Criterion used for information gain calculation: entropy, gini", "gini", TC.toString),
    })

    def __init__(self, **kwargs):
        super().__init__()
        keyword_init(self, kwargs)

    def _fit(self, dataset):
        forest, d = _train_forest_cls(self, dataset, 1, "all", False, 1.0, self.getImpurity())
        return DecisionTreeClassificationModel(forest, d, [1.0])


class DecisionTreeClassificationModel(_TreeClassifierModel):
    _params = DecisionTreeClassifier._params
    _counts_raw = True


class RandomForestClassifier(Estimator):
    _params = dict(_CLS, **_TREE, **_RF, **{
        "impurity": ("Criterion used for information gain calculation: entropy, gini", "gini", TC.toString),
    })

    def __init__(self, **kwargs):
        super().__init__()
        keyword_init(self, kwargs)

    def _fit(self, dataset):
        T_ = self.getNumTrees()
        forest, d = _train_forest_cls(self, dataset, T_, self.getFeatureSubsetStrategy(), self.getBootstrap(),
                                      self.getSubsamplingRate(), self.getImpurity())
        return RandomForestClassificationModel(forest, d, np.ones(T_))


class RandomForestClassificationModel(_TreeClassifierModel):
    _params = RandomForestClassifier._params

    @property
    def trees(self):
        return [DecisionTreeClassificationModel(_subforest(self._forest, t), self._numFeatures, [1.0])
                for t in range(len(self._forest.roots))]


class GBTClassifier(Estimator):
    """Spark GBT (LogLoss on labels mapped to ±1, variance-impurity trees on pseudo-residuals)."""
    _params = dict(_CLS, **_TREE, **_GBT, **{
        "lossType": ("Loss function which GBT tries to minimize: logistic", "logistic", TC.toString),
    })

    def __init__(self, **kwargs):
        super().__init__()
        keyword_init(self, kwargs)

    def _fit(self, dataset):
        from .regression import boost
        session, data, y, w, seed, meta = tree_fit_prepare(self, dataset, classification=False)
        ypm = (2 * y - 1).float()
        grad = lambda F: 4 * ypm / (1 + torch.exp(2 * ypm * F))  # noqa: E731  (negative gradient of LogLoss)
        forest, tw = boost(session, data, lambda F: ypm, grad, self.getMaxIter(), self, seed, 0.0)
        return GBTClassificationModel(forest, data.d, tw)


class GBTClassificationModel(_TreeModelBase):
    _params = GBTClassifier._params

    @property
    def numClasses(self):
        return 2

    @property
    def trees(self):
        from .regression import DecisionTreeRegressionModel
        return [DecisionTreeRegressionModel(_subforest(self._forest, t), self._numFeatures, [1.0])
                for t in range(len(self._forest.roots))]

    def _transform(self, dataset):
        fc = self.getFeaturesCol()
        require_vector(dataset, fc)
        names = (self.getRawPredictionCol(), self.getPredictionCol(), self.getProbabilityCol())
        forest, tw = self._forest, self._tree_w

        def fn(b, ctx):
            X = b.columns[fc].values
            F = forest.predict(X, tw)[:, 0].double() if X.shape[0] else torch.zeros(0, dtype=torch.float64,
                                                                                     device=X.device)
            raw = torch.stack([-F, F], 1)
            p1 = 1.0 / (1.0 + torch.exp(-2 * F))
            prob = torch.stack([1 - p1, p1], 1)
            return _append_cls_outputs(b, raw, prob, (F > 0).double(), names)
        return dataset._new(MapPlan(dataset._plan, "GBTClassificationModel", fn))


# =============================================================== NaiveBayes
class NaiveBayes(Estimator):
    _params = dict(_CLS, **{
        "smoothing": ("The smoothing parameter, should be >= 0", 1.0, TC.toFloat),
        "modelType": ("multinomial, bernoulli or gaussian", "multinomial", TC.toString),
        "weightCol": ("weight column name", None, TC.toString),
    })

    def __init__(self, **kwargs):
        super().__init__()
        keyword_init(self, kwargs)

    def _fit(self, dataset):
        X, y, w = local_xyw(dataset, self.getFeaturesCol(), self.getLabelCol(), self.getWeightCol())
        session = dataset._session
        C = max(_num_classes(session, y, None), 2)
        d = X.shape[1]
        ww = w if w is not None else torch.ones_like(y)
        Yoh = torch.nn.functional.one_hot(y.long(), C).double() * ww[:, None] if y.numel() else \
            torch.zeros((0, C), dtype=torch.float64, device=X.device)
        cnt = Yoh.sum(0)
        S = (Yoh.float().T @ X).double()
        SS = (Yoh.float().T @ (X * X)).double()
        session.comm.all_reduce_many([cnt, S, SS])
        lam = self.getSmoothing()
        mt = self.getModelType()
        pi = torch.log((cnt + lam) / (cnt.sum() + C * lam))
        if mt == "multinomial":
            theta = torch.log((S + lam) / (S.sum(1, keepdim=True) + d * lam))
            sigma = None
        elif mt == "bernoulli":
            theta = torch.log((S + lam) / (cnt[:, None] + 2 * lam))
            sigma = None
        else:
            mu = S / cnt.clamp_min(1)[:, None]
            var = SS / cnt.clamp_min(1)[:, None] - mu * mu
            theta, sigma = mu, var.clamp_min(1e-9) + 1e-9 * float(var.max())
        return NaiveBayesModel(pi.cpu().numpy(), theta.cpu().numpy(), None if sigma is None else sigma.cpu().numpy(),
                               mt)


class NaiveBayesModel(Model):
    _params = NaiveBayes._params

    def __init__(self, pi=None, theta=None, sigma=None, modelType="multinomial"):
        super().__init__()
        self._pi = np.asarray(pi if pi is not None else [])
        self._theta = np.asarray(theta if theta is not None else np.zeros((0, 0)))
        self._sigma = None if sigma is None else np.asarray(sigma)
        self._mt = modelType

    @property
    def pi(self):
        return DenseVector(self._pi)

    @property
    def theta(self):
        return DenseMatrix(self._theta.shape[0], self._theta.shape[1], self._theta.T.reshape(-1))

    def _transform(self, dataset):
        fc = self.getFeaturesCol()
        names = (self.getRawPredictionCol(), self.getPredictionCol(), self.getProbabilityCol())
        pi, th = torch.tensor(self._pi), torch.tensor(self._theta)
        sg = None if self._sigma is None else torch.tensor(self._sigma)
        mt = self._mt

        def fn(b, ctx):
            X = b.columns[fc].values.double()
            if mt == "multinomial":
                raw = X @ th.to(X.device).T + pi.to(X.device)
            elif mt == "bernoulli":
                t = th.to(X.device)
                neg = torch.log1p(-torch.exp(t).clamp(max=1 - 1e-12))
                raw = X @ (t - neg).T + neg.sum(1) + pi.to(X.device)
            else:
                mu, var = th.to(X.device), sg.to(X.device)
                raw = -0.5 * (((X[:, None, :] - mu[None]) ** 2) / var[None] + torch.log(2 * math.pi * var[None])).sum(
                    2) + pi.to(X.device)
            prob = torch.softmax(raw, 1)
            return _append_cls_outputs(b, raw, prob, torch.argmax(prob, 1), names)
        return dataset._new(MapPlan(dataset._plan, "NaiveBayesModel", fn))

    def _save_state(self):
        t = {"pi": torch.tensor(self._pi), "theta": torch.tensor(self._theta)}
        if self._sigma is not None:
            t["sigma"] = torch.tensor(self._sigma)
        return {"modelType": self._mt}, t

    def _load_state(self, extra, tensors, stages):
        self._pi, self._theta = tensors["pi"].numpy(), tensors["theta"].numpy()
        self._sigma = tensors["sigma"].numpy() if "sigma" in tensors else None
        self._mt = extra["modelType"]


class LinearSVC(Estimator):
    """Linear SVM (squared hinge smoothed with L-BFGS on device GEMV passes)."""
    _params = dict(_PRED, **{
        "rawPredictionCol": ("raw prediction column name", "rawPrediction", TC.toString),
        "maxIter": ("max number of iterations", 100, TC.toInt),
        "regParam": ("regularization parameter", 0.0, TC.toFloat),
        "tol": ("convergence tolerance", 1e-6, TC.toFloat),
        "fitIntercept": ("whether to fit an intercept term", True, TC.toBoolean),
        "threshold": ("threshold on the raw prediction", 0.0, TC.toFloat),
        "standardization": ("standardize features", True, TC.toBoolean),
        "weightCol": ("weight column name", None, TC.toString),
    })

    def __init__(self, **kwargs):
        super().__init__()
        keyword_init(self, kwargs)

    def _fit(self, dataset):
        X, y, w = local_xyw(dataset, self.getFeaturesCol(), self.getLabelCol(), self.getWeightCol())
        comm = dataset._session.comm
        d = X.shape[1]
        ys = (2 * y - 1)
        ww = w if w is not None else torch.ones_like(y)
        nt = torch.tensor([float(ww.sum())], dtype=torch.float64, device=X.device)
        comm.all_reduce(nt)
        n = float(nt)
        lam = self.getRegParam()

        def fg(theta):
            wt = torch.tensor(theta[:d], dtype=torch.float32, device=X.device)
            m = (X @ wt).double() + theta[d]
            marg = 1 - ys * m
            act = marg > 0
            loss = (ww * torch.where(act, marg * marg, torch.zeros_like(marg))).sum()
            r = torch.where(act, -2 * ys * marg, torch.zeros_like(marg)) * ww
            g = torch.cat([(r.float() @ X).double(), r.sum().reshape(1), loss.reshape(1)])
            comm.all_reduce(g)
            a = g.cpu().numpy() / n
            grad = a[: d + 1].copy()
            grad[:d] += lam * theta[:d]
            return a[d + 1] + 0.5 * lam * float(theta[:d] @ theta[:d]), grad
        theta, hist, it = minimize(fg, np.zeros(d + 1), self.getMaxIter(), self.getTol())
        return LinearSVCModel(theta[:d], theta[d])


class LinearSVCModel(Model):
    _params = LinearSVC._params

    def __init__(self, coefficients=None, intercept=0.0):
        super().__init__()
        self._w = np.asarray(coefficients if coefficients is not None else [])
        self._b = float(intercept)

    @property
    def coefficients(self):
        return DenseVector(self._w)

    @property
    def intercept(self):
        return self._b

    def _transform(self, dataset):
        fc, pc, rc = self.getFeaturesCol(), self.getPredictionCol(), self.getRawPredictionCol()
        wt = torch.tensor(self._w, dtype=torch.float32)
        b0, thr = self._b, self.getThreshold()

        def fn(b, ctx):
            X = b.columns[fc].values.float()
            m = (X @ wt.to(X.device)).double() + b0
            nb = b.with_column(rc, ColumnData(torch.stack([-m, m], 1).float(), T.VectorUDT()))
            return nb.with_column(pc, ColumnData((m > thr).double(), T.DoubleType()))
        return dataset._new(MapPlan(dataset._plan, "LinearSVCModel", fn))

    def _save_state(self):
        return {"intercept": self._b}, {"w": torch.tensor(self._w)}

    def _load_state(self, extra, tensors, stages):
        self._w, self._b = tensors["w"].numpy(), float(extra["intercept"])
