"""Regression algorithms.

LinearRegression: ONE pass of the fused MFMA Gram kernel (K1) per rank, one
RCCL all-reduce of the (d+2)² f64 statistics, then an exact host solve in the
standardized space (Cholesky / least squares for OLS & ridge, coordinate
descent for elastic net — all sufficient statistics are in the Gram, so no
further data passes are needed; cf. Labs/ML 02L:68-79 "matrix decomposition"
first, iterative fallback).

Tree regressors delegate to :mod:`cdnaml.models.tree.engine`.
"""
from __future__ import annotations

import math
import weakref
import zlib
from typing import Optional

import numpy as np
import torch

from ..ops import kernels as K
from ..sql import types as T
from ..sql.batch import ColumnData
from ..sql.dataframe import MapPlan
from .base import Estimator, Model
from .linalg import DenseVector, SparseVector
from .param import NO_DEFAULT, TypeConverters as TC, keyword_init
from .tree.binning import make_binned
from .tree.engine import ForestTrainer, TreeParams
from .tree import forest as _forest_mod
from .tree.forest import FitBins, Forest
from .util import (IllegalArgumentException, categorical_info, global_count, global_offset, gram_fp64_auto,
                   local_batch, local_xyw, require_vector, streamed_columns)

_PRED = {
    "featuresCol": ("features column name", "features", TC.toString),
    "labelCol": ("label column name", "label", TC.toString),
    "predictionCol": ("prediction column name", "prediction", TC.toString),
}


def _default_seed(cls) -> int:
    return zlib.crc32(cls.__name__.encode()) & 0x7FFFFFFF


# =============================================================== summaries
class _RegressionSummary:
    def __init__(self, predictions, labelCol, predictionCol, numFeatures=0):
        self.predictions = predictions
        self.labelCol = labelCol
        self.predictionCol = predictionCol
        self._acc = None
        self._numFeatures = numFeatures

    def _sums(self):
        if self._acc is None:
            from .evaluation import RegressionEvaluator
            b = local_batch(self.predictions, [self.labelCol, self.predictionCol])
            acc = K.reg_metrics(b.columns[self.labelCol].values, b.columns[self.predictionCol].values)
            self.predictions._session.comm.all_reduce(acc)
            self._acc = acc.cpu().numpy()
        return self._acc

    def _m(self, name):
        from .evaluation import _regression_metric
        return _regression_metric(name, self._sums())

    @property
    def rootMeanSquaredError(self):
        return self._m("rmse")

    @property
    def meanSquaredError(self):
        return self._m("mse")

    @property
    def meanAbsoluteError(self):
        return self._m("mae")

    @property
    def r2(self):
        return self._m("r2")

    @property
    def explainedVariance(self):
        return self._m("var")

    @property
    def numInstances(self):
        return int(self._sums()[0])

    @property
    def r2adj(self):
        n, p = self.numInstances, self._numFeatures
        return 1 - (1 - self.r2) * (n - 1) / max(n - p - 1, 1)

    @property
    def residuals(self):
        from ..sql import functions as F
        return self.predictions.select((F.col(self.labelCol) - F.col(self.predictionCol)).alias("residuals"))

    @property
    def degreesOfFreedom(self):
        return self.numInstances - self._numFeatures - 1


class LinearRegressionTrainingSummary(_RegressionSummary):
    def __init__(self, predictions, labelCol, predictionCol, numFeatures, objectiveHistory, totalIterations,
                 stderr=None, coef=None, intercept=None):
        super().__init__(predictions, labelCol, predictionCol, numFeatures)
        self.objectiveHistory = objectiveHistory
        self.totalIterations = totalIterations
        self._stderr = stderr
        self._coef = coef
        self._intercept = intercept

    @property
    def coefficientStandardErrors(self):
        if callable(self._stderr):
            self._stderr = self._stderr()
        if self._stderr is None:
            raise RuntimeError("No Std. Error of coefficients available for this LinearRegressionModel")
        return list(self._stderr)

    @property
    def tValues(self):
        se = self.coefficientStandardErrors
        vals = list(self._coef) + [self._intercept]
        return [v / s if s > 0 else float("nan") for v, s in zip(vals, se)]

    @property
    def pValues(self):
        from scipy import stats
        dof = max(self.degreesOfFreedom, 1)
        return [float(2 * stats.t.sf(abs(t), dof)) for t in self.tValues]


def _gram_fp64(prec: str, n: int, d: int) -> bool:
    """gramPrecision "auto" (util.gram_fp64_auto): course-sized problems take an fp64 library GEMM of the
    augmented matrix -- Spark's normal-equation solver works in fp64 and course-sized one-hot designs are
    ill-conditioned (condition ~1e4: the K1 kernel's fp32 block accumulation moved coefficients by ~2e-3
    relative); larger ones take K1 (fp32 MFMA, HBM-bound)."""
    if prec == "fp64":
        return True
    return prec == "auto" and gram_fp64_auto(n, d)


def _lr_shift(Xk: torch.Tensor, yk: torch.Tensor, comm, d: int) -> torch.Tensor:
    """[d + 1] fp64 common shift of the features and the label: the mean of every rank's leading rows (averaged
    over the ranks that have any).  It only conditions the f32 Gram; the solve un-shifts exactly with the host
    copy of the same values."""
    k = Xk.shape[0]
    if comm.distributed:
        sh = torch.cat([torch.mean(Xk, 0, dtype=torch.float64), yk.double().mean().reshape(1)]) if k else \
            torch.zeros(d + 1, dtype=torch.float64, device=Xk.device)
        cnt = torch.full((1,), 1.0 if k else 0.0, dtype=torch.float64, device=Xk.device)
        comm.all_reduce_many([sh, cnt])
        return sh / cnt.clamp_min(1.0)
    # one rank: fp64-accumulated column means of the fp32 rows (no fp64 copy of the block), no all-reduce
    return torch.cat([torch.mean(Xk, 0, dtype=torch.float64), yk.double().mean().reshape(1)]) if k else \
        torch.zeros(d + 1, dtype=torch.float64, device=Xk.device)


def _cho_factor(A):
    from scipy.linalg import cho_factor  # lazily: tree / xgboost imports of this module need no scipy
    return cho_factor(A, lower=True, check_finite=False)


def _cho_solve(cl, b):
    from scipy.linalg import cho_solve
    return cho_solve(cl, b, check_finite=False)


# =========================================================== LinearRegression
class LinearRegression(Estimator):
    _params = dict(_PRED, **{
        "maxIter": ("max number of iterations (>= 0)", 100, TC.toInt),
        "regParam": ("regularization parameter (>= 0)", 0.0, TC.toFloat),
        "elasticNetParam": ("the ElasticNet mixing parameter, in range [0, 1]", 0.0, TC.toFloat),
        "tol": ("the convergence tolerance for iterative algorithms (>= 0)", 1e-6, TC.toFloat),
        "fitIntercept": ("whether to fit an intercept term", True, TC.toBoolean),
        "standardization": ("whether to standardize the training features before fitting the model", True,
                            TC.toBoolean),
        "solver": ("the solver algorithm for optimization: auto, normal, l-bfgs", "auto", TC.toString),
        "weightCol": ("weight column name", None, TC.toString),
        "aggregationDepth": ("suggested depth for treeAggregate (>= 2)", 2, TC.toInt),
        "loss": ("the loss function to be optimized: squaredError, huber", "squaredError", TC.toString),
        "epsilon": ("the shape parameter to control the amount of robustness (huber)", 1.35, TC.toFloat),
        "gramPrecision": ("Gram precision: auto (fp64 library GEMM for small problems, else fp32), fp32 (K1 f32 MFMA "
                          "with fp32 block accumulation), bf16 (K1 bf16 MFMA) or fp64", "auto", TC.toString),
    })

    def __init__(self, featuresCol=None, labelCol=None, predictionCol=None, maxIter=None, regParam=None,
                 elasticNetParam=None, tol=None, fitIntercept=None, standardization=None, solver=None,
                 weightCol=None, aggregationDepth=None, loss=None, epsilon=None, gramPrecision=None):
        super().__init__()
        keyword_init(self, {k: v for k, v in locals().items() if k not in ("self", "__class__")})

    def _fit(self, dataset):
        fc, lc, wc = self.getFeaturesCol(), self.getLabelCol(), self.getWeightCol()
        require_vector(dataset, fc)
        from .util import require_numeric
        require_numeric(dataset, lc)
        src = streamed_columns(dataset, fc, [lc] + ([wc] if wc else []), head_rows=4096)
        if src is not None:
            return self._fit_streamed(dataset, src, lc, wc)
        X, y, w = local_xyw(dataset, fc, lc, wc, keep_f64=True)
        comm = dataset._session.comm
        d = X.shape[1]
        fit_int = self.getFitIntercept()
        # common shift (global mean of per-rank leading samples) keeps the f32 Gram well conditioned; it stays on
        # the device (the label shift is applied to y there), so the fit reads the host once, for the Gram
        bf16 = self.getGramPrecision() == "bf16"
        fp64 = _gram_fp64(self.getGramPrecision(), X.shape[0], d + (1 if w is not None else 0))
        sh = shift = None
        yc = y
        if fit_int:
            sh = _lr_shift(X[:4096], y[:4096], comm, d)
            shift = sh[:d].float()
            # y - mean in fp64, rounded to fp32, in one pass (the Gram reads the fp32 label)
            yc = K.shifted_f32(y, sh[d:]) if y.is_cuda else y - sh[d]
        if w is None:
            G = K.gram(X, yc, shift, 0.0, bf16=bf16, fp64=fp64) if X.shape[0] else \
                torch.zeros((d + 2, d + 2), dtype=torch.float64, device=X.device)
        else:
            # weighted Gram on K1 too: rows scaled by sqrt(w), with sqrt(w) itself as an extra feature column,
            # so [X' | sqrt(w) | 1 | y']^T [...] holds sum w x x^T, sum w x, sum w and the y blocks
            sw = torch.sqrt(w).float()[:, None]
            Xw = torch.cat([(X.float() - (shift if shift is not None else 0.0)) * sw, sw], 1)
            G3 = K.gram(Xw, (yc.float() * sw[:, 0]), None, 0.0, bf16=bf16, fp64=fp64) if X.shape[0] else \
                torch.zeros((d + 3, d + 3), dtype=torch.float64, device=X.device)
            keep = torch.tensor(list(range(d + 1)) + [d + 2], device=X.device)
            G = G3[keep][:, keep].contiguous()
        comm.all_reduce(G)
        host = torch.cat([G.reshape(-1), sh if sh is not None else G.new_zeros(d + 1)]).cpu().numpy()
        G = host[:(d + 2) * (d + 2)].reshape(d + 2, d + 2)
        yshift = float(host[-1]) if fit_int else 0.0
        # the f32 shift the Gram kernel subtracted, from the same host copy (no second device read)
        shift_h = host[(d + 2) * (d + 2):(d + 2) * (d + 2) + d].astype(np.float32).astype(np.float64) \
            if shift is not None else None
        coef, intercept, hist, iters, stderr = self._solve(G, d, shift_h, yshift)
        if X.dtype == torch.float64:
            coef, intercept = self._refine(X, y, w, comm, G, d, shift_h, yshift, coef, intercept)
        model = LinearRegressionModel(coef, intercept)
        model._post_fit(self)
        preds = model.transform(dataset)
        model.summary = LinearRegressionTrainingSummary(preds, lc, self.getPredictionCol(), d, hist, iters,
                                                        stderr, coef, intercept)
        return model

    def _fit_streamed(self, dataset, src, lc, wc):
        """Out-of-core fit: K1 Gram blocks accumulated chunk by chunk in fp64 (X never resident),
        the shift taken from the first chunk's leading rows, then the same solve as the materialised fit."""
        Xs, cd, _ = src
        comm = dataset._session.comm
        d = Xs.d
        y = cd[lc].values.double()
        w = cd[wc].values.double() if wc else None
        fit_int = self.getFitIntercept()
        bf16 = self.getGramPrecision() == "bf16"
        fp64 = _gram_fp64(self.getGramPrecision(), Xs.n, d + (1 if w is not None else 0))
        dev = Xs.device
        head = cd["__head__"]
        sh = _lr_shift(head, y[:head.shape[0]], comm, d) if fit_int else \
            torch.zeros(d + 1, dtype=torch.float64, device=dev)
        shift = sh[:d].float() if fit_int else None
        extra = 1 if w is not None else 0
        G = torch.zeros((d + 2 + extra, d + 2 + extra), dtype=torch.float64, device=dev)
        for r0, Xc in Xs:
            m = Xc.shape[0]
            yc_ = y[r0:r0 + m]
            ycc = yc_ - sh[d] if fit_int else yc_
            if m == 0:
                continue
            if w is None:
                G += K.gram(Xc, ycc, shift, 0.0, bf16=bf16, fp64=fp64)
            else:
                sw = torch.sqrt(w[r0:r0 + m]).float()[:, None]
                Xw = torch.cat([(Xc.float() - (shift if shift is not None else 0.0)) * sw, sw], 1)
                G += K.gram(Xw, ycc.float() * sw[:, 0], None, 0.0, bf16=bf16, fp64=fp64)
        if w is not None:
            keep = torch.tensor(list(range(d + 1)) + [d + 2], device=dev)
            G = G[keep][:, keep].contiguous()
        comm.all_reduce(G)
        host = torch.cat([G.reshape(-1), sh]).cpu().numpy()
        Gh = host[:(d + 2) * (d + 2)].reshape(d + 2, d + 2)
        yshift = float(host[-1]) if fit_int else 0.0
        shift_h = host[(d + 2) * (d + 2):(d + 2) * (d + 2) + d].astype(np.float32).astype(np.float64) \
            if fit_int else None
        coef, intercept, hist, iters, stderr = self._solve(Gh, d, shift_h, yshift)
        model = LinearRegressionModel(coef, intercept)
        model._post_fit(self)
        model.summary = LinearRegressionTrainingSummary(model.transform(dataset), lc, self.getPredictionCol(), d,
                                                        hist, iters, stderr, coef, intercept)
        return model

    def _solve(self, G, d, shift, yshift):
        n = G[d, d]
        if n <= 0:
            raise IllegalArgumentException("requirement failed: empty training dataset")
        sx, sy = G[:d, d], G[d + 1, d]
        Sxx, Sxy, Syy = G[:d, :d], G[:d, d + 1], G[d + 1, d + 1]
        fit_int = self.getFitIntercept()
        s = np.asarray(shift, dtype=np.float64) if shift is not None else np.zeros(d)
        mx = s + sx / n
        my = yshift + sy / n
        Cxx = Sxx - np.outer(sx, sx) / n
        Cxy = Sxy - sx * sy / n
        Cyy = Syy - sy * sy / n
        varx = np.clip(np.diag(Cxx) / n, 0, None)
        sdx = np.sqrt(varx)
        vary = max(Cyy / n, 0.0)
        sdy = math.sqrt(vary)
        lam, alpha = self.getRegParam(), self.getElasticNetParam()
        if fit_int and sdy > 0.0 and (lam == 0.0 or alpha == 0.0) and bool((sdx > 0).all()):
            fast = self._solve_ridge(sdx, sdy, lam, alpha, d, n, mx, my, Cxx, Cxy, Cyy)
            if fast is not None:
                return fast
        if fit_int:
            M, c, yy = Cxx / n, Cxy / n, Cyy / n
        else:
            # raw (uncentred) moments
            raw_xx = Sxx + np.outer(s, sx) + np.outer(sx, s) + n * np.outer(s, s)
            raw_xy = Sxy + s * sy + yshift * sx + n * s * yshift
            M, c = raw_xx / n, raw_xy / n
            yy = (Syy + 2 * yshift * sy + n * yshift ** 2) / n
        if sdy == 0.0 and fit_int:
            return np.zeros(d), float(my), [0.0], 0, None
        ystd = sdy if sdy > 0 else 1.0
        active = sdx > 0
        scale = np.where(active, sdx, 1.0)
        Ms = M / np.outer(scale, scale)
        cs = c / scale / ystd
        lam_eff = lam / ystd
        if self.getStandardization():
            p1, p2 = np.ones(d), np.ones(d)
        else:
            p1, p2 = 1.0 / scale, 1.0 / (scale * scale)
        idx = np.nonzero(active)[0]
        beta_s = np.zeros(d)
        hist, iters = [], 0
        stderr = None
        if len(idx):
            Ma, ca = Ms[np.ix_(idx, idx)], cs[idx]
            l1 = lam_eff * alpha * p1[idx]
            l2 = lam_eff * (1 - alpha) * p2[idx]
            if lam == 0.0 or alpha == 0.0:
                A = Ma + np.diag(l2)
                try:
                    # SPD: Cholesky (raises when not positive definite) + two triangular solves, in LAPACK
                    c_, low = _cho_factor(A)
                    b = _cho_solve((c_, low), ca)
                except np.linalg.LinAlgError:
                    b = np.linalg.lstsq(A, ca, rcond=None)[0]
                iters = 1
            else:
                b = np.zeros(len(idx))
                tol = max(self.getTol(), 1e-12)
                for it in range(max(self.getMaxIter(), 1) * 10):
                    mx_change = 0.0
                    for j in range(len(idx)):
                        r = ca[j] - Ma[j] @ b + Ma[j, j] * b[j]
                        nb = np.sign(r) * max(abs(r) - l1[j], 0.0) / (Ma[j, j] + l2[j])
                        mx_change = max(mx_change, abs(nb - b[j]))
                        b[j] = nb
                    iters = it + 1
                    obj = 0.5 * b @ Ma @ b - ca @ b + (l1 * np.abs(b)).sum() + 0.5 * (l2 * b * b).sum()
                    hist.append(float(obj + 0.5 * yy / (ystd * ystd)))
                    if mx_change < tol:
                        break
            beta_s[idx] = b
        coef = beta_s * ystd / scale
        coef[~active] = 0.0
        intercept = float(my - coef @ mx) if fit_int else 0.0
        if not hist:
            resid = yy / (ystd * ystd) - 2 * cs @ beta_s + beta_s @ Ms @ beta_s
            hist = [0.5 * float(resid)]
        if lam == 0.0 and fit_int and len(idx) == d:
            stderr = self._stderr_fn(coef, Cxx, Cxy, Cyy, n, d, mx)
        return coef, intercept, hist, iters, stderr

    def _refine(self, X, y, w, comm, G, d, shift, yshift, coef, intercept, steps: int = 3):
        """Iterative refinement of the closed-form solution on Double features (course scale): the normal
        equations square the design's condition number (the ML 03 one-hot Airbnb design: cond(X) ~4e6), so the
        Cholesky solution alone is good to ~cond(X)^2 eps ~1e-4.  Each step forms the exact gradient from the data
        -- g = sum w (x - mean) r with r = y - x.coef - b in fp64, one pass, all-reduced -- and solves the same
        system for the correction (corrected semi-normal equations): the coefficients converge to ~cond(X) eps,
        what a QR / SVD least-squares solve gives.  Only the closed-form case (intercept, L2 or no penalty, every
        feature varying) is refined; the other solvers are iterative already."""
        n = G[d, d]
        sx, sy = G[:d, d], G[d + 1, d]
        Cxx, Cyy = G[:d, :d] - np.outer(sx, sx) / n, G[d + 1, d + 1] - sy * sy / n
        sdx = np.sqrt(np.clip(np.diag(Cxx) / n, 0, None))
        sdy = math.sqrt(max(Cyy / n, 0.0))
        lam, alpha = self.getRegParam(), self.getElasticNetParam()
        if not (self.getFitIntercept() and sdy > 0.0 and (lam == 0.0 or alpha == 0.0) and bool((sdx > 0).all())):
            return coef, intercept
        A = Cxx.copy()
        if lam > 0.0:
            p2 = np.ones(d) if self.getStandardization() else 1.0 / (sdx * sdx)
            A += np.diag(n * (lam / sdy) * (1 - alpha) * p2 * sdx * sdx)
        try:
            cf = _cho_factor(A)
        except np.linalg.LinAlgError:
            return coef, intercept
        mx = (np.asarray(shift, np.float64) if shift is not None else 0.0) + sx / n
        pen = A - Cxx
        coef = np.asarray(coef, np.float64).copy()
        for _ in range(steps):
            cw = torch.tensor(coef, dtype=torch.float64, device=X.device)
            r = y - (X @ cw + intercept) if X.shape[0] else y
            if w is not None:
                r = r * w
            acc = torch.cat([X.T @ r, r.sum().reshape(1)]) if X.shape[0] else \
                torch.zeros(d + 1, dtype=torch.float64, device=X.device)
            comm.all_reduce(acc)
            a = acc.cpu().numpy()
            g = a[:d] - mx * a[d] - pen @ coef          # sum w (x - mean) r, less the ridge term
            delta = _cho_solve(cf, g)
            coef = coef + delta
            intercept = intercept + a[d] / n - float(mx @ delta)   # sum w r = 0 at the optimum
            if np.max(np.abs(delta)) <= 1e-15 * max(np.max(np.abs(coef)), 1e-300):
                break
        return coef, float(intercept)

    @staticmethod
    def _stderr_fn(coef, Cxx, Cxy, Cyy, n, d, mx):
        """Standard errors (unregularised normal-equation solution only), computed on first access: the d x d
        inverse cost ~1 ms of host BLAS per fit (half the fit time at 1e7 x 100 on MI355X) for a summary field
        most fits never read."""
        def stderr():
            try:
                sse = max(Cyy - 2 * coef @ Cxy + coef @ Cxx @ coef, 0.0)
                sigma2 = sse / max(n - d - 1, 1)
                inv = np.linalg.inv(Cxx)
                se_coef = np.sqrt(np.clip(np.diag(inv) * sigma2, 0, None))
                se_int = math.sqrt(max(sigma2 * (1.0 / n + mx @ inv @ mx), 0.0))
                return list(se_coef) + [se_int]
            except np.linalg.LinAlgError:
                return None
        return stderr

    def _solve_ridge(self, sdx, sdy, lam, alpha, d, n, mx, my, Cxx, Cxy, Cyy):
        """Fast path of _solve for the closed-form case (intercept, L2 or no penalty, every feature varying):
        the standardised system (D^-1 M D^-1 + L) b = D^-1 c / sd_y (M = Cxx / n, c = Cxy / n), coef =
        sd_y D^-1 b, has the same solution as (Cxx + n D L D) coef = Cxy -- one Cholesky of the unscaled
        covariance, no scaled copies (the general path's ~20 d x d numpy passes cost ~0.3 ms of host time per
        fit, a fifth of the fit at 1e7 x 100).  None when the system is not positive definite (the general
        path's least squares then)."""
        A = Cxx
        if lam > 0.0:
            p2 = np.ones(d) if self.getStandardization() else 1.0 / (sdx * sdx)
            A = Cxx + np.diag(n * (lam / sdy) * (1 - alpha) * p2 * sdx * sdx)
        try:
            coef = _cho_solve(_cho_factor(A), Cxy)
        except np.linalg.LinAlgError:
            return None
        intercept = float(my - coef @ mx)
        # the general path's objective history: 0.5 (yy - 2 c.coef + coef.M.coef) / sd_y^2, penalty not included
        obj = 0.5 * float(Cyy - 2 * Cxy @ coef + coef @ (Cxx @ coef)) / (n * sdy * sdy)
        stderr = self._stderr_fn(coef, Cxx, Cxy, Cyy, n, d, mx) if lam == 0.0 else None
        return coef, intercept, [obj], 1, stderr


class LinearRegressionModel(Model):
    _params = LinearRegression._params

    def __init__(self, coefficients=None, intercept=0.0):
        super().__init__()
        self._coef = np.asarray(coefficients if coefficients is not None else [], dtype=np.float64)
        self._intercept = float(intercept)
        self.summary = None

    @property
    def coefficients(self):
        return DenseVector(self._coef)

    @property
    def intercept(self):
        return self._intercept

    @property
    def numFeatures(self):
        return len(self._coef)

    @property
    def hasSummary(self):
        return self.summary is not None

    @property
    def scale(self):
        return 1.0

    def predict(self, features):
        x = features.toArray() if hasattr(features, "toArray") else np.asarray(features)
        return float(x @ self._coef + self._intercept)

    def _transform(self, dataset):
        fc, pc = self.getFeaturesCol(), self.getPredictionCol()
        require_vector(dataset, fc)
        coef = torch.tensor(self._coef, dtype=torch.float32)
        coef64 = torch.tensor(self._coef, dtype=torch.float64)
        icpt = self._intercept

        def fn(b, ctx):
            X = b.columns[fc].values
            if X.dtype == torch.float64:     # Double vectors: Spark's fp64 dot product
                p = X @ coef64.to(X.device) + icpt
            else:
                p = (X.float() @ coef.to(X.device)).double() + icpt if X.shape[0] else \
                    torch.zeros(0, dtype=torch.float64, device=X.device)
            return b.with_column(pc, ColumnData(p, T.DoubleType(), b.columns[fc].valid))
        return dataset._new(MapPlan(dataset._plan, f"LinearRegressionModel -> {pc}", fn))

    def evaluate(self, dataset):
        return _RegressionSummary(self.transform(dataset), self.getLabelCol(), self.getPredictionCol(),
                                  self.numFeatures)

    def _save_state(self):
        return {"intercept": self._intercept}, {"coefficients": torch.tensor(self._coef)}

    def _load_state(self, extra, tensors, stages):
        self._coef = tensors["coefficients"].numpy()
        self._intercept = float(extra["intercept"])
        self.summary = None

    def __repr__(self):
        return f"LinearRegressionModel: uid={self.uid}, numFeatures={self.numFeatures}"


# ================================================================ trees
_TREE = {
    "maxDepth": ("Maximum depth of the tree. (>= 0)", 5, TC.toInt),
    "maxBins": ("Max number of bins for discretizing continuous features. Must be >= 2 and >= number of "
                "categories for any categorical feature.", 32, TC.toInt),
    "minInstancesPerNode": ("Minimum number of instances each child must have after split.", 1, TC.toInt),
    "minWeightFractionPerNode": ("Minimum fraction of the weighted sample count that each child must have.",
                                 0.0, TC.toFloat),
    "minInfoGain": ("Minimum information gain for a split to be considered at a tree node.", 0.0, TC.toFloat),
    "maxMemoryInMB": ("Maximum memory in MB allocated to histogram aggregation.", 256, TC.toInt),
    "cacheNodeIds": ("If false, the algorithm will pass trees to executors to match instances with nodes.",
                     False, TC.toBoolean),
    "checkpointInterval": ("set checkpoint interval (>= 1) or disable checkpoint (-1).", 10, TC.toInt),
    "seed": ("random seed.", None, TC.toInt),
    "weightCol": ("weight column name.", None, TC.toString),
    "leafCol": ("Leaf indices column name.", "", TC.toString),
}
_RF = {
    "numTrees": ("Number of trees to train (>= 1).", 20, TC.toInt),
    "featureSubsetStrategy": ("The number of features to consider for splits at each tree node. Supported "
                              "options: 'auto', 'all', 'onethird', 'sqrt', 'log2', (0.0-1.0], [1-n].", "auto",
                              TC.toString),
    "subsamplingRate": ("Fraction of the training data used for learning each decision tree, in range (0, 1].",
                        1.0, TC.toFloat),
    "bootstrap": ("Whether bootstrap samples are used when building trees.", True, TC.toBoolean),
}


def resolve_subset(strategy: str, d: int, num_trees: int, classification: bool) -> Optional[int]:
    s = strategy.lower()
    if s == "auto":
        s = "all" if num_trees == 1 else ("sqrt" if classification else "onethird")
    if s == "all":
        return None
    if s == "sqrt":
        return max(1, int(math.ceil(math.sqrt(d))))
    if s == "log2":
        return max(1, int(math.ceil(math.log2(d))))
    if s == "onethird":
        return max(1, int(math.ceil(d / 3.0)))
    try:
        v = float(s)
    except ValueError:
        raise IllegalArgumentException(f"invalid featureSubsetStrategy {strategy}")
    if v.is_integer() and v >= 1 and "." not in s:
        return min(d, int(v))
    if 0 < v <= 1:
        return max(1, int(math.ceil(v * d)))
    raise IllegalArgumentException(f"invalid featureSubsetStrategy {strategy}")


def tree_fit_prepare(est, dataset, classification: bool, pre=None):
    """Common: device features/labels, categorical info, global row offset, binned data.

    pre(n_local, row_offset, seed, device, y): launched before the quantile sample is queued (the label's fp32
    copy and maximum, on a side stream); it may return a callable, run right before the binning is queued (the
    bootstrap draws: compute-bound, they overlap the memory-bound binning)."""
    fc, lc = est.getFeaturesCol(), est.getLabelCol()
    wc = est.getWeightCol() if est.hasParam("weightCol") else None
    require_vector(dataset, fc)
    session = dataset._session
    cols = [fc, lc] + ([wc] if wc else [])
    src = streamed_columns(dataset, fc, cols[1:])
    if src is not None:
        # out-of-core: X streamed chunk by chunk into the quantile sample and the bins, never resident
        X, cd, fmeta = src
        y = cd[lc].values.double()
        w = cd[wc].values.double() if wc else None
    else:
        b = local_batch(dataset, cols)
        fcol = b.columns[fc]
        fmeta = fcol.meta
        X = fcol.values.float()
        X = X if X.is_contiguous() else X.contiguous()
        y = b.columns[lc].values.double()
        w = b.columns[wc].values.double() if wc else None
    d = X.shape[1]
    cat = categorical_info(fmeta, d, fc)
    n = X.shape[0]
    n_global = global_count(session, n)
    off = global_offset(session, n)
    seed = est.getOrDefault("seed")
    if seed is None:
        seed = _default_seed(type(est))
    late = pre(n, off, seed, X.device, y) if pre is not None else None
    data = make_binned(session, X, cat, est.getMaxBins(), seed, off, n_global, before_binize=late)
    data.source_ref = weakref.ref(fcol.values) if src is None else None
    return session, data, y, w, seed, fmeta


def attach_fit_bins(forest: Forest, data) -> None:
    """Give a single-output forest the bins of its training tensor (``FitBins``): a transform of that same,
    unmodified tensor then predicts from the bins (REUSE_FIT_BINS; numeric features only)."""
    src = data.source_ref() if data.source_ref is not None else None
    if (_forest_mod.REUSE_FIT_BINS and src is not None and src.is_cuda and forest.K == 1 and not data.categorical
            and not data.missing_bin and data.bins is not None and data.bins.is_cuda):
        forest._fit_bins = FitBins(src, data.bins, data.thresholds, data.nthr, data.d, data.B)


def _num_classes(session, y: torch.Tensor, meta_label: Optional[dict]) -> int:
    if meta_label and meta_label.get("num_vals"):
        return int(meta_label["num_vals"])
    mx = torch.tensor([float(y.max()) if y.numel() else 0.0], dtype=torch.float64, device=session.comm.device)
    session.comm.all_reduce(mx, "max")
    return int(mx) + 1


class _TreeModelBase(Model):
    """Shared prediction + persistence for tree ensembles."""

    def __init__(self, forest: Optional[Forest] = None, numFeatures: int = 0, tree_weights=None):
        super().__init__()
        self._forest = forest
        self._numFeatures = numFeatures
        self._tree_w = np.asarray(tree_weights if tree_weights is not None else [], dtype=np.float64)

    @property
    def numFeatures(self):
        return self._numFeatures

    @property
    def featureImportances(self):
        imp = self._forest.feature_importances(self._numFeatures)
        nz = np.nonzero(imp)[0]
        return SparseVector(self._numFeatures, nz.tolist(), imp[nz].tolist())

    @property
    def getNumTrees(self):
        return len(self._forest.roots)

    @property
    def treeWeights(self):
        return list(self._tree_w)

    @property
    def totalNumNodes(self):
        return sum(len(self._forest.tree_nodes(t)) for t in range(len(self._forest.roots)))

    @property
    def numNodes(self):
        return self.totalNumNodes

    @property
    def depth(self):
        return int(self._forest.tree_depths().max()) if self._forest.roots else 0

    def toDebugString_tree(self, t, names=None):
        f = self._forest
        lines = []

        def rec(i, ind):
            pad = " " * ind
            if f.feat[i] < 0:
                v = f.value[i]
                lines.append(f"{pad}Predict: {float(v[0]) if len(v) == 1 else int(np.argmax(v)):g}")
                return
            fn = f"feature {f.feat[i]}"
            if f.is_cat[i]:
                cats = [c for c in range(256) if (int(f.catmask[i][c >> 5]) >> (c & 31)) & 1]
                lines.append(f"{pad}If ({fn} in {{{','.join(f'{c:.1f}' for c in cats)}}})")
                rec(f.left[i], ind + 1)
                lines.append(f"{pad}Else ({fn} not in {{{','.join(f'{c:.1f}' for c in cats)}}})")
            else:
                lines.append(f"{pad}If ({fn} <= {f.thr[i]})")
                rec(f.left[i], ind + 1)
                lines.append(f"{pad}Else ({fn} > {f.thr[i]})")
            rec(f.right[i], ind + 1)
        rec(f.roots[t], 1)
        return "\n".join(lines)

    @property
    def toDebugString(self):
        T_ = len(self._forest.roots)
        s = f"{type(self).__name__}: uid={self.uid}, depth={self.depth}, numNodes={self.totalNumNodes}, " \
            f"numFeatures={self._numFeatures}\n"
        if T_ == 1:
            return s + self.toDebugString_tree(0)
        return s + "\n".join(f"  Tree {t} (weight {self._tree_w[t] if t < len(self._tree_w) else 1.0}):\n" +
                             self.toDebugString_tree(t) for t in range(T_))

    def _save_state(self):
        return {"numFeatures": self._numFeatures, "K": self._forest.K}, dict(
            self._forest.state(), tree_w=torch.tensor(self._tree_w))

    def _load_state(self, extra, tensors, stages):
        self._forest = Forest.from_state(tensors)
        self._numFeatures = int(extra["numFeatures"])
        self._tree_w = tensors["tree_w"].numpy()

    def _leaf_col(self, b, out_cols):
        lc = self.getLeafCol() if self.hasParam("leafCol") else ""
        if lc:
            X = b.columns[self.getFeaturesCol()].values
            leaves = self._forest.predict_leaf_index(X).double().to(X.device)
            out_cols[lc] = ColumnData(leaves, T.VectorUDT())


class _TreeRegressorModel(_TreeModelBase):
    _base = 0.0

    def _transform(self, dataset):
        fc, pc = self.getFeaturesCol(), self.getPredictionCol()
        require_vector(dataset, fc)
        forest, tw, base = self._forest, self._tree_w, self._base

        from .inference import predictor_for
        predictor = predictor_for(self, "value", [base])  # forest uploaded once; recurring buffers graph-replayed

        def fn(b, ctx):
            X = b.columns[fc].values
            p = predictor(X, torch.float64)[:, 0] if X.shape[0] else \
                torch.zeros(0, dtype=torch.float64, device=X.device)
            out = {pc: ColumnData(p, T.DoubleType())}
            self._leaf_col(b, out)
            nb = b
            for k, v in out.items():
                nb = nb.with_column(k, v)
            return nb
        return dataset._new(MapPlan(dataset._plan, f"{type(self).__name__} -> {pc}", fn))

    def predict(self, features):
        x = torch.tensor(np.asarray(features.toArray() if hasattr(features, "toArray") else features),
                         dtype=torch.float32)[None, :]
        return float(self._forest.predict(x, self._tree_w, [self._base])[0, 0])

    def evaluate(self, dataset):
        return _RegressionSummary(self.transform(dataset), self.getLabelCol(), self.getPredictionCol(),
                                  self._numFeatures)


def _early_side_work(num_trees, bootstrap, rate, want_label_max=True, codes_ok=False):
    """(pre, early): ``pre`` for tree_fit_prepare queues the label's fp32 copy and max |label| on the side stream
    before the quantile sample, and returns the Poisson bootstrap draws (+ the largest weight) for
    tree_fit_prepare to queue on the side stream right before the binning; the first level reads the maxima
    without draining the queue.  ``early`` then holds "yf" (fp32 label) and "codes" (BootstrapCodes) or "w"
    (weights); call _join_early once the binning is queued."""
    early = {}

    def pre(n, off, seed_, dev, y_):
        if dev.type != "cuda":
            return None
        side = _side_stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        if want_label_max:
            early["yf"] = K.float_with_absmax(y_, stream=side)


        def draws():
            # queued right behind the quantile kernel, before the binning, on the MAIN stream (K.POISSON_STREAM
            # =side: the side stream).  Measured at 1e8 rows (profiles/r4/prologue_ab.md): beside the quantile sort
            # the draws kept its 1024-thread blocks off the CUs (2.1 ms for a 0.3 ms kernel); beside the binning --
            # itself ~60 % VALU-bound (6-step threshold search) -- they slowed it by more than their own 2.2 ms;
            # in series they cost exactly their 2.2 ms
            if bootstrap and num_trees > 1:
                if codes_ok and K.POISSON_CODES:
                    # the draws written straight as the engine's row codes + their max (no uint8 weights, no
                    # codes_init pass, no separate max reduction over T x n bytes); lazy: the trainer's level-0
                    # root histogram draws them itself when it can (K.POISSON_FUSED), else they run here on demand
                    with torch.cuda.stream(side if K.POISSON_STREAM == "side" else torch.cuda.current_stream(dev)):
                        early["codes"] = K.BootstrapCodes(num_trees, n, seed_, off, rate, dev,
                                                          lazy=K.POISSON_FUSED and K.POISSON_STREAM != "side")
                else:
                    early["w"] = _poisson_side(num_trees, n, seed_, off, rate, dev, join=False)
                    K.prefetch_max(early["w"], stream=side)
        return draws
    return pre, early


def _label_f32(early, y):
    """The fp32 label queued on the side stream (``early["yf"]``), else a cast of ``y`` (never both: a
    ``dict.get(k, y.float())`` default is evaluated eagerly -- a full extra cast of the label per fit, 0.27 ms at
    1e8 rows)."""
    yf = early.get("yf")
    return yf if yf is not None else y.float()


def _join_early(early, dev):
    for k in ("yf", "w"):
        if k in early:
            _join_side(early[k], dev)  # binning is queued: the trainer's first kernel waits for the side stream
    if "codes" in early:
        _join_side(early["codes"].codes, dev)


def _train_forest_regression(est, dataset, num_trees, subset, bootstrap, rate, impurity="variance"):
    pre, early = _early_side_work(num_trees, bootstrap, rate)
    session, data, y, w, seed, meta = tree_fit_prepare(est, dataset, classification=False, pre=pre)
    _join_early(early, data.bins.device)
    p = TreeParams(max_depth=est.getMaxDepth(), max_bins=est.getMaxBins(),
                   min_instances=float(est.getMinInstancesPerNode()), min_info_gain=est.getMinInfoGain(),
                   impurity=impurity, feature_subset=subset, bootstrap=bootstrap, subsampling_rate=rate, seed=seed)
    weights = early["w"] if "w" in early else _bag_weights(data, num_trees, bootstrap, rate, seed)
    if w is not None:
        weights = _combine_weights(weights, w, num_trees)
    trainer = ForestTrainer(session, data, p)
    forest = trainer.train(num_trees, {"v0": None, "v1": _label_f32(early, y)}, weights)
    attach_fit_bins(forest, data)
    return forest, data.d


_SIDE_STREAMS = {}


def _side_stream(dev):
    s = _SIDE_STREAMS.get(dev.index)
    if s is None:
        s = _SIDE_STREAMS[dev.index] = torch.cuda.Stream(device=dev)
    return s


def _poisson_side(T_, n, seed, row_offset, rate, dev, join: bool = True):
    """Compute-bound Philox Poisson draws on a side stream (they depend on nothing queued on the current one).
    join: the current stream waits for them before its next kernel (else call _join_side before using them)."""
    side = _side_stream(dev)
    with torch.cuda.stream(side):
        wts = K.poisson_weights(T_, n, seed, row_offset, rate, device=dev)
    if join:
        _join_side(wts, dev)
    return wts


def _join_side(wts, dev):
    main = torch.cuda.current_stream(dev)
    main.wait_stream(_side_stream(dev))
    wts.record_stream(main)


def _bag_weights(data, T_, bootstrap, rate, seed):
    n = data.n_local
    dev = data.bins.device
    if bootstrap and T_ > 1:
        if dev.type == "cuda":
            return _poisson_side(T_, n, seed, data.row_offset, rate, dev)
        return K.poisson_weights(T_, n, seed, data.row_offset, rate, device=dev)
    if rate < 1.0:
        u = torch.stack([K.uniform(n, seed, data.row_offset, 0x200 + t, device=dev) for t in range(T_)])
        return (u < rate).to(torch.uint8)
    return None


def _combine_weights(bag, w, T_):
    # instance weights must be small non-negative integers for the uint8 weight path
    wi = torch.round(w).clamp(0, 255).to(torch.uint8)
    if bag is None:
        return wi[None, :].expand(T_, -1).contiguous()
    return (bag.to(torch.int32) * wi.to(torch.int32)[None, :]).clamp(0, 255).to(torch.uint8)


class DecisionTreeRegressor(Estimator):
    _params = dict(_PRED, **_TREE, **{
        "impurity": ("Criterion used for information gain calculation. Supported: variance", "variance",
                     TC.toString),
        "varianceCol": ("column name for the biased sample variance of prediction", None, TC.toString),
    })

    def __init__(self, **kwargs):
        super().__init__()
        keyword_init(self, kwargs)

    def _fit(self, dataset):
        forest, d = _train_forest_regression(self, dataset, 1, None, False, 1.0)
        return DecisionTreeRegressionModel(forest, d, [1.0])


class DecisionTreeRegressionModel(_TreeRegressorModel):
    _params = DecisionTreeRegressor._params


class RandomForestRegressor(Estimator):
    """Bagged regression trees (ML 07:41; north-star benchmark model)."""
    _params = dict(_PRED, **_TREE, **_RF, **{
        "impurity": ("Criterion used for information gain calculation. Supported: variance", "variance",
                     TC.toString),
    })

    def __init__(self, **kwargs):
        super().__init__()
        keyword_init(self, kwargs)

    def _fit(self, dataset):
        T_ = self.getNumTrees()
        forest, dd = _train_rf_reg(self, dataset, T_)
        return RandomForestRegressionModel(forest, dd, np.full(T_, 1.0 / T_))


def _train_rf_reg(est, dataset, T_):
    pre, early = _early_side_work(T_, est.getBootstrap(), est.getSubsamplingRate(),
                                  codes_ok=not (est.hasParam("weightCol") and est.getWeightCol()))
    session, data, y, w, seed, meta = tree_fit_prepare(est, dataset, classification=False, pre=pre)
    _join_early(early, data.bins.device)
    subset = resolve_subset(est.getFeatureSubsetStrategy(), data.d, T_, False)
    p = TreeParams(max_depth=est.getMaxDepth(), max_bins=est.getMaxBins(),
                   min_instances=float(est.getMinInstancesPerNode()), min_info_gain=est.getMinInfoGain(),
                   impurity="variance", feature_subset=subset, bootstrap=est.getBootstrap(),
                   subsampling_rate=est.getSubsamplingRate(), seed=seed)
    bc = early.get("codes")
    if bc is not None:
        weights = None
    else:
        weights = early["w"] if "w" in early else \
            _bag_weights(data, T_, est.getBootstrap(), est.getSubsamplingRate(), seed)
    if w is not None:
        weights = _combine_weights(bc.weights() if bc is not None else weights, w, T_)
        bc = None
    forest = ForestTrainer(session, data, p).train(T_, {"v0": None, "v1": _label_f32(early, y)}, weights,
                                                   codes_pre=bc)
    attach_fit_bins(forest, data)
    return forest, data.d


class RandomForestRegressionModel(_TreeRegressorModel):
    _params = RandomForestRegressor._params

    @property
    def trees(self):
        out = []
        for t in range(len(self._forest.roots)):
            f = Forest(self._forest.K)
            sub = _subforest(self._forest, t)
            out.append(DecisionTreeRegressionModel(sub, self._numFeatures, [1.0]))
        return out


def _subforest(forest: Forest, t: int) -> Forest:
    idx = forest.tree_nodes(t)
    pos = {g: j for j, g in enumerate(idx)}
    f = Forest(forest.K)
    for g in idx:
        j = f.add(forest.value[g], forest.weight[g], forest.depth[g], forest.impurity[g])
        f.feat[j], f.thr[j], f.bin[j] = forest.feat[g], forest.thr[g], forest.bin[g]
        f.is_cat[j], f.catmask[j], f.gain[j] = forest.is_cat[g], forest.catmask[g], forest.gain[g]
    for g in idx:
        if forest.feat[g] >= 0:
            f.left[pos[g]], f.right[pos[g]] = pos[forest.left[g]], pos[forest.right[g]]
    f.roots = [0]
    return f


# ================================================================== GBT
_GBT = {
    "maxIter": ("max number of iterations (>= 0)", 20, TC.toInt),
    "stepSize": ("Step size (a.k.a. learning rate) in interval (0, 1] for shrinking the contribution of each "
                 "estimator.", 0.1, TC.toFloat),
    "subsamplingRate": ("Fraction of the training data used for learning each decision tree.", 1.0, TC.toFloat),
    "featureSubsetStrategy": ("The number of features to consider for splits at each tree node.", "all",
                              TC.toString),
    "validationIndicatorCol": ("name of the column that indicates whether each row is for training or for "
                               "validation.", None, TC.toString),
    "validationTol": ("Threshold for stopping early when fit with validation is used.", 0.01, TC.toFloat),
    "impurity": ("Criterion used for information gain calculation: variance", "variance", TC.toString),
}


def boost(session, data, y_target_fn, grad_fn, T_rounds, est, seed, init_margin, first_weight_one=True):
    """Generic gradient boosting on the shared binned data (variance-impurity trees on pseudo-residuals)."""
    dev = data.bins.device
    n = data.n_local
    subset = resolve_subset(est.getFeatureSubsetStrategy(), data.d, 1, False)
    p = TreeParams(max_depth=est.getMaxDepth(), max_bins=est.getMaxBins(),
                   min_instances=float(est.getMinInstancesPerNode()), min_info_gain=est.getMinInfoGain(),
                   impurity="variance", feature_subset=subset, seed=seed)
    trainer = ForestTrainer(session, data, p)
    forest = Forest(1)
    F = torch.full((n,), float(init_margin), dtype=torch.float32, device=dev)
    weights = []
    # checkpointInterval + SparkContext.setCheckpointDir: resume from the last saved round
    from .tree.checkpoint import RoundCheckpointer
    ck = RoundCheckpointer(session, est, data,
                           est.getCheckpointInterval() if est.hasParam("checkpointInterval") else None,
                           labels=y_target_fn(F))
    start = 0
    resumed = ck.load()
    if resumed is not None:
        start, forest, Fm, extra = resumed
        F = Fm.to(dev)
        weights = list(extra["weights"])
    for m in range(start, T_rounds):
        target = y_target_fn(F) if (m == 0 and first_weight_one) else grad_fn(F)
        bag = _bag_weights(data, 1, False, est.getSubsamplingRate(), seed + m)
        trainer.p.seed = seed + m
        trainer.train(1, {"v0": None, "v1": target.float()}, bag, forest)
        wgt = 1.0 if (m == 0 and first_weight_one) else est.getStepSize()
        nodes, vals, masks = forest.binned_arrays(dev, m)
        K.predict_binned_add(data.bins, nodes, 0, vals, masks, wgt, F)
        weights.append(wgt)
        ck.maybe_save(m + 1, forest, F, {"weights": weights})
    ck.finish()
    return forest, np.asarray(weights)


class GBTRegressor(Estimator):
    _params = dict(_PRED, **_TREE, **_GBT, **{
        "lossType": ("Loss function which GBT tries to minimize: squared, absolute", "squared", TC.toString),
    })

    def __init__(self, **kwargs):
        super().__init__()
        keyword_init(self, kwargs)

    def _fit(self, dataset):
        session, data, y, w, seed, meta = tree_fit_prepare(self, dataset, classification=False)
        yf = y.float()
        loss = self.getLossType()
        if loss == "squared":
            grad = lambda F: yf - F  # noqa: E731
        elif loss == "absolute":
            grad = lambda F: torch.sign(yf - F)  # noqa: E731
        else:
            raise IllegalArgumentException(f"unsupported lossType {loss}")
        forest, tw = boost(session, data, lambda F: yf, grad, self.getMaxIter(), self, seed, 0.0)
        return GBTRegressionModel(forest, data.d, tw)


class GBTRegressionModel(_TreeRegressorModel):
    _params = GBTRegressor._params

    @property
    def trees(self):
        return [DecisionTreeRegressionModel(_subforest(self._forest, t), self._numFeatures, [1.0])
                for t in range(len(self._forest.roots))]


class IsotonicRegression(Estimator):
    """Pool-adjacent-violators on the globally sorted (feature, label) pairs."""
    _params = dict(_PRED, **{
        "isotonic": ("whether the output sequence should be isotonic/increasing", True, TC.toBoolean),
        "featureIndex": ("index of the feature if featuresCol is a vector column", 0, TC.toInt),
        "weightCol": ("weight column name", None, TC.toString),
    })

    def __init__(self, **kwargs):
        super().__init__()
        keyword_init(self, kwargs)

    def _fit(self, dataset):
        pdf = dataset.select(self.getFeaturesCol(), self.getLabelCol()).toPandas()
        x = np.array([v[self.getFeatureIndex()] if hasattr(v, "toArray") else v
                      for v in pdf[self.getFeaturesCol()]], dtype=np.float64)
        yv = pdf[self.getLabelCol()].to_numpy(np.float64)
        sign = 1.0 if self.getIsotonic() else -1.0
        o = np.argsort(x, kind="stable")
        xs, ys = x[o], sign * yv[o]
        vals, wts, xs_b = [], [], []
        for xi, yi in zip(xs, ys):
            vals.append(yi)
            wts.append(1.0)
            xs_b.append([xi, xi])
            while len(vals) > 1 and vals[-2] > vals[-1]:
                v = (vals[-2] * wts[-2] + vals[-1] * wts[-1]) / (wts[-2] + wts[-1])
                wts[-2] += wts[-1]
                vals[-2] = v
                xs_b[-2][1] = xs_b[-1][1]
                vals.pop(); wts.pop(); xs_b.pop()
        bnd, pred = [], []
        for (a, b), v in zip(xs_b, vals):
            bnd += [a, b] if a != b else [a]
            pred += [sign * v] * (2 if a != b else 1)
        return IsotonicRegressionModel(np.array(bnd), np.array(pred))


class IsotonicRegressionModel(Model):
    _params = IsotonicRegression._params

    def __init__(self, boundaries=None, predictions=None):
        super().__init__()
        self._b = np.asarray(boundaries if boundaries is not None else [])
        self._p = np.asarray(predictions if predictions is not None else [])

    @property
    def boundaries(self):
        return DenseVector(self._b)

    @property
    def predictions(self):
        return DenseVector(self._p)

    def _transform(self, dataset):
        fc, pc, fi = self.getFeaturesCol(), self.getPredictionCol(), self.getFeatureIndex()
        bt, pt = torch.tensor(self._b), torch.tensor(self._p)

        def fn(b, ctx):
            v = b.columns[fc].values
            x = (v[:, fi] if v.dim() == 2 else v).double()
            out = torch.from_numpy(np.interp(x.cpu().numpy(), bt.numpy(), pt.numpy())).to(x.device)
            return b.with_column(pc, ColumnData(out, T.DoubleType()))
        return dataset._new(MapPlan(dataset._plan, "IsotonicRegressionModel", fn))

    def _save_state(self):
        return {}, {"b": torch.tensor(self._b), "p": torch.tensor(self._p)}

    def _load_state(self, extra, tensors, stages):
        self._b, self._p = tensors["b"].numpy(), tensors["p"].numpy()
