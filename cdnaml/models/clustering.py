"""Clustering: distributed k-means.

Each Lloyd iteration = one pass of the K10 ``kmeans_step`` HIP kernel
(nearest-centre assignment + LDS-privatised per-centre sums) and one RCCL
all-reduce of k*(d+1) doubles — the map → reduce → communicate pattern of
MLE 02 - K-Means.py:178-204.  ``maxIter=0`` returns the initial centres
(MLE 02:46-68).  Initialisation: k-means++ over a global sample
("k-means||" default) or random points, both seeded.
"""
from __future__ import annotations

import numpy as np
import torch

from ..ops import kernels as K
from ..sql import types as T
from ..sql.batch import ColumnData
from ..sql.dataframe import MapPlan
from .base import Estimator, Model
from .param import NO_DEFAULT, TypeConverters as TC, keyword_init
from .regression import _default_seed
from .util import global_count, global_offset, local_xyw, require_vector


class KMeans(Estimator):
    _params = {
        "featuresCol": ("features column name", "features", TC.toString),
        "predictionCol": ("prediction column name", "prediction", TC.toString),
        "k": ("The number of clusters to create. Must be > 1.", 2, TC.toInt),
        "initMode": ("The initialization algorithm: 'random' or 'k-means||'", "k-means||", TC.toString),
        "initSteps": ("The number of steps for k-means|| initialization mode. Must be > 0.", 2, TC.toInt),
        "tol": ("the convergence tolerance for iterative algorithms (>= 0)", 1e-4, TC.toFloat),
        "maxIter": ("max number of iterations (>= 0)", 20, TC.toInt),
        "seed": ("random seed", None, TC.toInt),
        "distanceMeasure": ("'euclidean' or 'cosine'", "euclidean", TC.toString),
        "weightCol": ("weight column name", None, TC.toString),
    }

    def __init__(self, **kwargs):
        super().__init__()
        keyword_init(self, kwargs)

    def _init_centres(self, session, X, k, seed):
        comm = session.comm
        n = X.shape[0]
        ng = global_count(session, n)
        off = global_offset(session, n)
        target = min(ng, max(20 * k, 10000))
        frac = min(1.0, target / max(ng, 1))
        u = K.uniform(n, seed, off, 21, device=X.device)
        samp = X[u < frac] if frac < 1 else X
        if comm.distributed:
            samp = torch.cat(comm.all_gather_varlen(samp.contiguous()))
        S = samp.double().cpu().numpy()
        rng = np.random.default_rng(seed)
        if len(S) == 0:
            return np.zeros((k, X.shape[1]))
        if self.getInitMode() == "random":
            idx = rng.choice(len(S), size=min(k, len(S)), replace=False)
            C = S[idx]
        else:  # k-means++ on the global sample (deterministic given seed)
            C = [S[rng.integers(len(S))]]
            d2 = ((S - C[0]) ** 2).sum(1)
            for _ in range(1, k):
                p = d2 / d2.sum() if d2.sum() > 0 else np.full(len(S), 1.0 / len(S))
                C.append(S[rng.choice(len(S), p=p)])
                d2 = np.minimum(d2, ((S - C[-1]) ** 2).sum(1))
            C = np.array(C)
        if len(C) < k:
            C = np.vstack([C, np.repeat(C[-1:], k - len(C), 0)])
        return C

    def _fit(self, dataset):
        fc = self.getFeaturesCol()
        X, _, w = local_xyw(dataset, fc, None, self.getWeightCol(), keep_f64=True)
        session = dataset._session
        comm = session.comm
        seed = self.getSeed() if self.getSeed() is not None else _default_seed(type(self))
        k = self.getK()
        cosine = self.getDistanceMeasure() == "cosine"
        if cosine:
            X = X / torch.linalg.vector_norm(X, dim=1, keepdim=True).clamp_min(1e-30)
        C = self._init_centres(session, X, k, seed)
        cost = float("nan")
        it = 0
        for it in range(self.getMaxIter()):
            Ct = torch.tensor(C, dtype=X.dtype, device=X.device)
            _, sums, counts, c = K.kmeans_step(X, Ct)
            acc = torch.cat([sums.reshape(-1), counts, c.reshape(1)])
            comm.all_reduce(acc)
            a = acc.cpu().numpy()
            S = a[: k * X.shape[1]].reshape(k, -1)
            N = a[k * X.shape[1]: k * X.shape[1] + k]
            newC = np.where(N[:, None] > 0, S / np.maximum(N, 1)[:, None], C)
            if cosine:
                newC = newC / np.maximum(np.linalg.norm(newC, axis=1, keepdims=True), 1e-30)
            moved = np.sqrt(((newC - C) ** 2).sum(1)).max()
            C = newC
            if moved <= self.getTol():
                it += 1
                break
        # final cost / sizes with the final centres
        Ct = torch.tensor(C, dtype=X.dtype, device=X.device)
        assign, _, counts, c = K.kmeans_step(X, Ct)
        acc = torch.cat([counts, c.reshape(1)])
        comm.all_reduce(acc)
        a = acc.cpu().numpy()
        model = KMeansModel(C)
        model._post_fit(self)
        model.summary = KMeansSummary(model, dataset, a[:k].astype(np.int64).tolist(), float(a[k]),
                                      self.getMaxIter() if self.getMaxIter() == 0 else it)
        return model


class KMeansSummary:
    def __init__(self, model, dataset, sizes, cost, iters):
        self._model = model
        self._dataset = dataset
        self.clusterSizes = sizes
        self.trainingCost = cost
        self.numIter = iters
        self.k = len(sizes)
        self.featuresCol = model.getFeaturesCol()
        self.predictionCol = model.getPredictionCol()

    @property
    def predictions(self):
        return self._model.transform(self._dataset)

    @property
    def cluster(self):
        return self.predictions.select(self.predictionCol)


class KMeansModel(Model):
    _params = KMeans._params

    def __init__(self, centers=None):
        super().__init__()
        self._C = np.asarray(centers if centers is not None else np.zeros((0, 0)), dtype=np.float64)
        self.summary = None

    def clusterCenters(self):
        return [c.copy() for c in self._C]

    @property
    def hasSummary(self):
        return self.summary is not None

    def predict(self, features):
        x = np.asarray(features.toArray() if hasattr(features, "toArray") else features)
        return int(np.argmin(((self._C - x) ** 2).sum(1)))

    def computeCost(self, dataset):
        X, _, _ = local_xyw(dataset, self.getFeaturesCol(), keep_f64=True)
        _, _, _, c = K.kmeans_step(X, torch.tensor(self._C, dtype=X.dtype, device=X.device), with_sums=False)
        t = torch.tensor([float(c)], dtype=torch.float64, device=dataset._session.comm.device)
        dataset._session.comm.all_reduce(t)
        return float(t)

    def _transform(self, dataset):
        fc, pc = self.getFeaturesCol(), self.getPredictionCol()
        require_vector(dataset, fc)
        Cd = torch.tensor(self._C, dtype=torch.float64)
        cosine = self.getDistanceMeasure() == "cosine"

        def fn(b, ctx):
            X = b.columns[fc].values
            X = X if X.dtype == torch.float64 else X.float()   # Double vectors: fp64 distances (kernel <double>)
            if cosine:
                X = X / torch.linalg.vector_norm(X, dim=1, keepdim=True).clamp_min(1e-30)
            if X.shape[0] == 0:
                a = torch.zeros(0, dtype=torch.int32, device=X.device)
            else:
                a, _, _, _ = K.kmeans_step(X, Cd.to(X.device, X.dtype), with_sums=False)
            return b.with_column(pc, ColumnData(a.to(torch.int32), T.IntegerType()))
        return dataset._new(MapPlan(dataset._plan, "KMeansModel", fn))

    def _save_state(self):
        return {}, {"centers": torch.tensor(self._C)}

    def _load_state(self, extra, tensors, stages):
        self._C = tensors["centers"].numpy()
        self.summary = None


class BisectingKMeans(KMeans):
    """Divisive k-means: repeatedly split the largest cluster with 2-means."""
    _params = dict(KMeans._params, minDivisibleClusterSize=("min points in a divisible cluster", 1.0, TC.toFloat))

    def _fit(self, dataset):
        fc = self.getFeaturesCol()
        X, _, _ = local_xyw(dataset, fc, keep_f64=True)
        session = dataset._session
        comm = session.comm
        seed = self.getSeed() if self.getSeed() is not None else _default_seed(type(self))
        centers = [None]
        mean = X.double().sum(0)
        cnt = torch.tensor([float(X.shape[0])], dtype=torch.float64, device=X.device)
        comm.all_reduce_many([mean, cnt])
        centers = [(mean / cnt).cpu().numpy()]
        rng = np.random.default_rng(seed)
        while len(centers) < self.getK():
            C = np.array(centers)
            assign, _, counts, _ = K.kmeans_step(X, torch.tensor(C, dtype=X.dtype, device=X.device))
            comm.all_reduce(counts)
            big = int(torch.argmax(counts))
            sub = X[assign.long() == big]
            base = centers[big]
            jitter = rng.normal(scale=1e-3, size=base.shape) * (np.abs(base) + 1)
            pair = np.stack([base + jitter, base - jitter])
            for _ in range(self.getMaxIter()):
                _, s2, c2, _ = K.kmeans_step(sub, torch.tensor(pair, dtype=X.dtype, device=X.device))
                acc = torch.cat([s2.reshape(-1), c2])
                comm.all_reduce(acc)
                a = acc.cpu().numpy()
                S2, N2 = a[: 2 * X.shape[1]].reshape(2, -1), a[2 * X.shape[1]:]
                newp = np.where(N2[:, None] > 0, S2 / np.maximum(N2, 1)[:, None], pair)
                if np.abs(newp - pair).max() < self.getTol():
                    pair = newp
                    break
                pair = newp
            centers = centers[:big] + [pair[0], pair[1]] + centers[big + 1:]
        model = KMeansModel(np.array(centers))
        model._post_fit(self)
        return model
