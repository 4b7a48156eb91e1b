"""``pyspark.ml.stat``: Correlation and Summarizer over device feature matrices."""
import numpy as np
import pandas as pd
import torch

from ..models.linalg import DenseMatrix, DenseVector
from ..ops import kernels as K


class Correlation:
    @staticmethod
    def corr(dataset, column, method="pearson"):
        from ..models.util import local_xyw
        X, _, _ = local_xyw(dataset, column)
        if method == "spearman":
            X = torch.argsort(torch.argsort(X, 0), 0).float()
        d = X.shape[1]
        G = K.gram(X) if X.shape[0] else torch.zeros((d + 2, d + 2), dtype=torch.float64, device=X.device)
        dataset._session.comm.all_reduce(G)
        n = float(G[d, d])
        s = G[:d, d]
        C = (G[:d, :d] - torch.outer(s, s) / n)
        sd = torch.sqrt(torch.diagonal(C).clamp_min(1e-300))
        R = (C / torch.outer(sd, sd)).cpu().numpy()
        return _MatrixFrame(R, method, column)


class _MatrixFrame:
    """Tiny stand-in for the 1x1 DataFrame of a Matrix (head()[0] is the matrix)."""

    def __init__(self, R, method, column):
        self._m = DenseMatrix(R.shape[0], R.shape[1], R.T.reshape(-1))
        self.columns = [f"{method}({column})"]

    def head(self):
        return [self._m]

    def collect(self):
        return [[self._m]]


class Summarizer:
    @staticmethod
    def metrics(*names):
        return _SummaryBuilder(names)

    @staticmethod
    def mean(col):
        return _SummaryBuilder(["mean"]), col


class _SummaryBuilder:
    def __init__(self, names):
        self.names = list(names)

    def summary(self, col):
        return (self, col)
