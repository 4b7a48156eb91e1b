"""ML vectors (``pyspark.ml.linalg`` surface).

On device a vector column is a dense float32 ``[n, d]`` matrix; these host
classes exist for ``collect()`` results, model coefficients and
``featureImportances`` (a SparseVector, ML 06 - Decision Trees.py:147-153).
"""
from __future__ import annotations

import numpy as np


class Vector:
    def toArray(self) -> np.ndarray:  # pragma: no cover - abstract
        raise NotImplementedError

    def __len__(self):
        return self.size

    def __iter__(self):
        return iter(self.toArray())

    def __getitem__(self, i):
        return self.toArray()[i]

    def dot(self, other):
        o = other.toArray() if hasattr(other, "toArray") else np.asarray(other)
        return float(np.dot(self.toArray(), o))

    def norm(self, p):
        return float(np.linalg.norm(self.toArray(), p))

    def __array__(self, dtype=None, copy=None):
        a = self.toArray()
        return a.astype(dtype) if dtype is not None else a


class DenseVector(Vector):
    def __init__(self, values):
        self.values = np.asarray(values, dtype=np.float64).reshape(-1)

    @property
    def size(self):
        return len(self.values)

    def toArray(self):
        return self.values

    def numNonzeros(self):
        return int(np.count_nonzero(self.values))

    def __eq__(self, other):
        return isinstance(other, Vector) and np.array_equal(self.toArray(), other.toArray())

    def __hash__(self):
        return hash(tuple(self.values.tolist()))

    def __repr__(self):
        return "DenseVector([" + ", ".join(repr(float(v)) for v in self.values) + "])"

    def __str__(self):
        return "[" + ",".join(str(float(v)) for v in self.values) + "]"

    def __add__(self, o):
        return DenseVector(self.values + np.asarray(o))

    def __sub__(self, o):
        return DenseVector(self.values - np.asarray(o))

    def __mul__(self, o):
        return DenseVector(self.values * np.asarray(o))


class SparseVector(Vector):
    def __init__(self, size, *args):
        self.size = int(size)
        if len(args) == 1:
            a = args[0]
            if isinstance(a, dict):
                items = sorted(a.items())
            else:
                items = sorted(a)
            self.indices = np.array([i for i, _ in items], dtype=np.int32)
            self.values = np.array([v for _, v in items], dtype=np.float64)
        else:
            self.indices = np.asarray(args[0], dtype=np.int32)
            self.values = np.asarray(args[1], dtype=np.float64)

    def toArray(self):
        a = np.zeros(self.size)
        a[self.indices] = self.values
        return a

    def numNonzeros(self):
        return int(np.count_nonzero(self.values))

    def __eq__(self, other):
        return isinstance(other, Vector) and np.array_equal(self.toArray(), other.toArray())

    def __hash__(self):
        return hash((self.size, tuple(self.indices.tolist())))

    def __repr__(self):
        return f"SparseVector({self.size}, {{" + ", ".join(
            f"{int(i)}: {float(v):.4f}" for i, v in zip(self.indices, self.values)) + "})"

    __str__ = __repr__


class Vectors:
    @staticmethod
    def dense(*values):
        if len(values) == 1 and not isinstance(values[0], (int, float)):
            return DenseVector(values[0])
        return DenseVector(values)

    @staticmethod
    def sparse(size, *args):
        return SparseVector(size, *args)

    @staticmethod
    def zeros(size):
        return DenseVector(np.zeros(size))

    @staticmethod
    def norm(v, p):
        return v.norm(p)

    @staticmethod
    def squared_distance(a, b):
        d = a.toArray() - b.toArray()
        return float(d @ d)


class DenseMatrix:
    def __init__(self, numRows, numCols, values, isTransposed=False):
        self.numRows, self.numCols = numRows, numCols
        v = np.asarray(values, dtype=np.float64)
        self.values = v
        self._a = v.reshape(numRows, numCols) if isTransposed else v.reshape(numCols, numRows).T

    def toArray(self):
        return self._a

    def __repr__(self):
        return f"DenseMatrix({self.numRows}, {self.numCols}, ...)"


class Matrices:
    @staticmethod
    def dense(numRows, numCols, values):
        return DenseMatrix(numRows, numCols, values)


def to_dense_vector(x) -> DenseVector:
    if isinstance(x, Vector):
        return DenseVector(x.toArray())
    return DenseVector(np.asarray(x))
