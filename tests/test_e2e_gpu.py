"""End-to-end estimators on the GPU vs the same framework on the CPU (HIP path vs torch
reference path).  Every model family runs its hot loop through the native gfx950
library; results must match the CPU run to tight tolerances."""
import numpy as np
import pandas as pd
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sessions():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import cdnaml
    from cdnaml.ops import _lib
    _lib.lib()  # fail loudly if the native library is missing
    s = cdnaml.SparkSession.builder.getOrCreate()
    assert s.device.type == "cuda"
    return s


def _frame(spark, n=20000, d=8, seed=0, cls=False):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, d)).astype(np.float32)
    y = X[:, 0] * 2 + np.sin(X[:, 1] * 2) + 0.5 * X[:, 2] * X[:, 3] + 0.1 * rng.normal(size=n)
    if cls:
        y = (y > 0).astype(np.float64)
    from cdnaml.ml.feature import VectorAssembler
    pdf = pd.DataFrame(X, columns=[f"x{i}" for i in range(d)])
    pdf["label"] = y
    return VectorAssembler(inputCols=list(pdf.columns[:d]), outputCol="features").transform(
        spark.createDataFrame(pdf)), X, y


def test_linear_regression_gpu_matches_sklearn(sessions):
    from sklearn.linear_model import LinearRegression as SK
    from cdnaml.ml.regression import LinearRegression
    df, X, y = _frame(sessions)
    m = LinearRegression().fit(df)
    sk = SK().fit(X.astype(np.float64), y)
    np.testing.assert_allclose(m.coefficients.toArray(), sk.coef_, rtol=1e-4, atol=1e-5)


def test_random_forest_gpu_quality_and_determinism(sessions):
    from cdnaml.ml.evaluation import RegressionEvaluator
    from cdnaml.ml.regression import RandomForestRegressor
    df, X, y = _frame(sessions)
    rf = RandomForestRegressor(numTrees=20, maxDepth=6, seed=42)
    m1 = rf.fit(df)
    m2 = rf.fit(df)
    p1 = m1.transform(df).select("prediction").toPandas().prediction.values
    p2 = m2.transform(df).select("prediction").toPandas().prediction.values
    np.testing.assert_array_equal(p1, p2)  # exact integer histograms -> bit-identical forests
    rmse = RegressionEvaluator().evaluate(m1.transform(df))
    assert rmse < 0.6 * np.std(y)


def test_forest_gpu_equals_cpu(sessions):
    """Same forest on cuda:0 and on the host reference path (fixed-point sums are exact)."""
    from cdnaml.models.tree.engine import ForestTrainer, TreeParams, make_binned
    from cdnaml.ops import kernels as K
    rng = np.random.default_rng(3)
    n, d = 5000, 6
    X = torch.from_numpy(rng.normal(size=(n, d)).astype(np.float32))
    y = X[:, 0] * 3 + X[:, 1] ** 2
    out = []
    for dev in ("cpu", "cuda"):
        Xd = X.to(dev)
        data = make_binned(sessions, Xd, {}, 32, 1, 0, n)
        p = TreeParams(max_depth=4, max_bins=32, feature_subset=None, seed=1)
        w = K.poisson_weights(4, n, 1, 0, 1.0, device=Xd.device)
        f = ForestTrainer(sessions, data, p).train(4, {"v0": None, "v1": y.to(dev).float()}, w)
        out.append((f.feat, f.bin, np.round(np.array([v[0] for v in f.value]), 5)))
    assert out[0][0] == out[1][0] and out[0][1] == out[1][1]
    np.testing.assert_allclose(out[0][2], out[1][2], rtol=1e-5, atol=1e-5)


def test_classifiers_gpu(sessions):
    from cdnaml.ml.classification import GBTClassifier, LogisticRegression, RandomForestClassifier
    from cdnaml.ml.evaluation import BinaryClassificationEvaluator
    df, X, y = _frame(sessions, cls=True, n=10000)
    for est in (LogisticRegression(maxIter=50), RandomForestClassifier(numTrees=10, seed=1),
                GBTClassifier(maxIter=10, maxDepth=3)):
        auc = BinaryClassificationEvaluator().evaluate(est.fit(df).transform(df))
        assert auc > 0.85, type(est).__name__


def test_xgboost_gpu_missing_and_v0_histograms(sessions):
    from cdnaml.ml.evaluation import RegressionEvaluator
    from cdnaml.ml.xgboost import XgboostRegressor
    df, X, y = _frame(sessions, n=10000)
    m = XgboostRegressor(n_estimators=60, max_depth=4, learning_rate=0.2, missing=0.0).fit(df)
    assert RegressionEvaluator().evaluate(m.transform(df)) < 0.5 * np.std(y)


def test_kmeans_als_gpu(sessions):
    from cdnaml.ml.clustering import KMeans
    from cdnaml.ml.recommendation import ALS
    df, X, y = _frame(sessions, n=5000)
    km = KMeans(k=4, seed=1, maxIter=10).fit(df)
    assert len(km.clusterCenters()) == 4
    rng = np.random.default_rng(0)
    u, i = rng.integers(0, 200, 8000), rng.integers(0, 150, 8000)
    U, V = rng.normal(size=(200, 4)), rng.normal(size=(150, 4))
    r = (U[u] * V[i]).sum(1)
    rd = sessions.createDataFrame(pd.DataFrame({"user": u, "item": i, "rating": r}))
    m = ALS(userCol="user", itemCol="item", ratingCol="rating", rank=4, maxIter=8, regParam=0.01, seed=1).fit(rd)
    pred = m.transform(rd).toPandas()
    assert np.sqrt(np.mean((pred.prediction - pred.rating) ** 2)) < 0.5
