"""Out-of-core fits: RandomForest / XGBoost / LinearRegression ``fit`` on a
streamed frame (``createDataFrameFromChunks``: pinned double buffers + copy stream on the GPU) never materialise
the feature matrix -- one pass collects the labels, one samples the quantile rows (Philox keyed by global row id,
the same rows as the materialised sample), one bins each chunk into its row slice of the resident uint8 bins; LR
accumulates K1 Gram blocks per chunk.  The models must equal the materialised fits: forests bit for bit, LR
coefficients to fp64 summation order (1e-9 relative).  Runs on cpu and (marked gpu) cuda."""
import numpy as np
import pytest


def _chunked(spark, X, y, rows):
    def chunks():
        for r0 in range(0, len(y), rows):
            yield {"features": X[r0:r0 + rows], "label": y[r0:r0 + rows]}
    return spark.createDataFrameFromChunks(chunks, max_rows=rows)


def _data(n, d, seed=0, cls=False):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, d)).astype(np.float32)
    z = X[:, 0] * 2 - X[:, 1] + np.sin(2 * X[:, 2]) + 0.3 * rng.normal(size=n)
    y = (z > 0).astype(np.float64) if cls else z.astype(np.float64)
    return X, y


@pytest.fixture
def streamed_calls(monkeypatch):
    from cdnaml.models import util
    seen = {"streamed": 0}
    orig = util.streamed_columns

    def counted(*a, **k):
        r = orig(*a, **k)
        seen["streamed"] += r is not None
        return r
    import cdnaml.models.regression as R
    import cdnaml.models.xgboost as XG
    monkeypatch.setattr(R, "streamed_columns", counted)
    monkeypatch.setattr(XG, "streamed_columns", counted)
    return seen


@pytest.mark.parametrize("d,rows", [(12, 1000), (100, 2048)])
def test_streamed_forests_equal_materialised(spark, streamed_calls, d, rows):
    import torch
    from cdnaml.ml.classification import RandomForestClassifier
    from cdnaml.ml.regression import RandomForestRegressor
    from cdnaml.ml.xgboost import XgboostRegressor
    from cdnaml.utils.synthetic import forest_digest
    n = 7003
    X, y = _data(n, d)
    Xc, yc = _data(n, d, seed=1, cls=True)
    mat = spark.createDataFrameFromLocalTensors({"features": torch.from_numpy(X).to(spark.device),
                                                 "label": torch.from_numpy(y).to(spark.device)})
    matc = spark.createDataFrameFromLocalTensors({"features": torch.from_numpy(Xc).to(spark.device),
                                                  "label": torch.from_numpy(yc).to(spark.device)})
    st, stc = _chunked(spark, X, y, rows), _chunked(spark, Xc, yc, rows)
    for est, a, b in [(RandomForestRegressor(numTrees=8, maxDepth=5, maxBins=40, seed=3), mat, st),
                      (RandomForestClassifier(numTrees=6, maxDepth=6, maxBins=32, seed=4), matc, stc),
                      (XgboostRegressor(n_estimators=4, max_depth=4, learning_rate=0.3, random_state=1, missing=0.0),
                       mat, st)]:
        before = streamed_calls["streamed"]
        ref = forest_digest(est.fit(a)._forest)
        got = forest_digest(est.fit(b)._forest)
        assert streamed_calls["streamed"] == before + 1, type(est).__name__
        assert got == ref, type(est).__name__


def test_streamed_linear_regression(spark, streamed_calls):
    import torch
    from cdnaml.ml.regression import LinearRegression
    n, d = 9001, 20
    X, y = _data(n, d, seed=5)
    y = y + X @ np.arange(1.0, d + 1)
    mat = spark.createDataFrameFromLocalTensors({"features": torch.from_numpy(X).to(spark.device),
                                                 "label": torch.from_numpy(y).to(spark.device)})
    ref = LinearRegression().fit(mat)
    got = LinearRegression().fit(_chunked(spark, X, y, 1500))
    assert streamed_calls["streamed"] == 1
    # cpu: fp64 Gram blocks (summation order only); cuda: K1 accumulates each block's rows in fp32 MFMA partial
    # slabs, so chunk boundaries move fp32 roundings (~1e-7 relative in the coefficients)
    tol = 1e-9 if spark.device.type == "cpu" else 2e-5
    np.testing.assert_allclose(got.coefficients.toArray(), ref.coefficients.toArray(), rtol=tol, atol=tol)
    assert got.intercept == pytest.approx(ref.intercept, rel=tol, abs=tol)


def test_streamed_fit_moves_the_features_once(spark, monkeypatch):
    """A host-chunk frame: the label pass copies only the label column, the quantile sample (frac < 1 here:
    40000 rows for a 10000-row target) gathers its rows from the host chunks, so only the binning pass streams
    the features (and only them) -- and the forest still equals the materialised fit."""
    import torch
    from cdnaml.ml.regression import RandomForestRegressor
    from cdnaml.models import inference
    from cdnaml.utils.synthetic import forest_digest
    passes = []
    orig = inference.HostChunkStream.iter_columns

    def rec(self, columns=None):
        passes.append(None if columns is None else tuple(columns))
        return orig(self, columns)
    monkeypatch.setattr(inference.HostChunkStream, "iter_columns", rec)
    n, d = 40000, 10
    X, y = _data(n, d, seed=7)
    mat = spark.createDataFrameFromLocalTensors({"features": torch.from_numpy(X).to(spark.device),
                                                 "label": torch.from_numpy(y).to(spark.device)})
    est = RandomForestRegressor(numTrees=4, maxDepth=4, maxBins=16, seed=9)
    ref = forest_digest(est.fit(mat)._forest)
    got = forest_digest(est.fit(_chunked(spark, X, y, 6000))._forest)
    assert got == ref
    assert passes == [("label",), ("features",)]
