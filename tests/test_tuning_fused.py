"""Fused tree tuning (models/tree/fused.py): one binned dataset, folds as weight masks, and the
(numTrees, maxDepth) grid as prefixes of one forest per fold -- exactly equal to fitting every map on its
own (ML 07 - Random Forests and Hyperparameter Tuning.py:72-158, Labs/ML 07L:105-141)."""
import numpy as np
import pandas as pd
import pytest

from cdnaml.utils.synthetic import forest_digest


def _df(spark, n=3000, d=8, seed=0, cls=False):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, d))
    y = 2 * X[:, 0] - X[:, 1] + np.sin(3 * X[:, 2]) + 0.2 * rng.normal(size=n)
    pdf = pd.DataFrame(X, columns=[f"x{i}" for i in range(d)])
    pdf["label"] = (y > 0).astype(float) if cls else y
    from cdnaml.ml.feature import VectorAssembler
    return VectorAssembler(inputCols=[f"x{i}" for i in range(d)], outputCol="features").transform(
        spark.createDataFrame(pdf))


def _est(kind, **kw):
    from cdnaml.ml.classification import DecisionTreeClassifier, RandomForestClassifier
    from cdnaml.ml.regression import DecisionTreeRegressor, RandomForestRegressor
    return {"rf": RandomForestRegressor, "rfc": RandomForestClassifier, "dt": DecisionTreeRegressor,
            "dtc": DecisionTreeClassifier}[kind](maxBins=32, seed=42, **kw) if kind in ("rf", "rfc") else \
        {"dt": DecisionTreeRegressor, "dtc": DecisionTreeClassifier}[kind](maxBins=32, **kw)


@pytest.mark.parametrize("kind", ["rf", "rfc", "dt", "dtc"])
def test_grid_prefix_models_equal_separate_fits(spark, kind):
    """Every map's model cut from the group's largest forest == that map fitted alone on the same split."""
    from cdnaml.ml.tuning import ParamGridBuilder
    from cdnaml.models.tree.fused import FusedTreeTuner
    df = _df(spark, cls=kind in ("rfc", "dtc"))
    train = df.randomSplit([0.7, 0.3], seed=7)[0].cache()
    est = _est(kind)
    gb = ParamGridBuilder().addGrid(est.maxDepth, [2, 4, 5])
    if kind in ("rf", "rfc"):
        gb = gb.addGrid(est.numTrees, [3, 7])
    maps = gb.build()
    tuner = FusedTreeTuner(est, maps, df)
    assert len(tuner.groups(8)) == 1
    fused, prefix = tuner.fit_split(train)
    assert prefix is None
    for j, pm in enumerate(maps):
        alone = est.fit(train, pm)
        assert forest_digest(fused[j]._forest) == forest_digest(alone._forest), pm


def _cv_both_ways(monkeypatch, make_cv, df):
    """(fused, generic) CrossValidatorModels of the same CV, plus the number of forests each trained."""
    from cdnaml.models.tree import engine, fused as fz
    calls = []
    orig = engine.ForestTrainer.train

    def counting(self, *a, **k):
        calls.append(1)
        return orig(self, *a, **k)
    monkeypatch.setattr(engine.ForestTrainer, "train", counting)
    out = []
    for flag in (True, False):
        monkeypatch.setattr(fz, "FUSED_TUNING", flag)
        calls.clear()
        out.append((make_cv().fit(df), len(calls)))
    return out


def test_cross_validator_fused_is_the_generic_cv(spark, monkeypatch):
    """ML 07:81-130: CrossValidator(rf, 2 x 2 grid, 3 folds) through the fused path equals the generic path --
    avgMetrics, bestModel -- bit for bit, with 3 forest fits + 1 refit instead of 12 + 1."""
    from cdnaml.ml.evaluation import RegressionEvaluator
    from cdnaml.ml.regression import RandomForestRegressor
    from cdnaml.ml.tuning import CrossValidator, ParamGridBuilder
    df = _df(spark, n=2500)
    rf = RandomForestRegressor(maxBins=40, seed=42)
    grid = ParamGridBuilder().addGrid(rf.maxDepth, [2, 5]).addGrid(rf.numTrees, [5, 10]).build()
    (fz, n_f), (gen, n_g) = _cv_both_ways(monkeypatch, lambda: CrossValidator(
        estimator=rf, estimatorParamMaps=grid, evaluator=RegressionEvaluator(), numFolds=3, seed=42), df)
    assert (n_f, n_g) == (3 + 1, 12 + 1)
    assert fz.avgMetrics == gen.avgMetrics
    assert forest_digest(fz.bestModel._forest) == forest_digest(gen.bestModel._forest)


def test_cross_validator_fused_pipeline_ml07(spark, monkeypatch):
    """ML 07:107 -- CrossValidator(estimator=Pipeline([StringIndexer, VectorAssembler, rf])): the prefix is fitted
    per fold as Spark does, the grid shares one forest per fold, and the result equals the generic path's."""
    from cdnaml.ml import Pipeline
    from cdnaml.ml.evaluation import RegressionEvaluator
    from cdnaml.ml.feature import StringIndexer, VectorAssembler
    from cdnaml.ml.regression import RandomForestRegressor
    from cdnaml.ml.tuning import CrossValidator, ParamGridBuilder
    rng = np.random.default_rng(4)
    n = 2400
    pdf = pd.DataFrame({"room": rng.choice(["entire", "private", "shared", "hotel"], n, p=[.5, .3, .15, .05]),
                        "hood": rng.choice([f"h{i}" for i in range(37)], n),
                        "beds": rng.integers(1, 6, n).astype(float), "lat": rng.normal(size=n)})
    pdf["price"] = 50 * pdf.beds + (pdf.room == "entire") * 80 + 5 * pdf.lat + rng.normal(size=n) * 10
    df = spark.createDataFrame(pdf)
    si = StringIndexer(inputCols=["room", "hood"], outputCols=["roomIndex", "hoodIndex"], handleInvalid="skip")
    va = VectorAssembler(inputCols=["roomIndex", "hoodIndex", "beds", "lat"], outputCol="features")
    rf = RandomForestRegressor(labelCol="price", maxBins=40, seed=42)
    pipe = Pipeline(stages=[si, va, rf])
    grid = ParamGridBuilder().addGrid(rf.maxDepth, [2, 5]).addGrid(rf.numTrees, [5, 10]).build()
    (fz, n_f), (gen, n_g) = _cv_both_ways(monkeypatch, lambda: CrossValidator(
        estimator=pipe, estimatorParamMaps=grid, evaluator=RegressionEvaluator(labelCol="price"), numFolds=3,
        seed=42), df)
    assert (n_f, n_g) == (3 + 1, 12 + 1)
    assert fz.avgMetrics == gen.avgMetrics
    assert forest_digest(fz.bestModel.stages[-1]._forest) == forest_digest(gen.bestModel.stages[-1]._forest)
    # a map touching a prefix stage keeps the generic path
    from cdnaml.models.tree.fused import FusedTreeTuner
    assert not FusedTreeTuner.supported(pipe, [{si.handleInvalid: "keep", rf.maxDepth: 2}])


def test_fused_groups_split_on_non_grid_params(spark):
    """Maps differing in a param other than numTrees / maxDepth form separate groups (separate forests), and
    numTrees == 1 (no bagging, all features under 'auto') never shares a forest with bagged maps."""
    from cdnaml.ml.regression import RandomForestRegressor
    from cdnaml.ml.tuning import ParamGridBuilder
    from cdnaml.models.tree.fused import FusedTreeTuner
    df = _df(spark, n=800)
    rf = RandomForestRegressor(maxBins=32, seed=1)
    maps = ParamGridBuilder().addGrid(rf.numTrees, [1, 4]).addGrid(rf.minInstancesPerNode, [1, 20]).build()
    tuner = FusedTreeTuner(rf, maps, df)
    assert len(tuner.groups(8)) == 4


def test_train_validation_split_fused(spark):
    from cdnaml.ml.evaluation import RegressionEvaluator
    from cdnaml.ml.regression import RandomForestRegressor
    from cdnaml.ml.tuning import ParamGridBuilder, TrainValidationSplit
    df = _df(spark, n=2000)
    rf = RandomForestRegressor(maxBins=32, seed=3)
    grid = ParamGridBuilder().addGrid(rf.maxDepth, [1, 6]).addGrid(rf.numTrees, [2, 8]).build()
    tvm = TrainValidationSplit(estimator=rf, estimatorParamMaps=grid, evaluator=RegressionEvaluator(),
                               trainRatio=0.75, seed=9).fit(df)
    assert len(tvm.validationMetrics) == 4
    assert int(np.argmin(tvm.validationMetrics)) in (1, 3)  # depth 6 beats depth 1 on this label
    assert tvm.bestModel.getMaxDepth() == 6
