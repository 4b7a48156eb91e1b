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
    """Every map's model cut from the group's largest forest == that map fitted alone (same fold mask)."""
    from cdnaml.ml.tuning import ParamGridBuilder
    from cdnaml.models.tree.fused import FusedTreeTuner
    df = _df(spark, cls=kind in ("rfc", "dtc"))
    est = _est(kind)
    gb = ParamGridBuilder().addGrid(est.maxDepth, [2, 4, 5])
    if kind in ("rf", "rfc"):
        gb = gb.addGrid(est.numTrees, [3, 7])
    maps = gb.build()
    tuner = FusedTreeTuner(est, maps, df)
    assert len(tuner.groups) == 1
    mask = tuner.fold_ids(7, 3) != 1
    fused = tuner.fit_split(mask)
    for j, pm in enumerate(maps):
        e = est.copy(pm)
        T = e.getNumTrees() if kind in ("rf", "rfc") else 1
        alone, _ = tuner.fit_forest(e, T, e.getMaxDepth(), mask)
        assert forest_digest(fused[j]._forest) == forest_digest(alone), pm


def test_cross_validator_fused_matches_per_map_fits_and_refit(spark):
    """CrossValidator through the fused path: avgMetrics equal evaluating each map fitted alone on each fold
    mask, and bestModel equals a plain fit of the best map on the whole dataset."""
    from cdnaml.ml.evaluation import RegressionEvaluator
    from cdnaml.ml.regression import RandomForestRegressor
    from cdnaml.ml.tuning import CrossValidator, ParamGridBuilder
    from cdnaml.models.tree.fused import FusedTreeTuner
    df = _df(spark, n=2500)
    rf = RandomForestRegressor(maxBins=40, seed=42)
    grid = ParamGridBuilder().addGrid(rf.maxDepth, [2, 5]).addGrid(rf.numTrees, [5, 10]).build()
    ev = RegressionEvaluator()
    cvm = CrossValidator(estimator=rf, estimatorParamMaps=grid, evaluator=ev, numFolds=3, seed=42).fit(df)
    tuner = FusedTreeTuner(rf, grid, df)
    tagged = df._with_global_uniform(42, "__u")
    from cdnaml.sql import functions as F
    tagged = tagged.withColumn("__fold", F.floor(F.col("__u") * 3).cast("int")).drop("__u")
    folds = tuner.fold_ids(42, 3)
    expect = np.zeros((4, 3))
    for f in range(3):
        valid = tagged.filter(F.col("__fold") == f).drop("__fold")
        for j, pm in enumerate(grid):
            e = rf.copy(pm)
            forest, d = tuner.fit_forest(e, e.getNumTrees(), e.getMaxDepth(), folds != f)
            expect[j, f] = ev.evaluate(tuner.model(e, forest, d).transform(valid))
    assert cvm.avgMetrics == pytest.approx(expect.mean(1).tolist(), rel=0, abs=0)
    best = int(np.argmin(expect.mean(1)))
    plain = rf.copy(grid[best]).fit(df)
    assert forest_digest(cvm.bestModel._forest) == forest_digest(plain._forest)
    assert cvm.bestModel.getMaxDepth() == grid[best][rf.maxDepth]


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
    assert len(tuner.groups) == 4


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
