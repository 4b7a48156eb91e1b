"""XGBoost-style GBDT (ML 11) and hyperopt (T3/T4; ML 08, L08)."""
import functools

import numpy as np
import pandas as pd
import pytest

from cdnaml.hyperopt import STATUS_OK, SparkTrials, Trials, anneal, fmin, hp, rand, space_eval, tpe
from cdnaml.ml import Pipeline, PipelineModel
from cdnaml.ml.evaluation import BinaryClassificationEvaluator, MulticlassClassificationEvaluator, \
    RegressionEvaluator
from cdnaml.ml.feature import StringIndexer, VectorAssembler
from cdnaml.ml.regression import RandomForestRegressor
from cdnaml.ml.xgboost import XgboostClassifier, XgboostRegressor
from cdnaml.sql import functions as F


def _reg(spark, n=3000, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, 4))
    X[rng.uniform(size=n) < 0.25, 0] = 0.0
    y = np.where(X[:, 0] == 0, 6.0, 2 * X[:, 0]) + X[:, 1] ** 2 + 0.1 * rng.normal(size=n)
    pdf = pd.DataFrame(X, columns=list("abcd"))
    pdf["label"] = y
    return VectorAssembler(inputCols=list("abcd"), outputCol="features").transform(spark.createDataFrame(pdf)), X, y


def test_xgb_regressor_learns_missing_direction(spark, tmp_path):
    df, X, y = _reg(spark)
    m = XgboostRegressor(n_estimators=100, learning_rate=0.1, max_depth=4, random_state=42, missing=0).fit(df)
    pred = m.transform(df)
    rmse = RegressionEvaluator().evaluate(pred)
    assert rmse < 0.25
    p = pred.toPandas()
    zero = X[:, 0] == 0
    # rows with a[0] == missing get the learned default branch: prediction near 6 + b^2
    assert np.abs(p.prediction.values[zero] - (6 + X[zero, 1] ** 2)).mean() < 0.4
    # save / load in a pipeline
    pm = Pipeline(stages=[XgboostRegressor(n_estimators=20, max_depth=3, missing=0)]).fit(df)
    path = str(tmp_path / "xgb")
    pm.write().overwrite().save(path)
    a = pm.transform(df).select("prediction").toPandas().prediction.values
    b = PipelineModel.load(path).transform(df).select("prediction").toPandas().prediction.values
    np.testing.assert_array_equal(a, b)
    assert m.get_booster().get_score(importance_type="gain")


def test_xgb_matches_sklearn_hist_gbdt_quality(spark):
    from sklearn.ensemble import HistGradientBoostingRegressor

    df, X, y = _reg(spark, seed=3)
    m = XgboostRegressor(n_estimators=60, learning_rate=0.2, max_depth=4, reg_lambda=1.0).fit(df)
    ours = RegressionEvaluator().evaluate(m.transform(df))
    sk = HistGradientBoostingRegressor(max_iter=60, learning_rate=0.2, max_depth=4, l2_regularization=1.0,
                                       early_stopping=False).fit(X, y)
    ref = float(np.sqrt(np.mean((sk.predict(X) - y) ** 2)))
    assert ours < 1.5 * ref + 0.05  # parity unpinned (xgboost not installed): same-quality bound vs sklearn


def test_xgb_pipeline_log_label(spark):
    """ML 11:36-103: StringIndexer + VectorAssembler + XgboostRegressor on log(price), exp back."""
    rng = np.random.default_rng(1)
    n = 2000
    hood = rng.choice(["a", "b", "c", "d"], n)
    acc = rng.integers(1, 8, n).astype(float)
    price = np.exp(3 + 0.2 * acc + (hood == "a") * 0.5 + 0.05 * rng.normal(size=n))
    df = spark.createDataFrame(pd.DataFrame({"hood": hood, "acc": acc, "price": price}))
    df = df.withColumn("label", F.log(F.col("price")))
    si = StringIndexer(inputCols=["hood"], outputCols=["hoodIdx"], handleInvalid="skip")
    va = VectorAssembler(inputCols=["hoodIdx", "acc"], outputCol="features")
    xgb = XgboostRegressor(n_estimators=100, learning_rate=0.1, max_depth=4, random_state=42, missing=0)
    pm = Pipeline(stages=[si, va, xgb]).fit(df)
    pred = pm.transform(df).withColumn("prediction", F.exp(F.col("prediction")))
    r2 = RegressionEvaluator(labelCol="price", metricName="r2").evaluate(pred)
    assert r2 > 0.95


def test_xgb_classifier_binary_multiclass_early_stop(spark):
    rng = np.random.default_rng(0)
    n = 3000
    X = rng.normal(size=(n, 3))
    yb = (X[:, 0] + X[:, 1] > 0).astype(float)
    ym = np.digitize(X[:, 0], [-0.5, 0.5]).astype(float)
    val = rng.uniform(size=n) < 0.2
    pdf = pd.DataFrame(X, columns=list("abc"))
    pdf["yb"], pdf["ym"], pdf["val"] = yb, ym, val
    df = VectorAssembler(inputCols=list("abc"), outputCol="features").transform(spark.createDataFrame(pdf))
    mb = XgboostClassifier(n_estimators=50, max_depth=3, labelCol="yb").fit(df)
    auc = BinaryClassificationEvaluator(labelCol="yb").evaluate(mb.transform(df))
    assert auc > 0.97
    mm = XgboostClassifier(n_estimators=30, max_depth=3, labelCol="ym").fit(df)
    acc = MulticlassClassificationEvaluator(labelCol="ym", metricName="accuracy").evaluate(mm.transform(df))
    assert acc > 0.95 and mm.numClasses == 3
    es = XgboostClassifier(n_estimators=500, learning_rate=0.3, max_depth=3, labelCol="yb",
                           validationIndicatorCol="val", early_stopping_rounds=5).fit(df)
    assert len(es._forest.roots) < 500


def test_hyperopt_fmin_tpe_and_space_eval():
    space = {"x": hp.uniform("x", -5, 5), "q": hp.quniform("q", 2, 10, 1),
             "c": hp.choice("c", ["a", "b", "c"]), "lr": hp.loguniform("lr", np.log(1e-4), 0.0)}

    def f(p):
        return (p["x"] - 1.3) ** 2 + 0.1 * (p["q"] - 7) ** 2 + {"a": 1, "b": 0, "c": 2}[p["c"]] + \
            abs(np.log10(p["lr"]) + 2)

    trials = Trials()
    best = fmin(f, space, algo=functools.partial(tpe.suggest, n_startup_jobs=5), max_evals=60, trials=trials,
                rstate=np.random.default_rng(42))
    assert best["c"] == 1  # choice -> index (Labs/ML 08L:118)
    assert space_eval(space, best)["c"] == "b"
    assert float(best["q"]).is_integer()
    assert min(trials.losses()) < 0.6
    # deterministic given rstate
    again = fmin(f, space, algo=functools.partial(tpe.suggest, n_startup_jobs=5), max_evals=60,
                 rstate=np.random.default_rng(42))
    assert again == best
    r = fmin(f, space, algo=rand.suggest, max_evals=30, rstate=np.random.RandomState(0))
    a = fmin(f, space, algo=anneal.suggest, max_evals=30, rstate=np.random.RandomState(0))
    assert set(r) == set(a) == {"x", "q", "c", "lr"}


def test_hyperopt_dict_results_failures_and_spark_trials():
    calls = []

    def f(p):
        calls.append(p)
        if p["x"] > 4.5:
            raise RuntimeError("boom")
        return {"loss": (p["x"] - 2) ** 2, "status": STATUS_OK}

    st = SparkTrials(parallelism=3)
    best = fmin(f, {"x": hp.uniform("x", 0, 5)}, algo=tpe.suggest, max_evals=24, trials=st,
                rstate=np.random.default_rng(1))
    assert len(st) == 24 and abs(best["x"] - 2) < 0.7
    assert st.best_trial["result"]["status"] == STATUS_OK
    with pytest.raises(ZeroDivisionError):  # plain Trials re-raise objective errors
        fmin(lambda p: 1 / 0, {"x": hp.uniform("x", 0, 1)}, max_evals=2)


def test_hyperopt_over_distributed_mllib(spark):
    """ML 08:78-170: objective builds pipeline.copy({rf.maxDepth: q, rf.numTrees: q}) and returns RMSE."""
    rng = np.random.default_rng(0)
    n = 1500
    X = rng.normal(size=(n, 3))
    y = np.sin(2 * X[:, 0]) * 3 + X[:, 1]
    pdf = pd.DataFrame(X, columns=list("abc"))
    pdf["price"] = y
    df = spark.createDataFrame(pdf)
    train, val = df.randomSplit([0.8, 0.2], seed=42)
    va = VectorAssembler(inputCols=list("abc"), outputCol="features")
    rf = RandomForestRegressor(labelCol="price", maxBins=40, seed=42)
    pipeline = Pipeline(stages=[va, rf])
    ev = RegressionEvaluator(labelCol="price")

    def objective(params):
        est = pipeline.copy({rf.maxDepth: params["max_depth"], rf.numTrees: params["num_trees"]})
        return ev.evaluate(est.fit(train).transform(val))

    space = {"max_depth": hp.quniform("max_depth", 2, 5, 1), "num_trees": hp.quniform("num_trees", 10, 30, 1)}
    best = fmin(objective, space, algo=tpe.suggest, max_evals=4, trials=Trials(), rstate=np.random.default_rng(42))
    assert 2 <= best["max_depth"] <= 5 and 10 <= best["num_trees"] <= 30


def test_fmin_trials_share_binned_data_only_inside_the_search(spark):
    """Verdict r2 item 6: fmin's trials reuse one binning of the training features (tuner-scoped cache keyed by
    the features' content, so the per-trial StringIndexer / VectorAssembler refit still hits); the losses equal
    fits outside fmin bit for bit, and after fmin returns a fit bins its data again (no global cache)."""
    from cdnaml.models.tree import bincache
    rng = np.random.default_rng(5)
    n = 2000
    X = rng.normal(size=(n, 3))
    pdf = pd.DataFrame(X, columns=list("abc"))
    pdf["room"] = rng.choice(["entire", "private", "shared"], n)
    pdf["price"] = np.sin(2 * X[:, 0]) * 3 + X[:, 1] + (pdf["room"] == "entire") * 2.0
    df = spark.createDataFrame(pdf)
    train, val = df.randomSplit([0.8, 0.2], seed=42)
    si = StringIndexer(inputCols=["room"], outputCols=["roomIdx"], handleInvalid="skip")
    va = VectorAssembler(inputCols=["roomIdx", "a", "b", "c"], outputCol="features")
    rf = RandomForestRegressor(labelCol="price", maxBins=40, seed=42)
    pipeline = Pipeline(stages=[si, va, rf])
    ev = RegressionEvaluator(labelCol="price")
    seen = []

    def objective(params):
        seen.append((int(params["max_depth"]), int(params["num_trees"])))
        est = pipeline.copy({rf.maxDepth: seen[-1][0], rf.numTrees: seen[-1][1]})
        return ev.evaluate(est.fit(train).transform(val))

    space = {"max_depth": hp.quniform("max_depth", 2, 5, 1), "num_trees": hp.quniform("num_trees", 10, 30, 1)}
    b0, h0 = bincache.stats["builds"], bincache.stats["hits"]
    trials = Trials()
    fmin(objective, space, algo=tpe.suggest, max_evals=4, trials=trials, rstate=np.random.default_rng(1))
    assert bincache.stats["builds"] - b0 == 1 and bincache.stats["hits"] - h0 == 3
    assert not bincache.active()
    for (dpt, nt), loss in zip(seen, trials.losses()):
        est = pipeline.copy({rf.maxDepth: dpt, rf.numTrees: nt})
        assert ev.evaluate(est.fit(train).transform(val)) == loss
    assert bincache.stats["builds"] - b0 == 1 + len(seen)


class _Crash(Exception):
    pass


@pytest.mark.parametrize("kind", ["xgb", "gbt"])
def test_boosting_checkpoint_resume_is_exact(spark, tmp_path, monkeypatch, kind):
    """a boosting fit interrupted after round 8 resumes from its round-8 checkpoint
    (SparkContext.setCheckpointDir + checkpoint interval 4) and gives the uninterrupted model."""
    from cdnaml.ml.regression import GBTRegressor
    from cdnaml.models.tree import checkpoint as ckm
    df, X, y = _reg(spark, n=1500, seed=5)
    spark.sparkContext.setCheckpointDir(str(tmp_path / "ck"))

    def make():
        if kind == "xgb":
            return XgboostRegressor(n_estimators=12, max_depth=3, learning_rate=0.3, subsample=0.8,
                                    random_state=7, checkpoint_interval=4)
        return GBTRegressor(maxIter=12, maxDepth=3, subsamplingRate=0.8, seed=7, checkpointInterval=4)

    full = make().fit(df).transform(df).select("prediction").toPandas().prediction.values
    import shutil
    shutil.rmtree(tmp_path / "ck")
    spark.sparkContext.setCheckpointDir(str(tmp_path / "ck"))
    orig = ckm.RoundCheckpointer.maybe_save

    def crashing(self, rounds_done, *a, **k):
        orig(self, rounds_done, *a, **k)
        if rounds_done == 10:
            raise _Crash()
    monkeypatch.setattr(ckm.RoundCheckpointer, "maybe_save", crashing)
    with pytest.raises(_Crash):
        make().fit(df)
    monkeypatch.setattr(ckm.RoundCheckpointer, "maybe_save", orig)
    seen = []
    orig_load = ckm.RoundCheckpointer.load

    def recording_load(self):
        r = orig_load(self)
        seen.append(None if r is None else r[0])
        return r
    monkeypatch.setattr(ckm.RoundCheckpointer, "load", recording_load)
    resumed_model = make().fit(df)
    assert seen == [8]  # resumed from the last complete interval before the crash
    resumed = resumed_model.transform(df).select("prediction").toPandas().prediction.values
    np.testing.assert_array_equal(full, resumed)
    spark.conf.unset("cdnaml.checkpoint.dir")


@pytest.mark.parametrize("kind", ["xgb", "gbt"])
def test_checkpoint_never_resumes_foreign_data(spark, tmp_path, kind):
    """two same-shape datasets fit in a row under one checkpoint dir give different models (the
    checkpoint key carries a data fingerprint), and a completed fit leaves no checkpoint behind."""
    import os
    from cdnaml.ml.regression import GBTRegressor
    spark.sparkContext.setCheckpointDir(str(tmp_path / "ck"))

    def make():
        if kind == "xgb":
            return XgboostRegressor(n_estimators=6, max_depth=3, random_state=7, checkpoint_interval=2)
        return GBTRegressor(maxIter=6, maxDepth=3, seed=7, checkpointInterval=2)

    df1, _, _ = _reg(spark, n=800, seed=1)
    df2, _, _ = _reg(spark, n=800, seed=2)
    p1 = make().fit(df1).transform(df2).select("prediction").toPandas().prediction.values
    left = [f for _, _, fs in os.walk(tmp_path / "ck") for f in fs]
    assert left == []
    p2 = make().fit(df2).transform(df2).select("prediction").toPandas().prediction.values
    assert not np.array_equal(p1, p2)
    spark.conf.unset("cdnaml.checkpoint.dir")
