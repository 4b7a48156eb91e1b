"""ML library on the CPU path (notebook invariants from Appendix A)."""
import numpy as np
import pandas as pd
import pytest

from cdnaml.ml import Pipeline, PipelineModel
from cdnaml.ml.classification import (DecisionTreeClassifier, GBTClassifier, LinearSVC, LogisticRegression,
                                      NaiveBayes, RandomForestClassifier)
from cdnaml.ml.clustering import BisectingKMeans, KMeans
from cdnaml.ml.evaluation import (BinaryClassificationEvaluator, MulticlassClassificationEvaluator,
                                  RegressionEvaluator)
from cdnaml.ml.feature import (Imputer, OneHotEncoder, RFormula, StandardScaler, StringIndexer,
                               VectorAssembler)
from cdnaml.ml.recommendation import ALS
from cdnaml.ml.regression import (DecisionTreeRegressor, GBTRegressor, LinearRegression,
                                  RandomForestRegressor)
from cdnaml.ml.tuning import CrossValidator, ParamGridBuilder, TrainValidationSplit
from cdnaml.sql import functions as F


def _reg_frame(spark, n=3000, d=5, seed=0, noise=0.1):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, d))
    w = np.arange(1, d + 1, dtype=float)
    y = X @ w + 3.0 + noise * rng.normal(size=n)
    pdf = pd.DataFrame(X, columns=[f"x{i}" for i in range(d)])
    pdf["label"] = y
    return spark.createDataFrame(pdf), X, y


def test_linear_regression_matches_sklearn(spark):
    from sklearn.linear_model import LinearRegression as SkLR

    df, X, y = _reg_frame(spark)
    va = VectorAssembler(inputCols=[f"x{i}" for i in range(5)], outputCol="features")
    m = LinearRegression(featuresCol="features", labelCol="label").fit(va.transform(df))
    sk = SkLR().fit(X, y)
    np.testing.assert_allclose(m.coefficients.toArray(), sk.coef_, rtol=1e-6, atol=1e-8)
    assert abs(m.intercept - sk.intercept_) < 1e-6
    pred = m.transform(va.transform(df))
    rmse = RegressionEvaluator(labelCol="label").evaluate(pred)
    r2 = RegressionEvaluator(labelCol="label", metricName="r2").evaluate(pred)
    assert rmse < 0.12 and r2 > 0.999


def test_weighted_linear_regression_matches_sklearn(spark):
    """weightCol: the weighted normal equations (K1 Gram over sqrt(w)-scaled rows with sqrt(w) as an extra
    column on the GPU) equal sklearn's sample_weight fit."""
    from sklearn.linear_model import LinearRegression as SkLR
    df, X, y = _reg_frame(spark, n=4000, seed=3, noise=0.5)
    wts = np.random.default_rng(4).integers(1, 6, len(y)).astype(float)
    pdf = df.toPandas()
    pdf["w"] = wts
    va = VectorAssembler(inputCols=[f"x{i}" for i in range(5)], outputCol="features")
    m = LinearRegression(featuresCol="features", labelCol="label", weightCol="w").fit(
        va.transform(spark.createDataFrame(pdf)))
    sk = SkLR().fit(X, y, sample_weight=wts)
    np.testing.assert_allclose(m.coefficients.toArray(), sk.coef_, rtol=2e-5, atol=2e-6)
    assert abs(m.intercept - sk.intercept_) < 2e-5


def test_lr_on_non_vector_column_fails(spark):
    """ML 02:80-89: estimators need a vector features column."""
    df, _, _ = _reg_frame(spark, n=100)
    with pytest.raises(Exception):
        LinearRegression(featuresCol="x0", labelCol="label").fit(df)


def test_ridge_elastic_net(spark):
    from sklearn.linear_model import ElasticNet, Ridge

    df, X, y = _reg_frame(spark, n=2000, seed=3, noise=1.0)
    va = VectorAssembler(inputCols=[f"x{i}" for i in range(5)], outputCol="features")
    vdf = va.transform(df)
    # Spark standardizes the label: its L2 objective in original units is
    # 1/(2n) ||y - Xw||^2 + lambda / (2 sigma_y) ||w||^2  (standardization=False), i.e. sklearn
    # Ridge(alpha = n lambda / sigma_y); the L1 term is unaffected (Lasso(alpha = lambda)).
    m = LinearRegression(regParam=0.5, elasticNetParam=0.0, standardization=False).fit(vdf)
    sk = Ridge(alpha=0.5 * len(y) / np.std(y)).fit(X, y)
    np.testing.assert_allclose(m.coefficients.toArray(), sk.coef_, rtol=1e-4)
    m1 = LinearRegression(regParam=0.1, elasticNetParam=1.0, standardization=False).fit(vdf)
    sk1 = ElasticNet(alpha=0.1, l1_ratio=1.0, tol=1e-10, max_iter=100000).fit(X, y)
    np.testing.assert_allclose(m1.coefficients.toArray(), sk1.coef_, rtol=1e-3, atol=1e-4)


def test_pipeline_si_ohe_va_lr_save_load(spark, tmp_path):
    rng = np.random.default_rng(0)
    n = 2000
    cat = rng.choice(["a", "b", "c", "d"], size=n)
    x = rng.normal(size=n)
    y = x * 2 + np.select([cat == "a", cat == "b", cat == "c"], [1.0, -1.0, 5.0], 0.0) + 0.01 * rng.normal(size=n)
    df = spark.createDataFrame(pd.DataFrame({"cat": cat, "x": x, "price": y}))
    si = StringIndexer(inputCols=["cat"], outputCols=["catIdx"], handleInvalid="skip")
    ohe = OneHotEncoder(inputCols=["catIdx"], outputCols=["catOHE"])
    va = VectorAssembler(inputCols=["catOHE", "x"], outputCol="features")
    lr = LinearRegression(labelCol="price", featuresCol="features")
    pm = Pipeline(stages=[si, ohe, va, lr]).fit(df)
    pred = pm.transform(df)
    rmse = RegressionEvaluator(labelCol="price").evaluate(pred)
    assert rmse < 0.02
    path = str(tmp_path / "pm")
    pm.write().overwrite().save(path)
    pm2 = PipelineModel.load(path)
    p1 = pred.select("prediction").toPandas().prediction.values
    p2 = pm2.transform(df).select("prediction").toPandas().prediction.values
    np.testing.assert_array_equal(p1, p2)
    # unseen category is skipped by handleInvalid="skip"
    new = spark.createDataFrame(pd.DataFrame({"cat": ["a", "zzz"], "x": [0.0, 0.0], "price": [0.0, 0.0]}))
    assert pm2.transform(new).count() == 1


def test_string_indexer_frequency_order(spark):
    df = spark.createDataFrame(pd.DataFrame({"c": ["x", "y", "y", "z", "z", "z"]}))
    m = StringIndexer(inputCol="c", outputCol="i").fit(df)
    assert list(m.labels) == ["z", "y", "x"]
    out = m.transform(df).toPandas()
    assert out.i.tolist() == [2.0, 1.0, 1.0, 0.0, 0.0, 0.0]


def test_rformula(spark):
    rng = np.random.default_rng(2)
    n = 1500
    cat = rng.choice(["p", "q"], size=n)
    x = rng.normal(size=n)
    y = 3 * x + (cat == "p") * 2.0
    df = spark.createDataFrame(pd.DataFrame({"cat": cat, "x": x, "price": y}))
    rf = RFormula(formula="price ~ .", featuresCol="features", labelCol="label", handleInvalid="skip")
    out = rf.fit(df).transform(df)
    m = LinearRegression().fit(out)
    # an exact linear law: fp64 feature vectors on the host; on the GPU features are fp32 vectors (7 digits)
    tol = 1e-6 if spark.device.type == "cpu" else 2e-5
    assert RegressionEvaluator().evaluate(m.transform(out)) < tol
    out2 = RFormula(formula="log_price ~ . - price").fit(df.withColumn("log_price", F.log(F.abs("price") + 1)))
    assert out2 is not None


def test_imputer_median(spark):
    df = spark.createDataFrame(pd.DataFrame({"a": [1.0, 2.0, None, 4.0, 100.0], "b": [None, 1.0, 1.0, 3.0, 5.0]}))
    m = Imputer(strategy="median", inputCols=["a", "b"], outputCols=["a", "b"]).fit(df)
    out = m.transform(df).toPandas()
    assert out.a.tolist()[2] in (2.0, 4.0)  # approxQuantile median of {1,2,4,100}
    assert out.b.tolist()[0] in (1.0, 3.0)
    assert not out.isna().any().any()


def _airbnb_like(spark, n=4000, ncat=36, seed=0):
    rng = np.random.default_rng(seed)
    nb = np.array([f"hood{i}" for i in range(ncat)])[rng.integers(0, ncat, n)]
    acc = rng.integers(1, 8, n).astype(float)
    beds = np.maximum(1, acc // 2 + rng.integers(0, 2, n))
    rev = rng.uniform(60, 100, n)
    base = {f"hood{i}": v for i, v in enumerate(rng.uniform(50, 300, ncat))}
    price = np.array([base[h] for h in nb]) + 40 * acc + 10 * beds + rng.normal(0, 10, n)
    return spark.createDataFrame(pd.DataFrame({"neighbourhood_cleansed": nb, "accommodates": acc, "beds": beds,
                                               "review_scores_rating": rev, "price": price}))


def test_decision_tree_maxbins_error_and_importances(spark):
    """ML 06:79-118: maxBins below a categorical arity fails; setMaxBins(40) fixes it."""
    df = _airbnb_like(spark)
    si = StringIndexer(inputCols=["neighbourhood_cleansed"], outputCols=["nIdx"], handleInvalid="skip")
    va = VectorAssembler(inputCols=["nIdx", "accommodates", "beds", "review_scores_rating"], outputCol="features")
    dt = DecisionTreeRegressor(labelCol="price")
    with pytest.raises(Exception, match="maxBins"):
        Pipeline(stages=[si, va, dt]).fit(df)
    dt.setMaxBins(40)
    pm = Pipeline(stages=[si, va, dt]).fit(df)
    m = pm.stages[-1]
    fi = m.featureImportances.toArray()
    assert abs(fi.sum() - 1.0) < 1e-9
    assert fi[3] < fi[0] and fi[3] < fi[1]  # review score is noise
    pred = pm.transform(df).toPandas()
    assert pred.prediction.max() <= pred.price.max() + 1e-9  # trees cannot extrapolate (ML 06:196-198)
    assert m.depth <= 5


def test_random_forest_regressor_beats_mean(spark):
    df = _airbnb_like(spark, n=3000)
    si = StringIndexer(inputCols=["neighbourhood_cleansed"], outputCols=["nIdx"], handleInvalid="skip")
    va = VectorAssembler(inputCols=["nIdx", "accommodates", "beds", "review_scores_rating"], outputCol="features")
    rf = RandomForestRegressor(labelCol="price", maxBins=40, numTrees=10, maxDepth=5, seed=42)
    train, test = df.randomSplit([0.8, 0.2], seed=42)
    pm = Pipeline(stages=[si, va, rf]).fit(train)
    ev = RegressionEvaluator(labelCol="price")
    rmse = ev.evaluate(pm.transform(test))
    mean = train.select(F.avg("price")).first()[0]
    base = ev.evaluate(test.withColumn("prediction", F.lit(mean)))
    assert rmse < 0.6 * base
    # same seed -> identical model
    pm2 = Pipeline(stages=[si, va, rf]).fit(train)
    a = pm.transform(test).select("prediction").toPandas().prediction.values
    b = pm2.transform(test).select("prediction").toPandas().prediction.values
    np.testing.assert_array_equal(a, b)
    assert len(pm.stages[-1].trees) == 10


def test_gbt_regressor(spark):
    df, X, y = _reg_frame(spark, n=2000, d=3)
    va = VectorAssembler(inputCols=["x0", "x1", "x2"], outputCol="features")
    m = GBTRegressor(maxIter=30, maxDepth=3, stepSize=0.3, seed=1).fit(va.transform(df))
    rmse = RegressionEvaluator().evaluate(m.transform(va.transform(df)))
    assert rmse < 0.35 * np.std(y)


def _cls_frame(spark, n=3000, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, 4))
    logit = 2 * X[:, 0] - 1.5 * X[:, 1] + 0.5
    y = (rng.uniform(size=n) < 1 / (1 + np.exp(-logit))).astype(float)
    pdf = pd.DataFrame(X, columns=["a", "b", "c", "d"])
    pdf["label"] = y
    df = VectorAssembler(inputCols=["a", "b", "c", "d"], outputCol="features").transform(spark.createDataFrame(pdf))
    return df, X, y


def test_logistic_regression_matches_sklearn(spark):
    from sklearn.linear_model import LogisticRegression as SkLog

    df, X, y = _cls_frame(spark)
    m = LogisticRegression(regParam=0.0, maxIter=200, tol=1e-10).fit(df)
    sk = SkLog(penalty=None, tol=1e-10, max_iter=2000).fit(X, y)
    np.testing.assert_allclose(m.coefficients.toArray(), sk.coef_[0], rtol=2e-3, atol=2e-3)
    pred = m.transform(df)
    auc = BinaryClassificationEvaluator().evaluate(pred)
    acc = MulticlassClassificationEvaluator(metricName="accuracy").evaluate(pred)
    from sklearn.metrics import roc_auc_score
    assert abs(auc - roc_auc_score(y, sk.decision_function(X))) < 2e-3
    assert acc > 0.7
    # L1 (OWL-QN) zeroes the noise features
    m1 = LogisticRegression(regParam=0.05, elasticNetParam=1.0).fit(df)
    c = m1.coefficients.toArray()
    assert abs(c[2]) < 1e-6 and abs(c[3]) < 1e-6 and abs(c[0]) > 0.1


def test_binary_evaluator_num_bins_downsampling(spark):
    """numBins (Spark's BinaryClassificationMetrics down-sampling): numBins=0 is the exact curve (== sklearn's
    roc_auc_score); the default 1000 with 5000 distinct scores keeps every 5th cumulative point of the descending
    order (Spark groups countsSize / numBins consecutive score points); fewer than 2 * numBins distinct scores
    stay exact."""
    from sklearn.metrics import roc_auc_score
    rng = np.random.default_rng(4)
    n = 5000
    s = rng.normal(size=n)
    yb = (rng.random(n) < 1 / (1 + np.exp(-2 * s))).astype(np.float64)
    df = spark.createDataFrame(pd.DataFrame({"rawPrediction": s, "label": yb}))
    exact = BinaryClassificationEvaluator(numBins=0).evaluate(df)
    assert abs(exact - roc_auc_score(yb, s)) < 1e-12
    order = np.argsort(-s)
    tp, fp = np.cumsum(yb[order]), np.cumsum(1 - yb[order])
    ends = np.arange(4, n, 5)
    tpr = np.r_[0.0, tp[ends] / tp[-1], 1.0]
    fpr = np.r_[0.0, fp[ends] / fp[-1], 1.0]
    assert abs(BinaryClassificationEvaluator().evaluate(df) - np.trapezoid(tpr, fpr)) < 1e-12
    assert BinaryClassificationEvaluator(numBins=5000).evaluate(df) == exact


def test_tree_classifiers_and_aupr(spark):
    df, X, y = _cls_frame(spark, n=2000)
    for est in (DecisionTreeClassifier(maxDepth=4), RandomForestClassifier(numTrees=10, seed=42),
                GBTClassifier(maxIter=10, maxDepth=3)):
        pred = est.fit(df).transform(df)
        auc = BinaryClassificationEvaluator(metricName="areaUnderROC").evaluate(pred)
        pr = BinaryClassificationEvaluator(metricName="areaUnderPR").evaluate(pred)
        assert auc > 0.8 and 0 < pr <= 1, type(est).__name__


def test_naive_bayes_and_svc(spark):
    df, X, y = _cls_frame(spark, n=1500)
    pred = LinearSVC(maxIter=50).fit(df).transform(df)
    assert MulticlassClassificationEvaluator(metricName="accuracy").evaluate(pred) > 0.7
    pos = df.withColumn("features", F.col("features"))  # NB needs non-negative features
    rng = np.random.default_rng(0)
    counts = rng.poisson(3, size=(500, 4)).astype(float)
    lab = (counts[:, 0] > counts[:, 1]).astype(float)
    pdf = pd.DataFrame(counts, columns=list("abcd"))
    pdf["label"] = lab
    nb_df = VectorAssembler(inputCols=list("abcd"), outputCol="features").transform(spark.createDataFrame(pdf))
    nb = NaiveBayes(smoothing=1.0).fit(nb_df)
    assert MulticlassClassificationEvaluator(metricName="accuracy").evaluate(nb.transform(nb_df)) > 0.6
    assert pos is not None


def test_kmeans_maxiter_zero_returns_init_centres(spark):
    """MLE 02: maxIter=0 returns the initial centres; more iterations reduce the cost."""
    from sklearn.datasets import load_iris

    X = load_iris().data[:, :2]
    df = VectorAssembler(inputCols=["a", "b"], outputCol="features").transform(
        spark.createDataFrame(pd.DataFrame(X, columns=["a", "b"])))
    m0 = KMeans(k=3, seed=221, maxIter=0).fit(df)
    m20 = KMeans(k=3, seed=221, maxIter=20).fit(df)
    c0 = np.array(m0.clusterCenters())
    np.testing.assert_array_equal(c0, np.array(KMeans(k=3, seed=221, maxIter=0).fit(df).clusterCenters()))
    rows = {tuple(r) for r in X.tolist()}  # vectors are Double, as Spark's VectorUDT
    cr = KMeans(k=3, seed=221, maxIter=0, initMode="random").fit(df).clusterCenters()
    assert all(tuple(c) in rows for c in np.array(cr).tolist())  # random init picks data points
    assert m20.summary.trainingCost <= m0.summary.trainingCost
    assert m20.transform(df).select("prediction").distinct().count() == 3
    bk = BisectingKMeans(k=3, seed=1).fit(df)
    assert len(bk.clusterCenters()) == 3


def test_als_cv_selects_planted_rank(spark):
    """MLE 01:186-202: the CV must choose rank 12 over rank 4."""
    rng = np.random.default_rng(0)
    nu, ni, r = 300, 200, 12
    U = rng.normal(size=(nu, r))
    V = rng.normal(size=(ni, r))
    mask = rng.uniform(size=(nu, ni)) < 0.3
    uu, ii = np.nonzero(mask)
    rating = (U[uu] * V[ii]).sum(1) + 0.1 * rng.normal(size=len(uu))
    df = spark.createDataFrame(pd.DataFrame({"userId": uu, "movieId": ii, "rating": rating}))
    als = ALS(userCol="userId", itemCol="movieId", ratingCol="rating", maxIter=5, seed=42,
              coldStartStrategy="drop", regParam=0.1)
    assert als.getItemCol() == "movieId"
    grid = ParamGridBuilder().addGrid(als.rank, [4, 12]).build()
    cv = CrossValidator(estimator=als, estimatorParamMaps=grid, evaluator=RegressionEvaluator(labelCol="rating"),
                        numFolds=3, seed=42)
    cvm = cv.fit(df)
    assert cvm.bestModel.rank == 12
    assert len(cvm.avgMetrics) == 2 and cvm.avgMetrics[1] < cvm.avgMetrics[0]


def test_cross_validator_in_pipeline_and_tvs(spark, tmp_path):
    df = _airbnb_like(spark, n=1500)
    si = StringIndexer(inputCols=["neighbourhood_cleansed"], outputCols=["nIdx"], handleInvalid="skip")
    va = VectorAssembler(inputCols=["nIdx", "accommodates", "beds"], outputCol="features")
    rf = RandomForestRegressor(labelCol="price", maxBins=40, seed=42)
    grid = ParamGridBuilder().addGrid(rf.maxDepth, [2, 5]).addGrid(rf.numTrees, [5, 10]).build()
    assert len(grid) == 4
    ev = RegressionEvaluator(labelCol="price")
    cv = CrossValidator(estimator=rf, evaluator=ev, estimatorParamMaps=grid, numFolds=3, seed=42, parallelism=4)
    pm = Pipeline(stages=[si, va, cv]).fit(df)
    cvm = pm.stages[-1]
    best = cvm.bestModel
    assert best.getMaxDepth() == 5
    metrics = list(zip(cvm.getEstimatorParamMaps(), cvm.avgMetrics))
    assert len(metrics) == 4
    path = str(tmp_path / "cvpm")
    pm.write().overwrite().save(path)
    again = PipelineModel.load(path)
    a = pm.transform(df).select("prediction").toPandas().prediction.values
    b = again.transform(df).select("prediction").toPandas().prediction.values
    np.testing.assert_array_equal(a, b)
    tvs = TrainValidationSplit(estimator=Pipeline(stages=[si, va, rf]), estimatorParamMaps=grid, evaluator=ev,
                               trainRatio=0.75, seed=1).fit(df)
    assert len(tvs.validationMetrics) == 4


def test_param_copy_coerces_floats(spark):
    """ML 08:97: hp.quniform yields floats; copy() must coerce integral floats."""
    rf = RandomForestRegressor()
    p = Pipeline(stages=[rf])
    p2 = p.copy({rf.maxDepth: 3.0, rf.numTrees: 57.0})
    st = p2.getStages()[0]
    assert st.getMaxDepth() == 3 and isinstance(st.getMaxDepth(), int)
    assert st.getNumTrees() == 57
    assert "maxDepth" in rf.explainParams()
    assert rf.getMaxDepth() == 5


def test_standard_scaler(spark):
    df, X, y = _reg_frame(spark, n=500)
    vdf = VectorAssembler(inputCols=[f"x{i}" for i in range(5)], outputCol="f").transform(df)
    out = StandardScaler(inputCol="f", outputCol="s", withMean=True, withStd=True).fit(vdf).transform(vdf)
    S = np.stack([r.s.toArray() for r in out.select("s").collect()])
    np.testing.assert_allclose(S.mean(0), 0, atol=1e-6)
    np.testing.assert_allclose(S.std(0, ddof=1), 1, atol=1e-5)


def test_linear_regression_standard_errors_ols(spark):
    """coefficientStandardErrors / tValues (computed on first access) equal the textbook OLS values
    sqrt(diag(sigma^2 (A^T A)^-1)) for [X | 1]."""
    import numpy as np
    import torch
    from cdnaml.models.regression import LinearRegression
    rng = np.random.default_rng(0)
    n, d = 500, 3
    X = rng.standard_normal((n, d))
    y = X @ np.array([1.5, -2.0, 0.5]) + 3.0 + rng.standard_normal(n) * 0.3
    df = spark.createDataFrameFromLocalTensors({"features": torch.from_numpy(X).float(),
                                                "label": torch.from_numpy(y)})
    m = LinearRegression(gramPrecision="fp32").fit(df)
    Xf = X.astype(np.float32).astype(np.float64)
    A = np.hstack([Xf, np.ones((n, 1))])
    beta, *_ = np.linalg.lstsq(A, y, rcond=None)
    sigma2 = ((y - A @ beta) ** 2).sum() / (n - d - 1)
    se = np.sqrt(np.diag(np.linalg.inv(A.T @ A)) * sigma2)
    np.testing.assert_allclose(m.summary.coefficientStandardErrors, se, rtol=1e-3)
    np.testing.assert_allclose(m.summary.tValues, beta / se, rtol=1e-3)
