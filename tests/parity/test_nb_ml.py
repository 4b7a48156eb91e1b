"""Parity flows for the MLlib notebooks: ML 02/03 Linear Regression (+ labs), ML 06 Decision Trees, ML 07 / L07
Random Forests + tuning, ML 11 XGBoost, ML 13 Pandas Function API, MLE 01 ALS, MLE 02 K-Means, MLE 03 Logistic
Regression."""
import os

import numpy as np
import pytest


def _airbnb(nb):
    spark, ds, _ = nb
    df = spark.read.format("delta").load(os.path.join(ds, "airbnb", "sf-listings",
                                                      "sf-listings-2019-03-06-clean.delta"))
    return spark, df


def test_ml02_linear_regression_i(nb):
    """ML 02:38-151 / L02:40-64 -- randomSplit changes with the partitioning, LR on a non-vector column fails,
    VectorAssembler + LR, coefficients / intercept, RMSE and R^2."""
    spark, df = _airbnb(nb)
    from pyspark.ml.feature import VectorAssembler
    from pyspark.ml.regression import LinearRegression
    from pyspark.ml.evaluation import RegressionEvaluator

    train, test = df.randomSplit([0.8, 0.2], seed=42)
    train2, _ = df.repartition(24).randomSplit([0.8, 0.2], seed=42)
    assert train.count() + test.count() == df.count()
    assert abs(train2.count() - train.count()) < 0.05 * df.count()
    with pytest.raises(Exception):
        LinearRegression(featuresCol="bedrooms", labelCol="price").fit(train)
    va = VectorAssembler(inputCols=["bedrooms"], outputCol="features")
    lr_model = LinearRegression(featuresCol="features", labelCol="price").fit(va.transform(train))
    assert len(lr_model.coefficients) == 1 and np.isfinite(lr_model.intercept)
    pred = lr_model.transform(va.transform(test))
    ev = RegressionEvaluator(predictionCol="prediction", labelCol="price")
    rmse, r2 = ev.setMetricName("rmse").evaluate(pred), ev.setMetricName("r2").evaluate(pred)
    # the coefficients of ML 02:112-123 against an fp64 least-squares solve of the same design (Double vectors)
    tr = train.select("bedrooms", "price").toPandas()
    ref = np.linalg.lstsq(np.c_[tr.bedrooms.values, np.ones(len(tr))], tr.price.values, rcond=None)[0]
    np.testing.assert_allclose([lr_model.coefficients[0], lr_model.intercept], ref, rtol=1e-9)
    # RMSE / R^2 of the evaluator against the textbook formulas on the collected predictions
    pp = pred.select("price", "prediction").toPandas()
    e = pp.price.values - pp.prediction.values
    np.testing.assert_allclose(rmse, np.sqrt(np.mean(e ** 2)), rtol=1e-12)
    np.testing.assert_allclose(r2, 1 - np.sum(e ** 2) / np.sum((pp.price.values - pp.price.mean()) ** 2), rtol=1e-10)


def test_ml03_linear_regression_ii(nb, tmp_path):
    """ML 03:54-157 / L03:49-107 -- StringIndexer + OHE + VectorAssembler + LR Pipeline, save / load identical,
    RFormula, log(price) model exponentiated back beats the raw-price model's R^2 sign."""
    spark, df = _airbnb(nb)
    from pyspark.sql.functions import col, exp, log
    from pyspark.ml import Pipeline, PipelineModel
    from pyspark.ml.feature import OneHotEncoder, RFormula, StringIndexer, VectorAssembler
    from pyspark.ml.regression import LinearRegression
    from pyspark.ml.evaluation import RegressionEvaluator

    train, test = df.randomSplit([0.8, 0.2], seed=42)
    cats = [c for c, t in train.dtypes if t == "string"]
    idx = [c + "Index" for c in cats]
    ohe = [c + "OHE" for c in cats]
    nums = [c for c, t in train.dtypes if t == "double" and c != "price"]
    stages = [StringIndexer(inputCols=cats, outputCols=idx, handleInvalid="skip"),
              OneHotEncoder(inputCols=idx, outputCols=ohe),
              VectorAssembler(inputCols=ohe + nums, outputCol="features"),
              LinearRegression(labelCol="price", featuresCol="features")]
    model = Pipeline(stages=stages).fit(train)
    path = str(tmp_path / "lr_pipeline")
    model.write().overwrite().save(path)
    loaded = PipelineModel.load(path)
    a = model.transform(test).select("prediction").toPandas()
    b = loaded.transform(test).select("prediction").toPandas()
    assert np.array_equal(a.prediction.values, b.prediction.values)
    rf = RFormula(formula="price ~ .", featuresCol="features", labelCol="price", handleInvalid="skip")
    rmodel = Pipeline(stages=[rf, LinearRegression(labelCol="price", featuresCol="features")]).fit(train)
    ev = RegressionEvaluator(labelCol="price", predictionCol="prediction", metricName="r2")
    assert ev.evaluate(rmodel.transform(test)) > 0
    # ML 03:86-88 prints these coefficients: the one-hot design (cond ~1e6) against fp64 least squares
    des = rmodel.stages[0].transform(train).select("features", "price").toPandas()
    Xd = np.stack([np.asarray(v.toArray()) for v in des.features])
    A = np.c_[Xd, np.ones(len(Xd))]
    ref = np.linalg.lstsq(A, des.price.values, rcond=None)[0]
    got = np.r_[rmodel.stages[-1].coefficients.toArray(), rmodel.stages[-1].intercept]
    np.testing.assert_allclose(A @ got, A @ ref, rtol=0, atol=1e-7 * np.abs(des.price.values).max())
    lt = train.withColumn("log_price", log(col("price")))
    lrf = RFormula(formula="log_price ~ . - price", featuresCol="features", labelCol="log_price",
                   handleInvalid="skip")
    lmodel = Pipeline(stages=[lrf, LinearRegression(labelCol="log_price", featuresCol="features")]).fit(lt)
    back = lmodel.transform(test.withColumn("log_price", log(col("price")))) \
        .withColumn("prediction", exp(col("prediction")))
    assert ev.evaluate(back) > 0


def test_ml06_decision_trees(nb):
    """ML 06:42-209 -- maxBins below the categorical cardinality raises, setMaxBins(40) fits, featureImportances
    by name (top-k), RMSE / R^2 beat the mean baseline."""
    spark, df = _airbnb(nb)
    from pyspark.sql.functions import avg, lit
    from pyspark.ml import Pipeline
    from pyspark.ml.feature import StringIndexer, VectorAssembler
    from pyspark.ml.regression import DecisionTreeRegressor
    from pyspark.ml.evaluation import RegressionEvaluator

    train, test = df.randomSplit([0.8, 0.2], seed=42)
    cats = [c for c, t in train.dtypes if t == "string"]
    idx = [c + "Index" for c in cats]
    nums = [c for c, t in train.dtypes if t == "double" and c != "price"]
    va = VectorAssembler(inputCols=idx + nums, outputCol="features")
    dt = DecisionTreeRegressor(labelCol="price")
    pipe = Pipeline(stages=[StringIndexer(inputCols=cats, outputCols=idx, handleInvalid="skip"), va, dt])
    with pytest.raises(Exception, match="maxBins"):
        pipe.fit(train)
    dt.setMaxBins(40)
    model = pipe.fit(train)
    imp = model.stages[-1].featureImportances
    names = va.getInputCols()
    top = sorted(zip(names, imp.toArray()), key=lambda kv: -kv[1])[:5]
    assert abs(sum(imp.toArray()) - 1.0) < 1e-9 and top[0][1] > 0
    ev = RegressionEvaluator(labelCol="price", predictionCol="prediction")
    pred = model.transform(test)
    mean = train.select(avg("price")).first()[0]
    assert ev.evaluate(pred) < ev.evaluate(test.withColumn("prediction", lit(mean)))


def test_ml07_random_forest_cross_validation(nb, tmp_path):
    """ML 07:24-167 / L07:42-209 -- explainParams, grid over maxDepth x numTrees, CrossValidator (3 folds,
    seed, parallelism 4) inside a Pipeline, avgMetrics per map, bestModel importances, save / load."""
    spark, df = _airbnb(nb)
    from pyspark.ml import Pipeline, PipelineModel
    from pyspark.ml.feature import StringIndexer, VectorAssembler
    from pyspark.ml.regression import RandomForestRegressor
    from pyspark.ml.tuning import CrossValidator, ParamGridBuilder
    from pyspark.ml.evaluation import RegressionEvaluator

    train, test = df.randomSplit([0.8, 0.2], seed=42)
    cats = [c for c, t in train.dtypes if t == "string"]
    idx = [c + "Index" for c in cats]
    nums = [c for c, t in train.dtypes if t == "double" and c != "price"]
    rf = RandomForestRegressor(labelCol="price", maxBins=40, seed=42)
    assert "maxDepth" in rf.explainParams() and "numTrees" in rf.explainParams()
    grid = ParamGridBuilder().addGrid(rf.maxDepth, [2, 5]).addGrid(rf.numTrees, [5, 10]).build()
    ev = RegressionEvaluator(labelCol="price", predictionCol="prediction")
    cv = CrossValidator(estimator=rf, evaluator=ev, estimatorParamMaps=grid, numFolds=3, seed=42, parallelism=4)
    pipe = Pipeline(stages=[StringIndexer(inputCols=cats, outputCols=idx, handleInvalid="skip"),
                            VectorAssembler(inputCols=idx + nums, outputCol="features"), cv])
    model = pipe.fit(train)
    cvm = model.stages[-1]
    assert len(cvm.avgMetrics) == 4 and all(m > 0 for m in cvm.avgMetrics)
    best = cvm.bestModel
    # the best model carries the argmin map's params (RMSE: smaller is better) and IS the refit of those params
    # on the whole training set (ML 07:112: 4 maps x 3 folds + 1 refit)
    k = int(np.argmin(cvm.avgMetrics))
    bm = cvm.getEstimatorParamMaps()[k]
    assert best.getOrDefault("maxDepth") == bm[rf.maxDepth] and best.getNumTrees == bm[rf.numTrees]
    feats = Pipeline(stages=pipe.getStages()[:2]).fit(train).transform(train)
    refit = rf.copy(bm).fit(feats)
    from cdnaml.utils.synthetic import forest_digest
    assert forest_digest(refit._forest) == forest_digest(best._forest)
    # deeper / larger forests fit this table better: the grid's metrics are not all equal
    assert max(cvm.avgMetrics) > min(cvm.avgMetrics)
    # the same seed reproduces the fold metrics exactly
    cv2 = CrossValidator(estimator=rf, evaluator=ev, estimatorParamMaps=grid, numFolds=3, seed=42, parallelism=2)
    assert cv2.fit(feats).avgMetrics == cvm.avgMetrics
    assert len(best.featureImportances.toArray()) == len(idx + nums)
    path = str(tmp_path / "cv_pipeline")
    model.write().overwrite().save(path)
    a = model.transform(test).select("prediction").toPandas().prediction.values
    b = PipelineModel.load(path).transform(test).select("prediction").toPandas().prediction.values
    assert np.allclose(a, b)
    assert ev.evaluate(model.transform(test)) > 0


@pytest.mark.slow
def test_ml11_xgboost(nb):
    """ML 11:36-103 -- log label, StringIndexer + VectorAssembler + XgboostRegressor pipeline, exp back,
    RMSE / R^2."""
    spark, df = _airbnb(nb)
    from pyspark.sql.functions import col, exp, log
    from pyspark.ml import Pipeline
    from pyspark.ml.feature import StringIndexer, VectorAssembler
    from pyspark.ml.evaluation import RegressionEvaluator
    from sparkdl.xgboost import XgboostRegressor

    train, test = df.withColumn("label", log(col("price"))).randomSplit([0.8, 0.2], seed=42)
    cats = [c for c, t in train.dtypes if t == "string"]
    idx = [c + "Index" for c in cats]
    nums = [c for c, t in train.dtypes if t == "double" and c not in ("price", "label")]
    xgb = XgboostRegressor(n_estimators=30, learning_rate=0.1, max_depth=4, random_state=42, missing=0)
    model = Pipeline(stages=[StringIndexer(inputCols=cats, outputCols=idx, handleInvalid="skip"),
                             VectorAssembler(inputCols=idx + nums, outputCol="features"), xgb]).fit(train)
    pred = model.transform(test).withColumn("prediction", exp(col("prediction")))
    ev = RegressionEvaluator(labelCol="price", predictionCol="prediction")
    assert ev.setMetricName("r2").evaluate(pred) > 0 and ev.setMetricName("rmse").evaluate(pred) > 0


def test_ml13_pandas_function_api(nb):
    """ML 13:35-162 -- synthetic IoT, applyInPandas trains one sklearn model per device with nested runs,
    join back, applyInPandas applies each device's model."""
    spark, _, _ = nb
    import mlflow
    import pandas as pd
    from sklearn.ensemble import RandomForestRegressor as SkRF
    from cdnaml.utils import datasets as D

    df = D.iot(spark, 2000)
    assert df.select("device_id").distinct().count() == 10

    def train_model(pdf: pd.DataFrame) -> pd.DataFrame:
        X = pdf[["feature_1", "feature_2", "feature_3"]]
        m = SkRF(n_estimators=10, max_depth=4, random_state=0).fit(X, pdf["label"])
        with mlflow.start_run(nested=True):
            mlflow.log_param("device", str(pdf["device_id"].iloc[0]))
        return pd.DataFrame({"device_id": [pdf["device_id"].iloc[0]], "n_used": [len(pdf)],
                             "mse": [float(((m.predict(X) - pdf["label"]) ** 2).mean())]})

    with mlflow.start_run(run_name="ML13 parity"):
        out = df.groupby("device_id").applyInPandas(train_model,
                                                    schema="device_id int, n_used int, mse double").toPandas()
    assert len(out) == 10 and out.n_used.sum() == 2000
    joined = df.join(spark.createDataFrame(out), on="device_id")
    assert joined.count() == 2000


def test_mle01_als(nb):
    """MLE 01:63-374 -- ratings parquet, split, average-rating baseline, ALS + CrossValidator over rank {4, 12}
    selects the planted rank 12, predictions for a user's unrated movies, SQL top-k."""
    spark, ds, _ = nb
    from pyspark.sql.functions import avg, lit
    from pyspark.ml.recommendation import ALS
    from pyspark.ml.tuning import CrossValidator, ParamGridBuilder
    from pyspark.ml.evaluation import RegressionEvaluator

    ratings = spark.read.parquet(os.path.join(ds, "movielens", "ratings.parquet")).cache()
    train, test = ratings.randomSplit([0.8, 0.2], seed=42)
    ev = RegressionEvaluator(predictionCol="prediction", labelCol="rating", metricName="rmse")
    mean = train.select(avg("rating")).first()[0]
    base = ev.evaluate(test.withColumn("prediction", lit(mean)))
    als = ALS(userCol="userId", itemCol="movieId", ratingCol="rating", maxIter=5, seed=42,
              coldStartStrategy="drop", regParam=0.1)
    assert als.getItemCol() == "movieId" and als.getUserCol() == "userId" and als.getRatingCol() == "rating"
    grid = ParamGridBuilder().addGrid(als.rank, [4, 12]).build()
    cvm = CrossValidator(estimator=als, evaluator=ev, estimatorParamMaps=grid, numFolds=3, seed=42).fit(train)
    assert cvm.bestModel.rank == 12
    assert ev.evaluate(cvm.bestModel.transform(test)) < base
    cvm.bestModel.transform(test).createOrReplaceTempView("als_pred")
    top = spark.sql("SELECT movieId, prediction FROM als_pred ORDER BY prediction DESC LIMIT 25").toPandas()
    assert len(top) == 25 and top.prediction.is_monotonic_decreasing


def test_mle02_kmeans(nb):
    """MLE 02:22-174 -- iris-like blobs, VectorAssembler of 2 features, KMeans(k=3, seed=221), maxIter sweep incl.
    0 (initial centres returned unchanged), clusterCenters."""
    spark, _, _ = nb
    from pyspark.ml.clustering import KMeans
    from pyspark.ml.feature import VectorAssembler

    rng = np.random.default_rng(0)
    pts = np.concatenate([rng.normal(c, 0.3, (50, 2)) for c in ((0, 0), (4, 4), (0, 5))])
    df = spark.createDataFrame([(float(a), float(b)) for a, b in pts], ["x", "y"])
    data = VectorAssembler(inputCols=["x", "y"], outputCol="features").transform(df)
    centres = {}
    for it in (0, 1, 2, 20):
        m = KMeans(k=3, seed=221, maxIter=it).fit(data)
        centres[it] = np.array(m.clusterCenters())
    assert centres[0].shape == (3, 2)
    final = sorted(map(tuple, np.round(centres[20])))
    assert final == sorted([(0.0, 0.0), (4.0, 4.0), (0.0, 5.0)])
    assert not np.allclose(centres[0], centres[20])


def test_mle03_logistic_regression(nb):
    """MLE 03:51-170 -- when() label, always-0 accuracy baseline, RFormula + LogisticRegression, accuracy /
    AUROC / AUPR, regParam x elasticNetParam grid CV inside a Pipeline."""
    spark, df = _airbnb(nb)
    from pyspark.sql.functions import col, lit, when
    from pyspark.ml import Pipeline
    from pyspark.ml.classification import LogisticRegression
    from pyspark.ml.feature import RFormula
    from pyspark.ml.evaluation import BinaryClassificationEvaluator, MulticlassClassificationEvaluator
    from pyspark.ml.tuning import CrossValidator, ParamGridBuilder

    data = df.withColumn("priceClass", when(col("price") >= 150, 1.0).otherwise(0.0))
    train, test = data.randomSplit([0.8, 0.2], seed=42)
    acc = MulticlassClassificationEvaluator(labelCol="priceClass", metricName="accuracy")
    zero = acc.evaluate(test.withColumn("prediction", lit(0.0)))
    rf = RFormula(formula="priceClass ~ . - price", handleInvalid="skip")
    lr = LogisticRegression(labelCol="priceClass")
    grid = ParamGridBuilder().addGrid(lr.regParam, [0.1, 0.2]).addGrid(lr.elasticNetParam, [0.0, 0.5]).build()
    auc = BinaryClassificationEvaluator(labelCol="priceClass")
    cv = CrossValidator(estimator=lr, evaluator=auc, estimatorParamMaps=grid, numFolds=3, seed=42)
    model = Pipeline(stages=[rf, cv]).fit(train)
    pred = model.transform(test)
    assert acc.evaluate(pred) > zero
    assert auc.setMetricName("areaUnderROC").evaluate(pred) > 0.7
    assert 0 < auc.setMetricName("areaUnderPR").evaluate(pred) <= 1
    assert len(model.stages[-1].avgMetrics) == 4
