import pytest
"""Parity flows for the MLOps / bridge notebooks: ML 04 MLflow Tracking, ML 05 Registry, ML 08 Hyperopt,
ML 09 AutoML, ML 10 Feature Store, ML 12 Pandas UDFs, ML 14 Koalas, MLE 00 Deployment (SURVEY Appendix A)."""
import os

import numpy as np
import pandas as pd


def _sf(ds, name):
    return os.path.join(ds, "airbnb", "sf-listings", name)


def _airbnb(nb):
    spark, ds, _ = nb
    return spark, spark.read.format("delta").load(_sf(ds, "sf-listings-2019-03-06-clean.delta"))


def test_ml04_mlflow_tracking(nb):
    """ML 04:77-260 -- three runs (single feature, all features via RFormula, log price + a figure),
    search_runs ordered by a metric, client queries, load_model round trip."""
    spark, df = _airbnb(nb)
    import mlflow
    import mlflow.spark
    from mlflow.tracking import MlflowClient
    from pyspark.ml import Pipeline
    from pyspark.ml.feature import RFormula, VectorAssembler
    from pyspark.ml.regression import LinearRegression
    from pyspark.ml.evaluation import RegressionEvaluator

    mlflow.set_experiment("/parity/ml04")
    train, test = df.randomSplit([0.8, 0.2], seed=42)
    ev = RegressionEvaluator(predictionCol="prediction", labelCol="price")
    with mlflow.start_run(run_name="LR-Single-Feature") as run1:
        pipe = Pipeline(stages=[VectorAssembler(inputCols=["bedrooms"], outputCol="features"),
                                LinearRegression(featuresCol="features", labelCol="price")])
        m1 = pipe.fit(train)
        mlflow.spark.log_model(m1, "model")
        mlflow.log_param("label", "price")
        mlflow.log_metric("rmse", ev.evaluate(m1.transform(test)))
    with mlflow.start_run(run_name="LR-All-Features"):
        m2 = Pipeline(stages=[RFormula(formula="price ~ .", featuresCol="features", labelCol="price",
                                       handleInvalid="skip"),
                              LinearRegression(labelCol="price", featuresCol="features")]).fit(train)
        mlflow.log_metric("rmse", ev.evaluate(m2.transform(test)))
    with mlflow.start_run(run_name="LR-Log-Price"):
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
        fig = plt.figure()
        plt.hist(df.select("price").toPandas().price.values, bins=20)
        mlflow.log_figure(fig, "price_hist.png")
        mlflow.log_metric("rmse", 1.0)
    runs = mlflow.search_runs(order_by=["metrics.rmse ASC"])
    assert len(runs) >= 3 and runs["metrics.rmse"].is_monotonic_increasing
    client = MlflowClient()
    r = client.get_run(run1.info.run_id)
    assert r.data.params["label"] == "price" and "rmse" in r.data.metrics
    loaded = mlflow.spark.load_model(f"runs:/{run1.info.run_id}/model")
    a = loaded.transform(test).select("prediction").toPandas().prediction.values
    b = m1.transform(test).select("prediction").toPandas().prediction.values
    assert np.allclose(a, b)


def test_ml05_model_registry(nb):
    """ML 05:60-331 / L05:47-428 -- sklearn model logged and registered, stage transitions with
    archive_existing_versions, description update, pyfunc load of a stage, version deletion."""
    spark, ds, _ = nb
    import mlflow
    import mlflow.sklearn
    from mlflow.tracking import MlflowClient
    from sklearn.linear_model import LinearRegression as SkLR, Ridge

    pdf = pd.read_csv(_sf(ds, "airbnb-cleaned-mlflow.csv").replace("dbfs:/", "/dbfs/"))  # ML 05:69
    X, y = pdf.drop(["price"], axis=1), pdf["price"]
    name = "parity_ml05"
    with mlflow.start_run(run_name="LR Model") as run:
        mlflow.sklearn.log_model(SkLR().fit(X, y), "model")
    v1 = mlflow.register_model(f"runs:/{run.info.run_id}/model", name)
    client = MlflowClient()
    client.update_registered_model(name=name, description="parity registry flow")
    client.transition_model_version_stage(name=name, version=v1.version, stage="Production")
    assert client.get_model_version(name, v1.version).current_stage == "Production"
    with mlflow.start_run(run_name="Ridge Model") as run2:
        mlflow.sklearn.log_model(Ridge(alpha=10).fit(X, y), "model", registered_model_name=name)
    v2 = client.get_latest_versions(name, stages=["None"])[0]
    client.transition_model_version_stage(name=name, version=v2.version, stage="Production",
                                          archive_existing_versions=True)
    assert client.get_model_version(name, v1.version).current_stage == "Archived"
    prod = mlflow.pyfunc.load_model(f"models:/{name}/Production")
    assert prod.predict(X.head(5)).shape == (5,)
    client.transition_model_version_stage(name=name, version=v1.version, stage="Archived")
    client.delete_model_version(name=name, version=v1.version)
    assert [v.version for v in client.search_model_versions(f"name='{name}'")] == [v2.version]
    assert run2.info.run_id != run.info.run_id


def test_ml08_hyperopt(nb):
    """ML 08:46-170 / L08:31-130 -- objective refitting a pipeline copy, quniform space, fmin TPE with Trials,
    refit on the union; SparkTrials over sklearn cross_val_score with hp.choice returning an index."""
    spark, df = _airbnb(nb)
    from hyperopt import SparkTrials, STATUS_OK, Trials, fmin, hp, tpe
    from pyspark.ml import Pipeline
    from pyspark.ml.feature import StringIndexer, VectorAssembler
    from pyspark.ml.regression import RandomForestRegressor
    from pyspark.ml.evaluation import RegressionEvaluator
    from sklearn.ensemble import RandomForestRegressor as SkRF
    from sklearn.model_selection import cross_val_score

    train, val = df.randomSplit([0.8, 0.2], seed=42)
    cats = [c for c, t in train.dtypes if t == "string"]
    idx = [c + "Index" for c in cats]
    nums = [c for c, t in train.dtypes if t == "double" and c != "price"]
    rf = RandomForestRegressor(labelCol="price", maxBins=40, seed=42)
    pipe = Pipeline(stages=[StringIndexer(inputCols=cats, outputCols=idx, handleInvalid="skip"),
                            VectorAssembler(inputCols=idx + nums, outputCol="features"), rf])
    ev = RegressionEvaluator(labelCol="price")

    def objective(params):
        est = pipe.copy({rf.maxDepth: int(params["max_depth"]), rf.numTrees: int(params["num_trees"])})
        return ev.evaluate(est.fit(train).transform(val))

    space = {"max_depth": hp.quniform("max_depth", 2, 5, 1), "num_trees": hp.quniform("num_trees", 5, 15, 1)}
    trials = Trials()
    best = fmin(fn=objective, space=space, algo=tpe.suggest, max_evals=4, trials=trials,
                rstate=np.random.default_rng(42))
    assert len(trials.trials) == 4 and 2 <= best["max_depth"] <= 5
    final = pipe.copy({rf.maxDepth: int(best["max_depth"]), rf.numTrees: int(best["num_trees"])})
    assert ev.evaluate(final.fit(train.union(val)).transform(val)) > 0

    pdf = df.select(*nums, "price").toPandas()

    def sk_objective(params):
        model = SkRF(n_estimators=int(params["n"]), max_depth=[3, 5][params["depth"]], random_state=0)
        return {"loss": -cross_val_score(model, pdf[nums], pdf["price"], cv=3).mean(), "status": STATUS_OK}

    best2 = fmin(fn=sk_objective, space={"n": hp.quniform("n", 5, 10, 1), "depth": hp.choice("depth", [0, 1])},
                 algo=tpe.suggest, max_evals=4, trials=SparkTrials(parallelism=2),
                 rstate=np.random.default_rng(0))
    assert best2["depth"] in (0, 1)                                      # hp.choice returns the index


@pytest.mark.slow
def test_ml09_automl(nb):
    """ML 09:29-90 -- automl.regress, best trial's run id, pyfunc.spark_udf predictions, RMSE."""
    spark, df = _airbnb(nb)
    import mlflow
    from databricks import automl
    from pyspark.ml.evaluation import RegressionEvaluator

    train, test = df.randomSplit([0.8, 0.2], seed=42)
    summary = automl.regress(train, target_col="price", primary_metric="rmse", timeout_minutes=5, max_trials=3)
    run_id = summary.best_trial.mlflow_run_id
    assert run_id
    predict = mlflow.pyfunc.spark_udf(spark, f"runs:/{run_id}/model")
    feats = [c for c in test.columns if c != "price"]
    pred = test.withColumn("prediction", predict(*feats))
    assert RegressionEvaluator(labelCol="price").evaluate(pred) > 0


def test_ml10_feature_store(nb):
    """ML 10:45-348 -- monotonically_increasing_id index, feature table create / write / read, FeatureLookup
    training set, fs.log_model + score_batch, overwrite with a new column."""
    spark, df = _airbnb(nb)
    from databricks import feature_store
    from databricks.feature_store import FeatureLookup
    from pyspark.sql.functions import monotonically_increasing_id
    from sklearn.ensemble import RandomForestRegressor as SkRF

    df = df.coalesce(1).withColumn("index", monotonically_increasing_id())
    nums = [c for c, t in df.dtypes if t == "double" and c != "price"][:6]
    fs = feature_store.FeatureStoreClient()
    table = "parity_ml10.airbnb_features"
    spark.sql("CREATE DATABASE IF NOT EXISTS parity_ml10")
    fs.create_table(name=table, primary_keys=["index"], df=df.select("index", *nums), description="parity")
    assert fs.read_table(name=table).count() == df.count()
    lookups = [FeatureLookup(table_name=table, feature_names=nums, lookup_key="index")]
    ts = fs.create_training_set(df.select("index", "price"), lookups, label="price", exclude_columns="index")
    tdf = ts.load_df().toPandas()
    assert set(nums) <= set(tdf.columns)
    model = SkRF(n_estimators=5, random_state=0).fit(tdf[nums], tdf["price"])
    import mlflow
    with mlflow.start_run():
        fs.log_model(model, "feature-store-model", flavor=mlflow.sklearn, training_set=ts,
                     registered_model_name="parity_ml10_model")
    scored = fs.score_batch("models:/parity_ml10_model/1", df.select("index"))
    assert "prediction" in scored.columns and scored.count() == df.count()
    from pyspark.sql.functions import col
    fs.write_table(name=table, df=df.select("index", *nums).withColumn("extra", col(nums[0]) * 2),
                   mode="overwrite")
    assert "extra" in fs.read_table(name=table).columns


def test_ml12_pandas_udfs(nb):
    """ML 12:27-143 / L12:33-96 -- sklearn model logged, scalar pandas UDF, iterator UDF, mapInPandas with a
    DDL schema, pyfunc.spark_udf -- all give the same predictions."""
    spark, df = _airbnb(nb)
    import mlflow
    import mlflow.sklearn
    from pyspark.sql.functions import pandas_udf
    from sklearn.ensemble import RandomForestRegressor as SkRF
    from typing import Iterator, Tuple

    nums = [c for c, t in df.dtypes if t == "double" and c != "price"][:5]
    pdf = df.select(*nums, "price").toPandas()
    with mlflow.start_run(run_name="sklearn-rf") as run:
        model = SkRF(n_estimators=10, max_depth=5, random_state=0).fit(pdf[nums], pdf["price"])
        mlflow.sklearn.log_model(model, "random-forest-model")
    uri = f"runs:/{run.info.run_id}/random-forest-model"
    ref = model.predict(pdf[nums])

    @pandas_udf("double")
    def predict(*args: pd.Series) -> pd.Series:
        m = mlflow.sklearn.load_model(uri)
        return pd.Series(m.predict(pd.concat(args, axis=1).set_axis(nums, axis=1)))

    @pandas_udf("double")
    def predict_iter(it: Iterator[Tuple[pd.Series, ...]]) -> Iterator[pd.Series]:
        m = mlflow.sklearn.load_model(uri)
        for feats in it:
            yield pd.Series(m.predict(pd.concat(feats, axis=1).set_axis(nums, axis=1)))

    def predict_map(it):
        m = mlflow.sklearn.load_model(uri)
        for batch in it:
            yield pd.DataFrame({"prediction": m.predict(batch[nums])})

    sel = df.select(*nums)
    a = sel.withColumn("p", predict(*nums)).toPandas().p.values
    b = sel.withColumn("p", predict_iter(*nums)).toPandas().p.values
    c = sel.mapInPandas(predict_map, schema="prediction double").toPandas().prediction.values
    d = sel.withColumn("p", mlflow.pyfunc.spark_udf(spark, uri)(*nums)).toPandas().p.values
    for v in (a, b, c, d):
        assert np.allclose(v, ref)


def test_ml14_koalas(nb):
    """ML 14:85-194 -- read via pandas / koalas / Spark, default index, conversions, value_counts, ks.sql."""
    spark, ds, _ = nb
    import databricks.koalas as ks

    path = _sf(ds, "sf-listings-2019-03-06-clean.parquet")
    kdf = ks.read_parquet(path)
    sdf = spark.read.parquet(path)
    assert len(kdf) == sdf.count()
    assert list(kdf.head(3).index) == [0, 1, 2]
    k2 = sdf.to_koalas()
    assert len(k2) == len(kdf)
    assert isinstance(kdf.to_pandas(), pd.DataFrame) and kdf.to_spark().count() == len(kdf)
    vc = kdf["room_type"].value_counts()
    assert int(vc.sum()) == len(kdf)
    out = ks.sql("SELECT COUNT(*) AS c FROM {kdf} WHERE price > 100", kdf=kdf)
    assert int(out["c"].to_numpy()[0]) == int((kdf["price"] > 100).sum())


def test_mle00_deployment_streaming(nb, tmp_path):
    """MLE 00:36-117 -- load a saved PipelineModel, readStream parquet one file per trigger, transform,
    memory sink with a checkpoint, SQL on the sink table, stop."""
    spark, ds, _ = nb
    from pyspark.ml import PipelineModel

    pm = PipelineModel.load(_sf(ds, "models/sf-listings-2019-03-06/pipeline_model"))
    src = _sf(ds, "sf-listings-2019-03-06-clean-100p.parquet")
    schema = spark.read.parquet(src).schema
    stream = spark.readStream.schema(schema).option("maxFilesPerTrigger", 1).parquet(src)
    q = (pm.transform(stream).select("price", "prediction").writeStream.queryName("parity_preds")
         .format("memory").option("checkpointLocation", str(tmp_path / "ckpt")).outputMode("append").start())
    q.processAllAvailable()
    n = spark.sql("SELECT COUNT(*) AS c FROM parity_preds").first().c
    q.stop()
    assert n == spark.read.parquet(src).count()
    assert not q.isActive
