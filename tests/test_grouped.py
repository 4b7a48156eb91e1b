"""Many models (ML 13 - Training with Pandas Function API.py:73-161): concurrent applyInPandas groups and
the batched GroupedEstimator (one forest pass for all groups, bit-identical to per-group fits)."""
import numpy as np
import pandas as pd
import pytest

from cdnaml.utils.synthetic import forest_digest


def _iot(spark, n=6000, groups=6, seed=0):
    """ML 13's IoT table: device_id = id % groups, feature_k = rand() * k, label = sum(features) + rand()."""
    rng = np.random.default_rng(seed)
    ids = np.arange(n)
    pdf = pd.DataFrame({"record_id": ids, "device_id": ids % groups})
    for k in (1, 2, 3):
        pdf[f"feature_{k}"] = rng.random(n) * k
    pdf["label"] = pdf[["feature_1", "feature_2", "feature_3"]].sum(1) + rng.random(n)
    from cdnaml.ml.feature import VectorAssembler
    return VectorAssembler(inputCols=["feature_1", "feature_2", "feature_3"], outputCol="features").transform(
        spark.createDataFrame(pdf))


@pytest.mark.parametrize("kind", ["rf", "dt", "rfc"])
def test_grouped_estimator_equals_per_group_fits(spark, kind):
    from cdnaml.ml.classification import RandomForestClassifier
    from cdnaml.ml.grouped import GroupedEstimator
    from cdnaml.ml.regression import DecisionTreeRegressor, RandomForestRegressor
    from cdnaml.models.tree.fused import FusedTreeTuner
    from cdnaml.sql import functions as F
    df = _iot(spark)
    if kind == "rfc":
        df = df.withColumn("label", (F.col("label") > 3.5).cast("double"))
    est = {"rf": RandomForestRegressor(numTrees=5, maxDepth=4, seed=3),
           "dt": DecisionTreeRegressor(maxDepth=5),
           "rfc": RandomForestClassifier(numTrees=4, maxDepth=3, seed=5)}[kind]
    gm = GroupedEstimator(estimator=est, groupCol="device_id").fit(df)
    assert sorted(gm.models) == list(range(6))
    tuner = FusedTreeTuner(est, [{}], df)
    keys = df.select("device_id").toPandas().device_id.to_numpy()
    import torch
    dev = tuner.prep(tuner.ests[0])[1].bins.device
    for g in range(6):
        mask = torch.from_numpy(keys == g).to(dev)
        T = est.getNumTrees() if kind != "dt" else 1
        alone, _ = tuner.fit_forest_mask(tuner.ests[0], T, est.getMaxDepth(), mask)
        assert forest_digest(gm.models[g]._forest) == forest_digest(alone), g
    # each row is scored by its own group's model
    pred = gm.transform(df).select("device_id", "features", "prediction").toPandas()
    one = pred[pred.device_id == 2]
    sub = df.filter(F.col("device_id") == 2)
    ref = gm.models[2].transform(sub).select("prediction").toPandas().prediction.to_numpy()
    np.testing.assert_allclose(one.prediction.to_numpy(), ref)


def test_apply_in_pandas_concurrent_matches_serial_with_nested_runs(spark, tmp_path):
    """The ML 13 flow: sklearn forest per device inside applyInPandas, logging nested runs; the
    thread-pooled groups give the serial loop's output, in group order, and one child run per device."""
    import cdnaml.tracking as mlflow
    from sklearn.ensemble import RandomForestRegressor as SkRF
    mlflow.set_tracking_uri(str(tmp_path / "mlruns"))
    df = _iot(spark)
    schema = "device_id integer, n_used integer, model_path string, mse float"

    def train_model(pdf):
        device_id = int(pdf["device_id"].iloc[0])
        X, y = pdf[["feature_1", "feature_2", "feature_3"]], pdf["label"]
        rf = SkRF(n_estimators=10, random_state=0).fit(X, y)
        mse = float(((rf.predict(X) - y) ** 2).mean())
        run_id = pdf["run_id"].iloc[0]
        with mlflow.start_run(run_id=run_id):
            with mlflow.start_run(run_name=str(device_id), nested=True) as run:
                mlflow.log_metric("mse", mse)
                path = f"runs:/{run.info.run_id}/{device_id}"
        return pd.DataFrame([[device_id, len(pdf), path, mse]], columns=["device_id", "n_used", "model_path", "mse"])

    from cdnaml.sql import functions as F
    with mlflow.start_run(run_name="Training session for all devices") as run:
        tagged = df.withColumn("run_id", F.lit(run.info.run_id))
        spark.conf.set("cdnaml.applyInPandas.parallelism", "1")
        serial = tagged.groupby("device_id").applyInPandas(train_model, schema=schema).toPandas()
        spark.conf.set("cdnaml.applyInPandas.parallelism", "6")
        par = tagged.groupby("device_id").applyInPandas(train_model, schema=schema).toPandas()
    assert serial.device_id.tolist() == par.device_id.tolist() == list(range(6))
    np.testing.assert_allclose(serial.mse.to_numpy(), par.mse.to_numpy())
    runs = mlflow.search_runs(experiment_ids=[run.info.experiment_id])
    child = runs[runs["tags.mlflow.parentRunId"] == run.info.run_id]
    assert len(child) == 12
