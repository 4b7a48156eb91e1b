"""MLflow-compatible tracking, registry and flavors (ML04, ML05, L05, ML12)."""
import os

import numpy as np
import pandas as pd
import pytest

from cdnaml import tracking as mlflow
from cdnaml.ml import Pipeline
from cdnaml.ml.evaluation import RegressionEvaluator
from cdnaml.ml.feature import VectorAssembler
from cdnaml.ml.regression import LinearRegression
from cdnaml.tracking import MlflowClient


@pytest.fixture
def tracking(tmp_path):
    mlflow.set_tracking_uri(str(tmp_path / "mlruns"))
    mlflow.set_experiment("/Users/me/exp")
    yield tmp_path
    while mlflow.active_run():
        mlflow.end_run()
    mlflow.set_tracking_uri(None)


def _frame(spark, n=500, seed=0):
    rng = np.random.default_rng(seed)
    pdf = pd.DataFrame({"bedrooms": rng.integers(1, 5, n).astype(float), "x": rng.normal(size=n)})
    pdf["price"] = 50 * pdf.bedrooms + 3 * pdf.x + rng.normal(size=n)
    return spark.createDataFrame(pdf), pdf


def test_runs_params_metrics_artifacts(tracking, spark):
    df, pdf = _frame(spark)
    with mlflow.start_run(run_name="LR-Single-Feature") as run:
        pm = Pipeline(stages=[VectorAssembler(inputCols=["bedrooms"], outputCol="features"),
                              LinearRegression(labelCol="price")]).fit(df)
        mlflow.log_param("label", "price")
        mlflow.log_params({"features": "bedrooms", "n": 500})
        rmse = RegressionEvaluator(labelCol="price").evaluate(pm.transform(df))
        mlflow.log_metric("rmse", rmse)
        for i in range(3):
            mlflow.log_metric("loss", 1.0 / (i + 1), step=i)
        mlflow.spark.log_model(pm, "model", input_example=pdf.head(3))
        mlflow.log_text("hello", "notes/a.txt")
        mlflow.log_dict({"k": 1}, "d.json")
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
        fig, ax = plt.subplots()
        ax.hist(pdf.price)
        mlflow.log_figure(fig, "hist.png")
        rid = run.info.run_id
    r = mlflow.get_run(rid)
    assert r.data.params["label"] == "price" and r.data.params["n"] == "500"
    assert abs(r.data.metrics["rmse"] - rmse) < 1e-12
    assert r.info.status == "FINISHED"
    client = MlflowClient()
    hist = client.get_metric_history(rid, "loss")
    assert [m.step for m in hist] == [0, 1, 2]
    arts = {a.path for a in client.list_artifacts(rid)}
    assert {"model", "hist.png", "d.json", "notes"} <= arts
    loaded = mlflow.spark.load_model(f"runs:/{rid}/model")
    a = loaded.transform(df).select("prediction").toPandas().prediction.values
    b = pm.transform(df).select("prediction").toPandas().prediction.values
    np.testing.assert_array_equal(a, b)
    # MLmodel file on disk
    base = r.info.artifact_uri.replace("file://", "")
    assert os.path.exists(os.path.join(base, "model", "MLmodel"))


def test_only_pipeline_models_can_be_logged(tracking, spark):
    df, _ = _frame(spark)
    lr = LinearRegression(featuresCol="features", labelCol="price").fit(
        VectorAssembler(inputCols=["x"], outputCol="features").transform(df))
    with mlflow.start_run():
        with pytest.raises(Exception):
            mlflow.spark.log_model(lr, "model")


def test_search_runs_filter_and_order(tracking, spark):
    for i, (path, ver) in enumerate([("a.delta", "0"), ("a.delta", "1"), ("b.delta", "0")]):
        with mlflow.start_run(run_name=f"r{i}"):
            mlflow.log_param("data_path", path)
            mlflow.log_param("data_version", ver)
            mlflow.log_metric("rmse", float(i))
    exp = mlflow.get_experiment_by_name("/Users/me/exp")
    runs = mlflow.search_runs(exp.experiment_id)
    assert isinstance(runs, pd.DataFrame) and len(runs) == 3
    f = mlflow.search_runs(exp.experiment_id, filter_string="params.data_path='a.delta' and params.data_version='0'")
    assert len(f) == 1 and f["metrics.rmse"].iloc[0] == 0.0
    g = mlflow.search_runs(exp.experiment_id, filter_string="metrics.rmse > 0.5")
    assert len(g) == 2
    client = MlflowClient()
    latest = client.search_runs(exp.experiment_id, order_by=["attributes.start_time desc"], max_results=1)
    assert latest[0].data.metrics["rmse"] == 2.0
    assert any(e.name == "/Users/me/exp" for e in client.list_experiments())


def test_nested_and_resumed_runs(tracking):
    with mlflow.start_run(run_name="parent") as parent:
        with mlflow.start_run(run_name="child", nested=True) as child:
            mlflow.log_param("device", "3")
        pid = parent.info.run_id
    c = mlflow.get_run(child.info.run_id)
    assert c.data.tags["mlflow.parentRunId"] == pid
    with mlflow.start_run(run_id=child.info.run_id):
        mlflow.log_metric("m", 1.0)
    assert mlflow.get_run(child.info.run_id).data.metrics["m"] == 1.0
    with mlflow.start_run():
        with pytest.raises(Exception):
            mlflow.start_run()


def test_registry_lifecycle(tracking):
    """ML 05: sklearn flavor, register, describe, stage transitions, archive, delete."""
    from sklearn.linear_model import LinearRegression as SkLR
    from sklearn.linear_model import Ridge

    rng = np.random.default_rng(0)
    X = pd.DataFrame(rng.normal(size=(100, 3)), columns=list("abc"))
    y = X.a * 2 + 1
    name = "airbnb_model"
    with pytest.raises(Exception):
        mlflow.register_model("runs:/x/model", "bad/name")
    with mlflow.start_run() as run:
        m1 = SkLR().fit(X, y)
        sig = mlflow.models.infer_signature(X, m1.predict(X))
        mlflow.sklearn.log_model(m1, "model", input_example=X.head(2), signature=sig)
    mv = mlflow.register_model(f"runs:/{run.info.run_id}/model", name)
    assert mv.name == name and int(mv.version) == 1
    client = MlflowClient()
    assert client.get_model_version(name, 1).status == "READY"
    client.update_registered_model(name, description="predicts price")
    client.update_model_version(name, 1, description="v1")
    client.transition_model_version_stage(name, 1, "Production")
    assert client.get_model_version(name, 1).current_stage == "Production"
    with mlflow.start_run() as run2:
        mlflow.sklearn.log_model(Ridge(alpha=0.9).fit(X, y), "model", registered_model_name=name)
    assert int(client.get_latest_versions(name, ["None"])[0].version) == 2
    client.transition_model_version_stage(name, 2, "Production", archive_existing_versions=True)
    assert client.get_model_version(name, 1).current_stage == "Archived"
    pm = mlflow.pyfunc.load_model(f"models:/{name}/Production")
    np.testing.assert_allclose(pm.predict(X), Ridge(alpha=0.9).fit(X, y).predict(X))
    np.testing.assert_allclose(mlflow.pyfunc.load_model(f"models:/{name}/1").predict(X), m1.predict(X))
    vs = client.search_model_versions(f"name = '{name}'")
    assert sorted(int(v.version) for v in vs) == [1, 2]
    client.transition_model_version_stage(name, 1, "Archived")
    client.delete_model_version(name, 1)
    assert [int(v.version) for v in client.search_model_versions(f"name = '{name}'")] == [2]
    client.transition_model_version_stage(name, 2, "Archived")
    client.delete_registered_model(name)
    assert run2 is not None


def test_pyfunc_spark_udf_native(tracking, spark):
    df, pdf = _frame(spark)
    pm = Pipeline(stages=[VectorAssembler(inputCols=["bedrooms", "x"], outputCol="features"),
                          LinearRegression(labelCol="price")]).fit(df)
    with mlflow.start_run() as run:
        mlflow.spark.log_model(pm, "model", input_example=pdf[["bedrooms", "x"]].head(3),
                               signature=mlflow.models.infer_signature(pdf[["bedrooms", "x"]]))
    udf = mlflow.pyfunc.spark_udf(spark, f"runs:/{run.info.run_id}/model")
    out = df.withColumn("prediction", udf("bedrooms", "x")).toPandas()
    ref = pm.transform(df).toPandas().prediction.values
    np.testing.assert_allclose(out.prediction.values, ref)
    pyf = mlflow.pyfunc.load_model(f"runs:/{run.info.run_id}/model")
    np.testing.assert_allclose(pyf.predict(pdf[["bedrooms", "x"]]), ref)


def test_autolog_logs_fits(tracking, spark):
    df, _ = _frame(spark)
    mlflow.pyspark.ml.autolog(log_models=False)
    try:
        with mlflow.start_run() as run:
            LinearRegression(labelCol="price", regParam=0.1).fit(
                VectorAssembler(inputCols=["x"], outputCol="features").transform(df))
        r = mlflow.get_run(run.info.run_id)
        assert r.data.params.get("regParam") == "0.1"
        # engine metrics of the fit
        assert r.data.metrics["engine.fit_ms"] > 0 and "engine.collective_calls" in r.data.metrics
    finally:
        mlflow.pyspark.ml.autolog(disable=True)


def test_tracing_spans_comm_rate_and_roctx(spark):
    """spans carry collective byte counts -> GB/s in the summary; roctx ranges push/pop cleanly
    (a no-op when libroctx64 is absent)."""
    import time as _t
    from cdnaml.utils import tracing
    tracing.reset()
    tracing.enable()
    tracing.enable_roctx(True)
    try:
        with tracing.span("tree.allreduce", cat="comm", bytes=4_000_000):
            _t.sleep(0.002)
        with tracing.span("tree.hist"):
            pass
        st = tracing.stats()
        assert st["tree.allreduce"]["bytes"] == 4e6 and 0 < st["tree.allreduce"]["GB_s"] < 2.1
        assert "GB/s" in tracing.summary()
    finally:
        tracing.enable_roctx(False)
        tracing.disable()
        tracing.reset()
