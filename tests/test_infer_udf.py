"""Config 5 through the reference's API (ML 12 - Inference with Pandas UDFs.py:73-143,
ML 09 - AutoML.py:78-82, Solutions/Labs/ML 12L - Pandas UDF Lab.py:78-96): a forest logged with the tracking
flavour and loaded with ``spark_udf(spark, "runs:/...")`` predicts a STREAMED frame batch by batch through the
same native path as ``model.transform`` -- one plan and one forest predictor for every batch, no pandas
conversion, graph-replayed predict on the GPU -- and gives the transform's predictions bit for bit."""
import numpy as np
import pytest
import torch

from cdnaml import tracking as mlflow


@pytest.fixture
def tracking(tmp_path):
    mlflow.set_tracking_uri(str(tmp_path / "mlruns"))
    mlflow.set_experiment("/Users/me/infer")
    yield tmp_path
    while mlflow.active_run():
        mlflow.end_run()
    mlflow.set_tracking_uri(None)


def test_spark_udf_streamed_forest(tracking, spark, monkeypatch):
    from cdnaml.ml import Pipeline
    from cdnaml.ml.regression import RandomForestRegressor
    from cdnaml.models.inference import predictor_for
    from cdnaml.sql import batch as B
    rng = np.random.default_rng(3)
    d, rows, nchunks = 16, 4096, 5
    Xtr = rng.normal(size=(20000, d)).astype(np.float32)
    ytr = Xtr[:, 0] * 2 - Xtr[:, 1] + np.sin(Xtr[:, 2])
    train = spark.createDataFrameFromLocalTensors({"features": torch.from_numpy(Xtr).to(spark.device),
                                                   "label": torch.from_numpy(ytr).double().to(spark.device)})
    pm = Pipeline(stages=[RandomForestRegressor(numTrees=8, maxDepth=5, maxBins=32, seed=1)]).fit(train)
    with mlflow.start_run() as run:
        mlflow.spark.log_model(pm, "model")
    udf = mlflow.pyfunc.spark_udf(spark, f"runs:/{run.info.run_id}/model")
    X = rng.normal(size=(rows * nchunks, d)).astype(np.float32)

    def chunks():
        for i in range(nchunks):
            yield {"features": X[i * rows:(i + 1) * rows]}
    df = spark.createDataFrameFromChunks(chunks, rows)
    conv = {"n": 0}
    orig = B.Batch.to_pandas

    def counted(self):
        conv["n"] += 1
        return orig(self)
    monkeypatch.setattr(B.Batch, "to_pandas", counted)
    got, ref = [], []
    df.withColumn("prediction", udf("features")).foreachBatch(
        lambda b: got.append(b.columns["prediction"].values.cpu().clone()))
    pm.transform(df).foreachBatch(lambda b: ref.append(b.columns["prediction"].values.cpu().clone()))
    assert conv["n"] == 0  # no pandas round trip for our flavour
    assert udf.batches == nchunks and udf.plans_built == 1  # one plan, re-run per batch
    got, ref = torch.cat(got), torch.cat(ref)
    assert got.dtype == torch.float64 and torch.equal(got, ref)
    pr = predictor_for(udf.pm.stages[-1], "value", [0.0])
    if spark.device.type == "cuda":
        assert pr.replays > 0  # the staging buffers' predicts are replayed HIP graphs


def test_spark_udf_reentrant_threads(tracking, spark):
    """One ``spark_udf`` evaluated over two different frames from 4 threads at once gives the serial results bit
    for bit (the current batch is per thread, not instance state: ADVICE r5; ML 12:73-143 under
    CrossValidator(parallelism=4)-style thread pools)."""
    from concurrent.futures import ThreadPoolExecutor

    from cdnaml.ml import Pipeline
    from cdnaml.ml.regression import RandomForestRegressor
    rng = np.random.default_rng(5)
    d = 8
    Xtr = rng.normal(size=(6000, d)).astype(np.float32)
    ytr = Xtr[:, 0] * 2 - Xtr[:, 1] + np.sin(Xtr[:, 2])
    train = spark.createDataFrameFromLocalTensors({"features": torch.from_numpy(Xtr).to(spark.device),
                                                   "label": torch.from_numpy(ytr).double().to(spark.device)})
    pm = Pipeline(stages=[RandomForestRegressor(numTrees=6, maxDepth=5, maxBins=32, seed=2)]).fit(train)
    with mlflow.start_run() as run:
        mlflow.spark.log_model(pm, "model")
    udf = mlflow.pyfunc.spark_udf(spark, f"runs:/{run.info.run_id}/model")
    frames = []
    for seed, n in ((11, 3000), (12, 1700)):
        X = np.random.default_rng(seed).normal(size=(n, d)).astype(np.float32)
        frames.append(spark.createDataFrameFromLocalTensors({"features": torch.from_numpy(X).to(spark.device)}))

    def run_one(i):
        out = frames[i % 2].withColumn("prediction", udf("features")).select("prediction")._plan.execute()
        return torch.cat([b.columns["prediction"].values.cpu() for b in out])
    serial = [run_one(0), run_one(1)]
    import time
    orig = udf._plan_for

    def slow_plan_for(sess, part):  # widen the window between "batch set" and "plan executes"
        time.sleep(0.01)
        return orig(sess, part)
    udf._plan_for = slow_plan_for
    with ThreadPoolExecutor(4) as ex:
        got = list(ex.map(run_one, range(16)))
    for i, g in enumerate(got):
        assert torch.equal(g, serial[i % 2]), i
    assert udf.plans_built == 1
