"""Batch inference engine (models/inference.py): streamed DataFrames over host / device chunks, the
cached device-resident forest predictor and its HIP-graph replays (ML 12 - Inference with Pandas
UDFs.py:73-143, Labs/ML 12L:78-96)."""
import numpy as np
import pytest
import torch


def _model(spark, d=6, n=3000):
    from cdnaml.ml.regression import RandomForestRegressor
    g = torch.Generator().manual_seed(0)
    X = torch.randn(n, d, generator=g)
    y = (X[:, 0] * 2 - X[:, 1] + torch.sin(3 * X[:, 2])).double()
    df = spark.createDataFrameFromLocalTensors({"features": X.to(spark.device), "label": y.to(spark.device)})
    return RandomForestRegressor(numTrees=6, maxDepth=4, seed=3).fit(df)


def _chunks(n_chunks, rows, d, seed=1):
    rng = np.random.default_rng(seed)
    data = [rng.normal(size=(rows, d)).astype(np.float32) for _ in range(n_chunks)]
    data[-1] = data[-1][: rows // 2 + 1]  # a short last chunk
    return data


def test_streamed_transform_matches_materialised(spark):
    model = _model(spark)
    data = _chunks(5, 700, 6)
    df = spark.createDataFrameFromChunks(lambda: ({"features": c} for c in data), max_rows=700)
    assert df._plan.streamable and df.count() == sum(len(c) for c in data)
    got = []
    model.transform(df).foreachBatch(lambda b: got.append(b.columns["prediction"].values.cpu().clone()))
    assert [len(g) for g in got] == [len(c) for c in data]
    full = spark.createDataFrameFromLocalTensors({"features": torch.from_numpy(np.concatenate(data)).to(
        spark.device)})
    ref = model.transform(full).toPandas()["prediction"].to_numpy()
    np.testing.assert_allclose(torch.cat(got).numpy(), ref, rtol=0, atol=0)
    # a streamed source can still be materialised (batches are cloned out of the reused staging buffers)
    mat = model.transform(df).toPandas()["prediction"].to_numpy()
    np.testing.assert_allclose(mat, ref, rtol=0, atol=0)


def test_device_chunks_source(spark):
    from cdnaml.models.inference import device_chunks
    model = _model(spark)
    rows, chunk = 2500, 600
    base = torch.randn(rows, 6, generator=torch.Generator().manual_seed(4)).to(spark.device)

    def make(r0, n, bufs):
        bufs["features"][:n].copy_(base[r0:r0 + n])
    df = device_chunks(spark, rows, chunk, make, {"features": ((6,), torch.float32)})
    out = []
    model.transform(df).foreachBatch(lambda b: out.append(b.columns["prediction"].values.clone()))
    ref = model.transform(spark.createDataFrameFromLocalTensors({"features": base})).toPandas()["prediction"]
    np.testing.assert_allclose(torch.cat(out).cpu().numpy(), ref.to_numpy(), rtol=0, atol=0)


def test_predictor_cached_per_model(spark):
    from cdnaml.models.inference import predictor_for
    model = _model(spark)
    p1 = predictor_for(model, "value", [0.0])
    p2 = predictor_for(model, "value", [0.0])
    assert p1 is p2


@pytest.mark.gpu
def test_graph_replayed_predict_matches_direct(gpu_device):
    """Recurring staging buffers: captured once, then replayed; every replay equals a direct predict."""
    import cdnaml
    from cdnaml.models.inference import ForestPredictor
    spark = cdnaml.SparkSession.builder.getOrCreate()
    model = _model(spark, d=20, n=20000)
    pr = ForestPredictor(model._forest, model._tree_w, [0.0])
    buf = torch.empty((50000, 20), device=gpu_device)
    for i in range(4):
        buf.copy_(torch.randn(50000, 20, device=gpu_device))
        got = pr(buf)
        ref = pr._launch(buf)
        assert torch.equal(got, ref)
    assert pr.captures == 1 and pr.replays == 3
