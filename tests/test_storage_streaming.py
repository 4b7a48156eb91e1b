"""Versioned tables, catalog, streaming and the Python batch bridge
(ML00c, E00, ML12, ML13)."""
import json
import os
import time
from typing import Iterator

import numpy as np
import pandas as pd
import pytest

from cdnaml.sql import functions as F
from cdnaml.sql import types as T
from cdnaml.storage.delta import DeltaTable


def _listings(spark, n=200, seed=0):
    rng = np.random.default_rng(seed)
    return spark.createDataFrame(pd.DataFrame({
        "neighbourhood_cleansed": rng.choice(["Bayview", "Mission", "SoMa"], n),
        "price": rng.uniform(50, 500, n), "bedrooms": rng.integers(0, 4, n).astype(float)}))


def test_delta_versions_time_travel_history(spark, tmp_path):
    path = str(tmp_path / "delta")
    df = _listings(spark)
    df.write.format("delta").mode("overwrite").save(path)
    log = sorted(os.listdir(os.path.join(path, "_delta_log")))
    assert log[0] == "00000000000000000000.json"
    actions = [json.loads(line) for line in open(os.path.join(path, "_delta_log", log[0]))]
    kinds = {k for a in actions for k in a}
    assert {"add", "commitInfo", "metaData", "protocol"} <= kinds
    # version 1 overwrites with a filtered table
    df.filter(F.col("price") > 200).write.format("delta").mode("overwrite").save(path)
    assert spark.read.format("delta").load(path).count() < 200
    v0 = spark.read.format("delta").option("versionAsOf", 0).load(path)
    assert v0.count() == 200
    hist = DeltaTable.forPath(spark, path).history().toPandas()
    assert sorted(hist.version.tolist()) == [0, 1]
    h2 = spark.sql(f"DESCRIBE HISTORY delta.`{path}`").toPandas()
    assert len(h2) == 2
    ts = DeltaTable.forPath(spark, path).history().orderBy("version").toPandas().timestamp.iloc[0]
    assert spark.read.format("delta").option("timestampAsOf", str(ts)).load(path).count() == 200


def test_delta_schema_evolution(spark, tmp_path):
    path = str(tmp_path / "d2")
    df = _listings(spark)
    df.write.format("delta").save(path)
    wider = df.withColumn("extra", F.lit(1.0))
    with pytest.raises(Exception):
        wider.write.format("delta").mode("append").save(path)
    wider.write.format("delta").mode("append").option("mergeSchema", "true").save(path)
    out = spark.read.format("delta").load(path)
    assert "extra" in out.columns and out.count() == 400
    assert out.filter(F.col("extra").isNull()).count() == 200
    df.select("price").write.format("delta").mode("overwrite").option("overwriteSchema", "true").save(path)
    assert spark.read.format("delta").load(path).columns == ["price"]


def test_delta_partition_by_and_vacuum_guard(spark, tmp_path):
    path = str(tmp_path / "d3")
    df = _listings(spark)
    df.write.format("delta").mode("overwrite").partitionBy("neighbourhood_cleansed").save(path)
    assert os.path.isdir(os.path.join(path, "neighbourhood_cleansed=Bayview"))
    back = spark.read.format("delta").load(path)
    assert back.count() == 200 and "neighbourhood_cleansed" in back.columns
    df.limit(10).write.format("delta").mode("overwrite").save(path)
    dt = DeltaTable.forPath(spark, path)
    with pytest.raises(Exception):
        dt.vacuum(0)
    spark.conf.set("spark.databricks.delta.retentionDurationCheck.enabled", "false")
    dt.vacuum(0)
    assert spark.read.format("delta").load(path).count() == 10
    with pytest.raises(Exception):
        spark.read.format("delta").option("versionAsOf", 0).load(path).count()


def test_catalog_database_tables(spark):
    spark.sql("CREATE DATABASE IF NOT EXISTS course_db")
    spark.sql("USE course_db")
    _listings(spark).write.format("delta").mode("overwrite").saveAsTable("listings")
    assert spark.table("listings").count() == 200
    assert spark.sql("SELECT COUNT(*) AS c FROM listings").first().c == 200
    spark.sql("DROP TABLE IF EXISTS listings")
    with pytest.raises(Exception):
        spark.table("listings").count()
    spark.sql("DROP DATABASE IF EXISTS course_db CASCADE")


def test_json_reader_on_commit_log(spark, tmp_path):
    path = str(tmp_path / "d4")
    _listings(spark).write.format("delta").save(path)
    j = spark.read.json(os.path.join(path, "_delta_log", "00000000000000000000.json"))
    assert "commitInfo" in j.columns or "add" in j.columns


def test_streaming_memory_sink_with_checkpoint(spark, tmp_path):
    src = tmp_path / "src"
    src.mkdir()
    rng = np.random.default_rng(0)
    for i in range(4):
        pd.DataFrame({"x": rng.normal(size=25), "i": np.full(25, i)}).to_parquet(src / f"part-{i:05d}.parquet")
    schema = spark.read.parquet(str(src)).schema
    stream = spark.readStream.schema(schema).option("maxFilesPerTrigger", 1).parquet(str(src))
    q = (stream.withColumn("y", F.col("x") * 2).writeStream.format("memory")
         .option("checkpointLocation", str(tmp_path / "ckpt")).outputMode("append").queryName("pred_stream").start())
    q.processAllAvailable()
    assert spark.sql("SELECT COUNT(*) AS c FROM pred_stream").first().c == 100
    assert q.isActive and len(q.recentProgress) >= 4
    assert q in spark.streams.active
    q.stop()
    assert not q.isActive
    with pytest.raises(Exception):
        spark.readStream.parquet(str(src))  # a schema is required (MLE 00:48)


def test_pandas_udfs_and_map_in_pandas(spark):
    from cdnaml.sql.functions import pandas_udf

    df = spark.createDataFrame(pd.DataFrame({"a": np.arange(20.0), "b": np.ones(20)}))

    @pandas_udf("double")
    def add(a: pd.Series, b: pd.Series) -> pd.Series:
        return a + b

    out = df.withColumn("s", add("a", "b")).toPandas()
    np.testing.assert_array_equal(out.s.values, np.arange(20.0) + 1)

    @pandas_udf("double")
    def it(batches: Iterator[pd.DataFrame]) -> Iterator[pd.Series]:
        for feats in batches:
            yield pd.concat(feats, axis=1).sum(axis=1) if isinstance(feats, tuple) else feats.sum(axis=1)

    out2 = df.withColumn("t", it("a", "b")).toPandas()
    np.testing.assert_array_equal(out2.t.values, np.arange(20.0) + 1)

    def fn(it_):
        for pdf in it_:
            pdf["prediction"] = pdf.a * 10
            yield pdf

    schema = df.withColumn("prediction", F.lit(None).cast(T.DoubleType())).schema
    m = df.mapInPandas(fn, schema=schema).toPandas()
    np.testing.assert_array_equal(m.prediction.values, np.arange(20.0) * 10)
    m2 = df.mapInPandas(fn, schema="a double, b double, prediction double").toPandas()
    assert m2.shape == (20, 3)


def test_apply_in_pandas_groups(spark):
    """ML 13: one model per device_id group."""
    rng = np.random.default_rng(0)
    n = 1000
    pdf = pd.DataFrame({"device_id": np.arange(n) % 10, "f": rng.uniform(size=n)})
    pdf["label"] = pdf.f * (pdf.device_id + 1)
    df = spark.createDataFrame(pdf)
    out_schema = T.StructType([T.StructField("device_id", T.IntegerType()), T.StructField("n_used", T.IntegerType()),
                               T.StructField("slope", T.FloatType())])

    def train(g: pd.DataFrame) -> pd.DataFrame:
        slope = float(np.polyfit(g.f, g.label, 1)[0])
        return pd.DataFrame([[int(g.device_id.iloc[0]), len(g), slope]], columns=["device_id", "n_used", "slope"])

    res = df.groupby("device_id").applyInPandas(train, schema=out_schema).orderBy("device_id").toPandas()
    assert res.device_id.tolist() == list(range(10))
    np.testing.assert_allclose(res.slope.values, np.arange(1, 11), rtol=1e-5)
    joined = df.join(spark.createDataFrame(res), on="device_id")
    assert joined.count() == n


def test_arrow_batch_size_conf(spark):
    spark.conf.set("spark.sql.execution.arrow.maxRecordsPerBatch", 7)
    from cdnaml.sql.functions import pandas_udf
    sizes = []

    @pandas_udf("double")
    def probe(a: pd.Series) -> pd.Series:
        sizes.append(len(a))
        return a

    spark.range(0, 30).coalesce(1).withColumn("p", probe(F.col("id").cast("double"))).count()
    assert max(sizes) <= 7
