"""Parity flows for the data notebooks: ML 00b Spark Review, ML 00c Delta Review, ML 01 Data Cleansing,
Labs/ML 00L Dedup, Labs/ML 01L Data Exploration."""
import os

import pytest

from cdnaml.utils.dbutils import dbutils


def _sf(ds, name):
    return os.path.join(ds, "airbnb", "sf-listings", name)


def test_ml00b_spark_review(nb):
    """ML 00b:33-117 -- range + rand, lazy count, sample, temp view + SQL, partitions, cache, limit().toPandas()."""
    spark, _, _ = nb
    from pyspark.sql.functions import col, rand

    df = spark.range(1, 10001).withColumn("x", rand(seed=42)).withColumn("y", col("x") * 2)
    assert df.count() == 10000 and df.columns == ["id", "x", "y"]
    assert df.filter(col("x") > 2).count() == 0                       # rand in [0, 1)
    s = df.sample(fraction=0.1, seed=7)
    assert 700 < s.count() < 1300
    df.createOrReplaceTempView("ml00b")
    assert spark.sql("SELECT COUNT(*) AS c FROM ml00b WHERE id <= 10").first().c == 10
    assert df.rdd.getNumPartitions() >= 1
    df.cache()
    pdf = df.limit(5).toPandas()
    assert list(pdf.columns) == ["id", "x", "y"] and len(pdf) == 5
    assert (pdf.y == pdf.x * 2).all()


def test_ml00c_delta_review(nb):
    """ML 00c:46-254 -- parquet -> delta, partitionBy + overwriteSchema, versions, history, time travel,
    vacuum guard then vacuum(0)."""
    spark, ds, work = nb
    from delta.tables import DeltaTable

    df = spark.read.parquet(_sf(ds, "sf-listings-2019-03-06-clean.parquet"))
    path = os.path.join(work, "delta-ml00c")
    df.write.format("delta").mode("overwrite").save(path)
    v0 = spark.read.format("delta").load(path).count()
    (df.write.format("delta").mode("overwrite").option("overwriteSchema", "true")
       .partitionBy("neighbourhood_cleansed").save(path))
    df.filter(df.price > 100).write.format("delta").mode("overwrite").save(path)
    log = os.path.join(path, "_delta_log")
    assert path.startswith("dbfs:/")
    assert sorted(f.name for f in dbutils.fs.ls(log) if f.name.endswith(".json"))[0] == "00000000000000000000.json"
    assert spark.read.json(os.path.join(log, "00000000000000000000.json")).count() >= 1
    dt = DeltaTable.forPath(spark, path)
    hist = dt.history()
    assert hist.count() == 3
    assert spark.read.format("delta").option("versionAsOf", 0).load(path).count() == v0
    assert spark.read.format("delta").load(path).count() < v0
    with pytest.raises(Exception):
        dt.vacuum(0)                                                    # under the 7-day retention guard
    spark.conf.set("spark.databricks.delta.retentionDurationCheck.enabled", "false")
    dt.vacuum(0)
    assert spark.read.format("delta").load(path).count() < v0


def test_ml01_data_cleansing(nb):
    """ML 01:32-265 -- multiLine CSV, price '$'/',' strip + cast, describe/summary, filter, groupBy-count,
    int -> double, _na flags + Imputer(median)."""
    spark, ds, _ = nb
    from pyspark.sql.functions import col, translate, when
    from pyspark.ml.feature import Imputer

    raw = spark.read.csv(_sf(ds, "sf-listings-2019-03-06.csv"), header="true", inferSchema="true",
                         multiLine="true", escape='"')
    assert dict(raw.dtypes)["price"] == "string"
    base = raw.select("host_is_superhost", "neighbourhood_cleansed", "room_type", "accommodates", "bedrooms",
                      "beds", "minimum_nights", "review_scores_rating", "price")
    fixed = base.withColumn("price", translate(col("price"), "$,", "").cast("double"))
    assert dict(fixed.dtypes)["price"] == "double"
    summ = fixed.select("price").summary().toPandas()
    assert {"count", "mean", "min", "max", "50%"} <= set(summ["summary"])
    pos = fixed.filter(col("price") > 0)
    counts = pos.groupBy("room_type").count().orderBy(col("count").desc()).toPandas()
    assert counts["count"].is_monotonic_decreasing
    nums = [c for c, t in pos.dtypes if t in ("int", "bigint", "double") and c != "price"]
    for c in nums:
        pos = pos.withColumn(c, col(c).cast("double"))
    for c in nums:
        pos = pos.withColumn(c + "_na", when(col(c).isNull(), 1.0).otherwise(0.0))
    imputed = Imputer(strategy="median", inputCols=nums, outputCols=nums).fit(pos).transform(pos)
    assert all(imputed.filter(col(c).isNull()).count() == 0 for c in nums)


def test_l00_dedup_lab(nb):
    """Labs/ML 00L:66-147 -- ':'-CSV, shuffle.partitions = 8, case- and SSN-format-insensitive
    dropDuplicates, 8 parquet part files, 100,000 rows, checked with the lab's own answer hashes."""
    spark, ds, work = nb
    from pyspark.sql.functions import col, lower, translate
    from cdnaml.utils import Classroom

    from cdnaml.utils import datasets as D

    # full-size people file (the installed datasets are scaled down): 100,000 people + 3,000 re-cased duplicates
    src = f"{work}/people-with-dups.txt"
    dbutils.fs.mkdirs(work)
    D.people_with_dups(n_unique=100000, n_dups=3000).to_csv(src.replace("dbfs:/", "/dbfs/"), sep=":", index=False)
    spark.conf.set("spark.sql.shuffle.partitions", 8)
    df = spark.read.csv(src, header=True, sep=":", inferSchema=True)
    assert df.count() == 103000
    dedup = (df.select(col("*"), lower(col("firstName")).alias("lcFirstName"),
                       lower(col("lastName")).alias("lcLastName"), lower(col("middleName")).alias("lcMiddleName"),
                       translate(col("ssn"), "-", "").alias("ssnNums"))
             .dropDuplicates(["lcFirstName", "lcMiddleName", "lcLastName", "ssnNums", "gender", "birthDate",
                              "salary"])
             .drop("lcFirstName", "lcMiddleName", "lcLastName", "ssnNums"))
    dest = os.path.join(work, "people.parquet")
    dedup.write.mode("overwrite").parquet(dest)
    parts = len([f for f in dbutils.fs.ls(dest) if f.name.endswith(".parquet")])  # L00:139
    final = spark.read.parquet(dest).count()
    cr = Classroom(spark, lesson="ML 00L", install=False)
    assert cr.validateYourAnswer("01 Parquet File Exists", 1276280174, parts)
    assert cr.validateYourAnswer("02 Expected 100000 Records", 972882115, final)


def test_l01_data_exploration(nb):
    """Labs/ML 01L:33-185 -- log(price), ordered group counts, avg / approxQuantile median baselines, RMSE."""
    spark, ds, _ = nb
    from pyspark.sql.functions import avg, col, lit, log
    from pyspark.ml.evaluation import RegressionEvaluator

    df = spark.read.format("delta").load(_sf(ds, "sf-listings-2019-03-06-clean.delta"))
    lp = df.select(log("price").alias("log_price"))
    assert lp.filter(col("log_price").isNull()).count() == 0
    top = df.groupBy("neighbourhood_cleansed").count().orderBy(col("count").desc()).limit(5).toPandas()
    assert top["count"].is_monotonic_decreasing
    train, test = df.randomSplit([0.8, 0.2], seed=42)
    mean_price = train.select(avg("price")).first()[0]
    median_price = train.approxQuantile("price", [0.5], 0.0)[0]
    ev = RegressionEvaluator(predictionCol="pred", labelCol="price", metricName="rmse")
    rmse_mean = ev.evaluate(test.withColumn("pred", lit(mean_price)))
    rmse_median = ev.evaluate(test.withColumn("pred", lit(median_price)))
    assert rmse_mean > 0 and rmse_median >= rmse_mean * 0.9    # the mean minimises squared error in-sample
