"""DataFrame / SQL engine."""
import numpy as np
import pandas as pd
import pytest

from cdnaml.sql import functions as F
from cdnaml.sql import types as T


def test_range_rand_lazy_count(spark):
    # ML 00b:35-37
    df = spark.range(1, 1000000).select((F.col("id") / 1000).cast("int").alias("id"), F.rand(seed=1).alias("v"))
    assert df.count() == 999999
    pdf = df.limit(5).toPandas()
    assert list(pdf.columns) == ["id", "v"]
    assert ((pdf.v >= 0) & (pdf.v < 1)).all()
    # rand(seed) is a pure function of (seed, row id)
    again = spark.range(1, 1000000).select(F.rand(seed=1).alias("v")).limit(5).toPandas()
    np.testing.assert_array_equal(pdf.v.values, again.v.values)


def test_create_from_pandas_and_tuples(spark):
    pdf = pd.DataFrame({"a": [1, 2, 3], "b": [0.5, 1.5, None], "s": ["x", "y", "x"]})
    df = spark.createDataFrame(pdf)
    assert df.count() == 3
    assert dict(df.dtypes)["s"] == "string"
    out = df.toPandas()
    assert out.s.tolist() == ["x", "y", "x"]
    assert np.isnan(out.b.iloc[2])
    df2 = spark.createDataFrame([(1, "a"), (2, "b")], ["k", "v"])
    assert [r.v for r in df2.collect()] == ["a", "b"]


def test_select_withcolumn_filter_drop(spark):
    df = spark.createDataFrame(pd.DataFrame({"price": ["$1,200.00", "$85.00", "$10,000.00"], "n": [1, 2, 3]}))
    df = df.withColumn("price", F.translate(F.col("price"), "$,", "").cast("double"))
    assert df.toPandas().price.tolist() == [1200.0, 85.0, 10000.0]
    f = df.filter(F.col("price") > 100).drop("n")
    assert f.columns == ["price"]
    assert f.count() == 2
    r = df.withColumnRenamed("n", "m").select("m", (F.col("m") * 2 + 1).alias("z")).collect()
    assert [x.z for x in r] == [3, 5, 7]


def test_when_otherwise_isnull_isin(spark):
    df = spark.createDataFrame(pd.DataFrame({"x": [1.0, None, 3.0, 4.0]}))
    out = df.select(F.when(F.col("x").isNull(), 1.0).otherwise(0.0).alias("na"),
                    F.col("x").isin(3.0, 4.0).alias("in")).toPandas()
    assert out.na.tolist() == [0.0, 1.0, 0.0, 0.0]
    assert out["in"].tolist() == [False, None, True, True]  # SQL three-valued logic


def test_groupby_count_orderby(spark):
    pdf = pd.DataFrame({"k": list("aabbbc"), "v": [1.0, 2.0, 3.0, 4.0, 5.0, 6.0]})
    df = spark.createDataFrame(pdf)
    out = df.groupBy("k").count().orderBy(F.col("count").desc(), "k").toPandas()
    assert out.k.tolist() == ["b", "a", "c"]
    assert out["count"].tolist() == [3, 2, 1]
    agg = df.groupBy("k").agg(F.avg("v").alias("m"), F.max("v").alias("mx")).orderBy("k").toPandas()
    np.testing.assert_allclose(agg.m.values, [1.5, 4.0, 6.0])
    np.testing.assert_allclose(agg.mx.values, [2.0, 5.0, 6.0])


def test_join_union_dedup(spark):
    a = spark.createDataFrame(pd.DataFrame({"id": [1, 2, 3], "x": [10.0, 20.0, 30.0]}))
    b = spark.createDataFrame(pd.DataFrame({"id": [2, 3, 4], "y": ["b", "c", "d"]}))
    inner = a.join(b, on="id").orderBy("id").toPandas()
    assert inner.id.tolist() == [2, 3]
    left = a.join(b, on="id", how="left").orderBy("id").toPandas()
    assert left.id.tolist() == [1, 2, 3]
    assert left.y.isna().tolist() == [True, False, False]
    u = a.union(a)
    assert u.count() == 6
    assert u.dropDuplicates().count() == 3
    assert u.dropDuplicates(["id"]).count() == 3


def test_describe_summary_quantile(spark):
    rng = np.random.default_rng(0)
    x = rng.normal(size=10001)
    df = spark.createDataFrame(pd.DataFrame({"x": x}))
    d = df.describe().toPandas().set_index("summary")
    assert float(d.loc["count", "x"]) == 10001
    assert abs(float(d.loc["mean", "x"]) - x.mean()) < 1e-9
    assert abs(float(d.loc["stddev", "x"]) - x.std(ddof=1)) < 1e-9
    s = df.summary().toPandas().set_index("summary")
    assert "50%" in s.index
    med = df.approxQuantile("x", [0.5], 0.01)[0]
    assert abs(med - np.median(x)) < 0.05


def test_random_split_partition_invariant(spark):
    df = spark.range(0, 100000)
    a, b = df.randomSplit([0.8, 0.2], seed=42)
    n_a = a.count()
    assert a.count() + b.count() == 100000
    assert 78000 < n_a < 82000
    # Philox(seed, global row id): same split whatever the partition count
    a2, _ = spark.range(0, 100000, numPartitions=7).randomSplit([0.8, 0.2], seed=42)
    assert set(a2.toPandas().id) == set(a.toPandas().id)
    # a shuffling repartition reorders rows and so changes the split, as in Spark (ML 02:43-52)
    a3, _ = df.repartition(24).randomSplit([0.8, 0.2], seed=42)
    assert a3.count() + _.count() == 100000


def test_cache_repartition_partitions(spark):
    df = spark.range(0, 1000).repartition(24)
    assert df.rdd.getNumPartitions() == 24
    c = df.coalesce(1)
    assert c.rdd.getNumPartitions() == 1
    cached = df.cache()
    assert cached.count() == 1000
    assert cached.count() == 1000


def test_sql_temp_view(spark):
    pdf = pd.DataFrame({"k": list("aabbbc"), "v": [1.0, 2.0, 3.0, 4.0, 5.0, 6.0]})
    spark.createDataFrame(pdf).createOrReplaceTempView("t")
    out = spark.sql("SELECT k, COUNT(*) AS c, AVG(v) AS m FROM t GROUP BY k HAVING COUNT(*) > 1 ORDER BY c DESC")
    p = out.toPandas()
    assert p.k.tolist() == ["b", "a"]
    assert p.c.tolist() == [3, 2]
    assert spark.sql("SELECT * FROM t LIMIT 2").count() == 2


def test_sql_join(spark):
    spark.createDataFrame(pd.DataFrame({"id": [1, 2], "t": ["x", "y"]})).createOrReplaceTempView("m")
    spark.createDataFrame(pd.DataFrame({"id": [1, 1, 2], "r": [3.0, 4.0, 5.0]})).createOrReplaceTempView("r")
    p = spark.sql("SELECT m.t, AVG(r.r) AS a FROM r JOIN m ON r.id = m.id GROUP BY m.t ORDER BY a DESC").toPandas()
    assert p.t.tolist() == ["y", "x"]
    np.testing.assert_allclose(p.a.values, [5.0, 3.5])


def test_schema_ddl_and_types(spark):
    s = T._parse_datatype_string("a INT, b DOUBLE, c STRING")
    assert [f.name for f in s.fields] == ["a", "b", "c"]
    assert s["a"].dataType == T.IntegerType()
    df = spark.createDataFrame([(1, 2.0, "x")], s)
    assert df.schema["b"].dataType == T.DoubleType()
    assert T.StructType.fromJson(df.schema.jsonValue()) == df.schema


def test_monotonic_id_and_hash(spark):
    df = spark.range(0, 10).coalesce(1).withColumn("mid", F.monotonically_increasing_id())
    assert df.toPandas().mid.tolist() == list(range(10))
    h = spark.createDataFrame(pd.DataFrame({"s": ["a", "b", "a"]})).select(F.abs(F.hash("s")).alias("h")).toPandas()
    assert h.h.iloc[0] == h.h.iloc[2] and h.h.iloc[0] != h.h.iloc[1]


def test_string_functions_and_log_exp(spark):
    df = spark.createDataFrame(pd.DataFrame({"s": ["Ab", "aB", "c"], "x": [1.0, 2.0, 4.0]}))
    p = df.select(F.lower("s").alias("l"), F.log("x").alias("lg"), F.exp(F.log("x")).alias("e")).toPandas()
    assert p.l.tolist() == ["ab", "ab", "c"]
    np.testing.assert_allclose(p.lg.values, np.log([1, 2, 4]))
    np.testing.assert_allclose(p.e.values, [1, 2, 4])


def test_dedup_lab_semantics(spark, tmp_path):
    """Labs/ML 00L: case / SSN-format-insensitive dedup, 8 parquet part files."""
    rng = np.random.default_rng(1)
    n = 1000
    first = [f"Name{i}" for i in range(n)]
    ssn = [f"{rng.integers(100, 999)}-{rng.integers(10, 99)}-{rng.integers(1000, 9999)}{i}" for i in range(n)]
    dup = rng.choice(n, 30, replace=False)
    rows = [(first[i], ssn[i]) for i in range(n)] + [(first[i].upper(), ssn[i].replace("-", "")) for i in dup]
    df = spark.createDataFrame(rows, ["firstName", "ssn"])
    spark.conf.set("spark.sql.shuffle.partitions", 8)
    dd = (df.withColumn("lf", F.lower("firstName")).withColumn("s2", F.translate("ssn", "-", ""))
          .dropDuplicates(["lf", "s2"]).drop("lf", "s2"))
    assert dd.count() == n
    out = tmp_path / "dedup"
    dd.write.mode("overwrite").parquet(str(out))
    parts = [p for p in out.iterdir() if p.name.endswith(".parquet")]
    assert len(parts) == 8
    assert spark.read.parquet(str(out)).count() == n


def test_csv_roundtrip(spark, tmp_path):
    p = tmp_path / "x.csv"
    p.write_text('a,b,price\n1,"hello, world","$1,000"\n2,bye,$5\n')
    df = spark.read.csv(str(p), header=True, inferSchema=True, multiLine=True, escape='"')
    pdf = df.toPandas()
    assert pdf.b.tolist() == ["hello, world", "bye"]
    assert dict(df.dtypes)["a"] in ("int", "bigint")
    q = tmp_path / "people.txt"
    q.write_text("first:last\nA:B\nC:D\n")
    assert spark.read.csv(str(q), header=True, sep=":").count() == 2


def test_sample_and_first(spark):
    df = spark.range(0, 100000)
    s = df.sample(fraction=0.01, seed=3).count()
    assert 700 < s < 1300
    assert df.first().id == 0


def test_to_pandas_vector_column(spark):
    from cdnaml.ml.feature import VectorAssembler

    df = spark.createDataFrame(pd.DataFrame({"a": [1.0, 2.0], "b": [3.0, 4.0]}))
    v = VectorAssembler(inputCols=["a", "b"], outputCol="f").transform(df)
    rows = v.collect()
    assert rows[1].f.toArray().tolist() == [2.0, 4.0]


def _mle01_tables(spark, seed=0):
    rng = np.random.default_rng(seed)
    n_movies, n_users = 400, 300
    movies = pd.DataFrame({"ID": np.arange(n_movies), "title": [f"movie {i}" for i in range(n_movies)]})
    # popular movies get many ratings, so both HAVING thresholds select a proper subset
    mid = np.minimum(rng.zipf(1.3, 60000) - 1, n_movies - 1)
    ratings = pd.DataFrame({"userId": rng.integers(1, n_users, 60000), "movieId": mid,
                            "rating": rng.integers(1, 6, 60000).astype(np.float64)})
    pred = movies.rename(columns={"ID": "movieId"}).assign(userId=0)
    pred["prediction"] = np.round(rng.random(n_movies) * 5, 3)
    return movies, ratings, pred


def test_sql_join_aliases_mle01_verbatim(spark):
    """Both MLE 01 queries verbatim (S/ML Electives/MLE 01 - Collaborative Filtering Lab.py:246-252,366-374)
    on tables that share userId / movieId / rating, checked against pandas."""
    movies, ratings, pred = _mle01_tables(spark)
    spark.createDataFrame(movies).createOrReplaceTempView("movies")
    spark.createDataFrame(ratings).createOrReplaceTempView("ratings")
    spark.createDataFrame(pred).createOrReplaceTempView("predictions")
    q1 = spark.sql("""
        SELECT movieId, title, AVG(rating) AS avg_rating, COUNT(*) AS num_ratings
        FROM ratings r JOIN movies m ON (r.movieID = m.ID)
        GROUP BY r.movieId, m.title
        HAVING COUNT(*) > 500
        ORDER BY avg_rating DESC
        LIMIT 100""").toPandas()
    m = ratings.merge(movies, left_on="movieId", right_on="ID")
    e1 = (m.groupby(["movieId", "title"]).agg(avg_rating=("rating", "mean"), num_ratings=("rating", "size"))
          .reset_index())
    e1 = e1[e1.num_ratings > 500].sort_values("avg_rating", ascending=False).head(100)
    assert list(q1.columns) == ["movieId", "title", "avg_rating", "num_ratings"]
    assert 0 < len(q1) == len(e1)
    np.testing.assert_allclose(q1.avg_rating.values, e1.avg_rating.values)
    assert sorted(q1.movieId.tolist()) == sorted(e1.movieId.tolist())

    q2 = spark.sql("""
        SELECT p.title, p.prediction AS your_predicted_rating
        FROM ratings r INNER JOIN predictions p
        ON (r.movieID = p.movieID)
        WHERE p.userId = 0
        GROUP BY p.title, p.prediction
        HAVING COUNT(*) > 75
        ORDER BY p.prediction DESC
        LIMIT 25""").toPandas()
    j = ratings.merge(pred, on="movieId", suffixes=("_r", "_p"))
    j = j[j.userId_p == 0]
    e2 = j.groupby(["title", "prediction"]).size().reset_index(name="n")
    e2 = e2[e2.n > 75].sort_values("prediction", ascending=False).head(25)
    assert list(q2.columns) == ["title", "your_predicted_rating"]
    assert 0 < len(q2) == len(e2)
    np.testing.assert_allclose(q2.your_predicted_rating.values, e2.prediction.values)


def test_sql_qualified_and_ambiguous_names(spark):
    from cdnaml.sql.column import AnalysisException
    spark.createDataFrame(pd.DataFrame({"k": [1, 2, 3], "v": [10.0, 20.0, 30.0]})).createOrReplaceTempView("ta")
    spark.createDataFrame(pd.DataFrame({"k": [1, 2, 4], "v": [-1.0, -2.0, -4.0]})).createOrReplaceTempView("tb")
    out = spark.sql("SELECT b.v FROM ta a JOIN tb b ON (a.k = b.k) ORDER BY b.v").toPandas()
    assert out.v.tolist() == [-2.0, -1.0]
    out = spark.sql("SELECT a.v AS av, b.v AS bv FROM ta a JOIN tb b ON a.k = b.k ORDER BY a.k").toPandas()
    assert out.av.tolist() == [10.0, 20.0] and out.bv.tolist() == [-1.0, -2.0]
    # the table name qualifies when there is no alias
    out = spark.sql("SELECT tb.v FROM ta JOIN tb ON ta.k = tb.k WHERE ta.v > 15").toPandas()
    assert out.v.tolist() == [-2.0]
    with pytest.raises(AnalysisException, match="ambiguous"):
        spark.sql("SELECT v FROM ta a JOIN tb b ON (a.k = b.k)").toPandas()
    # USING merges the key: a bare key is not ambiguous, and both qualifiers reach it
    out = spark.sql("SELECT k, a.k AS ak, b.v FROM ta a JOIN tb b USING (k) ORDER BY k").toPandas()
    assert out.k.tolist() == [1, 2] and out.ak.tolist() == [1, 2] and out.v.tolist() == [-1.0, -2.0]
    out = spark.sql("SELECT a.*, b.v AS w FROM ta a LEFT JOIN tb b ON a.k = b.k ORDER BY a.k").toPandas()
    assert list(out.columns) == ["k", "v", "w"]
    assert out.w.isna().tolist() == [False, False, True]
    # a known qualifier whose source lacks the column does not fall back to the other side
    spark.createDataFrame(pd.DataFrame({"k": [1, 2], "x": [5.0, 6.0]})).createOrReplaceTempView("tc")
    with pytest.raises(AnalysisException, match="cannot resolve"):
        spark.sql("SELECT a.x FROM ta a JOIN tc c ON a.k = c.k").toPandas()
    assert spark.sql("SELECT c.x FROM ta a JOIN tc c ON a.k = c.k ORDER BY c.x").toPandas().x.tolist() == [5.0, 6.0]
